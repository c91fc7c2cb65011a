// rt_spec_cc -- compiles ONE specialised variant of the render kernel with
// hipRTC, in a process of its own, for librtamd.so (rt_kernel.hip
// spec_compile). A compiler backend error ("illegal VGPR to SGPR copy" and
// the like) aborts the process it runs in; here that is this helper, not the
// caller's renderer, which then renders with the generic kernel. The helper
// also has its own environment, so the host's setenv / unsetenv during a
// compile cannot touch it.
//
//   rt_spec_cc OUT NAME_EXPR [compiler option ...]
// writes the code object to OUT and the kernel's lowered name to OUT.name;
// exit 0 on success, 1 with the compiler log on stderr otherwise. The device
// sources are the library's own (rt_jit_src.inc, embedded at build time).
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "rt_jit_src.inc"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s OUT NAME_EXPR [option ...]\n", argv[0]);
    return 2;
  }
  const std::string out = argv[1];
  const char* name = argv[2];
  // test hook (tests/test_specialize.py): die the way a compiler backend
  // assertion does, to show that only this process goes down
  if (getenv("RT_SPEC_CC_ABORT")) abort();
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, "#include \"rt_render.h\"\n", "rt_spec.hip", k_jit_nsrc, k_jit_srcs,
                                       k_jit_names);
  if (r != HIPRTC_SUCCESS) {
    fprintf(stderr, "hiprtcCreateProgram: %s\n", hiprtcGetErrorString(r));
    return 1;
  }
  r = hiprtcAddNameExpression(prog, name);
  if (r == HIPRTC_SUCCESS) r = hiprtcCompileProgram(prog, argc - 3, (const char**)(argv + 3));
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    std::string log;
    if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
      log.resize(n);
      (void)hiprtcGetProgramLog(prog, &log[0]);
    }
    fprintf(stderr, "hiprtcCompileProgram: %s\n%s\n", hiprtcGetErrorString(r), log.c_str());
    return 1;
  }
  const char* low = nullptr;
  size_t n = 0;
  if (hiprtcGetLoweredName(prog, name, &low) != HIPRTC_SUCCESS || !low) {
    fprintf(stderr, "hiprtcGetLoweredName failed\n");
    return 1;
  }
  if (hiprtcGetCodeSize(prog, &n) != HIPRTC_SUCCESS || n == 0) {
    fprintf(stderr, "hiprtcGetCodeSize failed\n");
    return 1;
  }
  std::vector<char> code(n);
  if (hiprtcGetCode(prog, code.data()) != HIPRTC_SUCCESS) {
    fprintf(stderr, "hiprtcGetCode failed\n");
    return 1;
  }
  FILE* f = fopen(out.c_str(), "wb");
  FILE* g = fopen((out + ".name").c_str(), "wb");
  const bool ok = f && g && fwrite(code.data(), 1, n, f) == n && fputs(low, g) >= 0;
  if (f) fclose(f);
  if (g) fclose(g);
  (void)hiprtcDestroyProgram(&prog);
  if (!ok) {
    fprintf(stderr, "cannot write %s\n", out.c_str());
    return 1;
  }
  return 0;
}
