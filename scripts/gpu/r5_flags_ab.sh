# Round 5: compiler-option A/B of the specialised kernels (hipRTC options via
# RT_SPEC_EXTRA_FLAGS; LLVM scheduler strategies, -O2), C3 bench line and
# c4csg whole frames, interleaved rounds. (-amdgpu-sched-strategy=iterative-ilp
# crashed the compiler inside hipRTC: segfault, not run again.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_flags_ab}
mkdir -p $O
b() {  # name flags config
  RT_SPEC_EXTRA_FLAGS="$2" timeout -k 10 300 python3 bench.py --config $3 --steps 20 --warmup 3 --cpu-baseline off --companion off > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('%-22s %.4f ms/step' % ('$1', d['ms_per_step']))"
}
for r in 1 2 3; do
  b c3_base$r "" c3 && b c3_o2$r "-O2" c3 && b c3_memclause$r "-mllvm -amdgpu-sched-strategy=max-memory-clause" c3 && \
  b c3_maxilp$r "-mllvm -amdgpu-sched-strategy=max-ilp" c3 && \
  b c3_nounclust$r "-mllvm -amdgpu-disable-unclustered-high-rp-reschedule" c3 && \
  b c3_trackers$r "-mllvm -amdgpu-use-amdgpu-trackers=1" c3 || exit 1
done
for r in 1 2; do
  b csg_base$r "" c4csg && b csg_o2$r "-O2" c4csg && b csg_memclause$r "-mllvm -amdgpu-sched-strategy=max-memory-clause" c4csg && \
  b csg_maxilp$r "-mllvm -amdgpu-sched-strategy=max-ilp" c4csg || exit 1
done
