"""Executed-work roofline fields of the render kernel from rocprofv3 --pmc passes.

bench.py's `roofline.frac` prices the REFERENCE's algorithmic FP64 work (SURVEY
§8(d): Intersect calls x per-kind flops + shading), which the culled kernel
does not all execute. This script turns the counter passes of the same kernel
build into what the kernel actually executes, per launch (average dispatch):

  executed_fp64_flops = (ADD_F64 + MUL_F64 + TRANS_F64 + 2 * FMA_F64) wave-instructions
                        x 64 lanes x lane utilisation
      lane utilisation  = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)
                          (all VALU instructions; the FP64 ones are assumed alike)
  kernel_cycles       = GRBM_GUI_ACTIVE / XCDs  (the counter sums the 8 XCDs)
  simd_cycles         = SIMDs (256 CU x 4) x kernel_cycles
  fp64_pipe_busy      = FP64 wave-instructions x 4 cycles / simd_cycles
                        (a wave64 FP64 op occupies a SIMD16 for 4 cycles)
  valu_busy           = SQ_ACTIVE_INST_VALU x 4 / simd_cycles
                        (SQ_ACTIVE_INST_VALU counts in 4-cycle units, like SQ_WAVE_CYCLES)
  issue_util          = 4 x (SQ_INSTS_VALU + SQ_INSTS_SALU) / simd_cycles
                        (one VALU or SALU issue per wave per 4 cycles: the share of
                        each SIMD's issue cycles the instruction stream takes --
                        the bound the C3 kernel sits at)

bench.py divides executed_fp64_flops by its own live kernel time (HIP events)
to report `roofline.executed_frac` next to the algorithmic `frac`.

usage: python scripts/pmc_roofline.py 'gpurun_out/pmc_c3/p[12]/*counter_collection.csv' \
           profiles/pmc_c3.json [kernel-name-substring]
"""
import collections
import csv
import glob
import json
import os
import sys

CUS, SIMDS_PER_CU, XCDS = 256, 4, 8


def main():
    pat, out = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from __graft_entry__ import load_package
    kernel_src = load_package().render.kernel_source_id()  # the device code these counters come from
    kname = sys.argv[3] if len(sys.argv) > 3 else "rt_render"
    files = sorted(glob.glob(pat))
    from pmc_common import frame_counters, kept_dispatches
    agg = frame_counters(pat, kname)  # frame launches only (no estimate / companion)
    kept, dropped = kept_dispatches(pat, kname)
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    need = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
            "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"]
    missing = [k for k in need if k not in a]
    if missing:
        raise SystemExit("missing counters: %s" % ", ".join(missing))
    f64_insts = a["SQ_INSTS_VALU_ADD_F64"] + a["SQ_INSTS_VALU_MUL_F64"] + a["SQ_INSTS_VALU_TRANS_F64"] + \
        a["SQ_INSTS_VALU_FMA_F64"]
    f64_ops = f64_insts + a["SQ_INSTS_VALU_FMA_F64"]  # an FMA is two flops
    lane_util = a["SQ_THREAD_CYCLES_VALU"] / (a["SQ_ACTIVE_INST_VALU"] * 64.0)
    kcyc = a["GRBM_GUI_ACTIVE"] / XCDS
    simd_cyc = CUS * SIMDS_PER_CU * kcyc
    res = {
        "kernel": kname,
        "counters": {k: a[k] for k in sorted(a)},
        "dispatches": {k: len(v) for k, v in sorted(agg.items())},
        "executed_fp64_flops": f64_ops * 64.0 * lane_util,
        "fp64_wave_insts": f64_insts,
        "lane_util": lane_util,
        "kernel_cycles": kcyc,
        "fp64_pipe_busy": f64_insts * 4.0 / simd_cyc,
        "valu_busy": a["SQ_ACTIVE_INST_VALU"] * 4.0 / simd_cyc,
        "issue_util": 4.0 * (a["SQ_INSTS_VALU"] + a["SQ_INSTS_SALU"]) / simd_cyc,
        "fp64_share_of_valu": f64_insts / a["SQ_INSTS_VALU"],
        "source": [os.path.relpath(f) for f in files],
        "kernel_src": kernel_src,
        "dispatches_dropped": dropped,
        "note": "per-launch averages; see scripts/pmc_roofline.py for the definitions",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("executed_fp64_flops", "lane_util", "fp64_pipe_busy", "valu_busy",
                                          "issue_util", "fp64_share_of_valu")}))


if __name__ == "__main__":
    main()
