"""The executed-work roofline fields bench.py reports come from committed
rocprofv3 PMC summaries (profiles/pmc_<config>.json, scripts/pmc_roofline.py).
Recompute them from the committed raw counter CSVs and check the summaries
(and the bench's reader) against that -- the numbers are reproducible from the
files, as DESIGN.md §4 says."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["pmc_c3", "pmc_c3cone", "pmc_c4", "pmc_c4csg", "pmc_c5", "pmc_c5_bf_rows2048-2304"])
def test_pmc_summary_recomputes_from_committed_csvs(tmp_path, name):
    ref = json.load(open(os.path.join(ROOT, "profiles", name + ".json")))
    srcs = [os.path.join(ROOT, f) for f in ref["source"]]
    assert srcs and all(os.path.exists(f) for f in srcs), ref["source"]
    pattern = os.path.join(os.path.dirname(srcs[0]), os.path.basename(srcs[0]).split("_p")[0] + "_p[12]_*.csv")
    assert sorted(glob.glob(pattern)) == sorted(srcs)
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_roofline.py"), pattern, str(out), "rt_render"],
                   check=True, capture_output=True, cwd=ROOT)
    got = json.load(open(out))
    for k in ("executed_fp64_flops", "lane_util", "fp64_pipe_busy", "valu_busy", "issue_util"):
        assert got[k] == pytest.approx(ref[k], rel=1e-12), k
    # the definitions: FP64 ops x 64 lanes x lane utilisation; 4-cycle wave64 FP64 ops over 1024 SIMDs
    c = got["counters"]
    f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_TRANS_F64"] + \
        2 * c["SQ_INSTS_VALU_FMA_F64"]
    assert got["executed_fp64_flops"] == pytest.approx(f64 * 64 * got["lane_util"], rel=1e-12)
    simd_cycles = 1024 * c["GRBM_GUI_ACTIVE"] / 8
    assert got["valu_busy"] == pytest.approx(c["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles, rel=1e-12)


def test_bench_reads_the_committed_summary():
    sys.path.insert(0, ROOT)
    import bench
    ex, src = bench.pmc_executed("c3")
    assert src == os.path.join("profiles", "pmc_c3.json")
    assert ex["executed_fp64_flops"] > 1e10 and 0 < ex["issue_util"] < 1.5
    assert bench.pmc_executed("no_such_config") == (None, None)


def test_committed_bench_line_keeps_the_contract():
    """The committed round bench line (profiles/r04/final/bench_c3.json) has the
    driver's fields, and its derived numbers agree with each other: value =
    rays per step / ms per step, frac = achieved / peak, and the GPU span per
    frame from the rocprofv3 kernel trace of the same command
    (scripts/trace_span.py; frames in flight overlap, so the span, not a
    dispatch's duration, is the kernel time) is within 5 % of the in-bench
    kernel time."""
    d = json.load(open(os.path.join(ROOT, "profiles", "r04", "final", "bench_c3.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["dtype"] == "f64" and d["n_gpus"] == 1 and d["higher_is_better"] is True
    assert "workload" in d["config"] and d["config"]["width"] == 3840 and d["config"]["height"] == 2160
    assert d["config"]["frames_in_flight"] >= 1
    assert d["value"] == pytest.approx(d["config"]["rays_per_step"] / d["ms_per_step"] / 1e3, rel=2e-3)
    r = d["roofline"]
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)
    assert r["achieved"] == pytest.approx(r["flops_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e12, rel=2e-3)
    assert r["kernel_ms"] <= d["ms_per_step"] * 1.001
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0
    t = json.load(open(os.path.join(ROOT, "profiles", "r04", "final", "trace_span_c3.json")))
    assert t["dispatches"] == 30
    prof = json.load(open(os.path.join(ROOT, "profiles", "r04", "final", "rocprof_bench.json")))
    assert t["span_ms_per_frame"] == pytest.approx(prof["roofline"]["kernel_ms"], rel=0.05)
    assert t["span_ms_per_frame"] == pytest.approx(r["kernel_ms"], rel=0.05)


def test_trace_span_matches_a_serial_trace():
    """Without overlap the span per frame is the average dispatch duration plus
    the gaps between launches (round-3 serial trace)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import trace_span
    t = trace_span.span(os.path.join(ROOT, "profiles", "r03", "final", "kernel_trace_c3.csv"), 30)
    assert t["overlap_fraction_of_span"] == 0.0
    assert t["avg_dispatch_ms"] <= t["span_ms_per_frame"] <= t["avg_dispatch_ms"] * 1.02
