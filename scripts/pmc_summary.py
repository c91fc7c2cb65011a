"""Summarise rocprofv3 --pmc CSVs for one kernel (average per frame
dispatch; the tile-cost estimate launch is left out, see pmc_common.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_common import frame_counters  # noqa: E402

pat = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "rt_render"
agg = frame_counters(pat, kname)
for k in sorted(agg):
    v = agg[k]
    print("%-28s n=%d avg=%.4g" % (k, len(v), sum(v) / len(v)))
a = {k: sum(v) / len(v) for k, v in agg.items()}
if "SQ_THREAD_CYCLES_VALU" in a and "SQ_ACTIVE_INST_VALU" in a:
    print("lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*64)) = %.3f" % (a["SQ_THREAD_CYCLES_VALU"] / (a["SQ_ACTIVE_INST_VALU"] * 64)))
if "SQ_WAVE_CYCLES" in a and "SQ_WAIT_ANY" in a:
    print("wait_any / wave_cycles = %.3f ; wait_inst_any / wave_cycles = %.3f" % (a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"]))
