"""Summarise rocprofv3 --pmc CSVs for one kernel (average per dispatch)."""
import collections
import csv
import glob
import sys

pat = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "rt_render"
agg = collections.defaultdict(list)
for f in glob.glob(pat):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print("%-28s n=%d avg=%.4g" % (k, len(v), sum(v) / len(v)))
a = {k: sum(v) / len(v) for k, v in agg.items()}
if "SQ_THREAD_CYCLES_VALU" in a and "SQ_ACTIVE_INST_VALU" in a:
    print("lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*64)) = %.3f" % (a["SQ_THREAD_CYCLES_VALU"] / (a["SQ_ACTIVE_INST_VALU"] * 64)))
if "SQ_WAVE_CYCLES" in a and "SQ_WAIT_ANY" in a:
    print("wait_any / wave_cycles = %.3f ; wait_inst_any / wave_cycles = %.3f" % (a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"]))
