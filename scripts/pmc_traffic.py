"""Per-launch HBM traffic of the render kernel from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters from the TCC
EA read/write requests, MI355X_MICROARCH.md §HBM; Infinity-Cache hits are
counted, not excluded). The guide calibrates only 16-B/lane streams, so the
counters are calibrated here on the render kernel's own widths with
build_variants/pmc_calib (scripts/pmc_calib.hip: 512 MiB each of 8-B/lane
loads, 8-B/lane stores, 4-B/lane stores): bytes = counter / (counter per byte
of the matching calibration kernel). Reads: 8-B frame fields (the scene and
the jump table are in LDS); writes: 8-B frame fields and 4-B pixels (the
8-B/lane factor is applied to all writes; the 4-B factor is reported).

usage: python scripts/pmc_traffic.py 'gpurun_out/pmc_c3/p[34]/*counter_collection.csv' out.json \
           ['gpurun_out/pmc_c3/cal_*/*counter_collection.csv']
"""
import collections
import csv
import glob
import json
import os
import sys

CAL_BYTES = 512 << 20  # bytes each calibration kernel moves


def collect(pattern, match):
    agg = collections.defaultdict(list)
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if match(r["Kernel_Name"]):
                agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmc_common import frame_counters, kept_dispatches  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

a = frame_counters(sys.argv[1])  # frame launches only (no estimate / companion)
avg = {c: sum(v) / len(v) for c, v in a.items()}
raw_fetch = avg.get("FETCH_SIZE", 0.0) * 1024.0
raw_write = avg.get("WRITE_SIZE", 0.0) * 1024.0
out = {
    "raw_fetch_bytes": raw_fetch,
    "raw_write_bytes": raw_write,
    "dispatches": {c: len(v) for c, v in a.items()},
    "dispatches_dropped": kept_dispatches(sys.argv[1])[1],
    "kernel_src": load_package().render.kernel_source_id(),  # the device code these counters come from
}
cal = {}
if len(sys.argv) > 3:
    for (k, c), v in collect(sys.argv[3], lambda k: any(n in k for n in ("read8", "write8", "write4"))).items():
        name = next(n for n in ("read8", "write8", "write4") if n in k)
        cal["%s/%s" % (name, c)] = (sum(v) / len(v)) * 1024.0 / CAL_BYTES
if cal:
    f_read = cal.get("read8/FETCH_SIZE")
    f_write = cal.get("write8/WRITE_SIZE")
    out["calibration_counter_bytes_per_byte"] = cal
    out["fetch_bytes"] = raw_fetch / f_read if f_read else raw_fetch
    out["write_bytes"] = raw_write / f_write if f_write else raw_write
    out["note"] = ("FETCH_SIZE / WRITE_SIZE (KB->B) per launch, divided by the counter-per-byte of the "
                   "8-B/lane calibration kernels (scripts/pmc_calib.hip)")
else:
    out["fetch_bytes"] = raw_fetch
    out["write_bytes"] = raw_write
    out["note"] = "raw FETCH_SIZE+WRITE_SIZE (KB->B) per launch (uncalibrated)"
out["traffic_bytes"] = out["fetch_bytes"] + out["write_bytes"]
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
