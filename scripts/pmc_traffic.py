"""Per-launch HBM traffic of the render kernel from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters from the TCC
EA read/write requests). Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reads half
the bytes of wide (16 B/lane) coalesced streaming loads; this kernel's loads
are not of that kind (scene in LDS, 8-B frame fields), so the raw sum is
reported and labelled as such. Writes: frame-stack pushes (8 B/lane fields)
and 4 B/pixel framebuffer stores.

usage: python scripts/pmc_traffic.py 'gpurun_out/pmcT/*/*counter_collection.csv' out.json
"""
import collections
import csv
import glob
import json
import sys

agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1]):
    for r in csv.DictReader(open(f)):
        if "rt_render" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in agg.items()}
out = {
    "fetch_bytes": a.get("FETCH_SIZE", 0.0) * 1024.0,
    "write_bytes": a.get("WRITE_SIZE", 0.0) * 1024.0,
    "dispatches": {k: len(v) for k, v in agg.items()},
    "note": "raw FETCH_SIZE+WRITE_SIZE (KB->B) per launch; FETCH not doubled (loads are not 16B/lane streams)",
}
out["traffic_bytes"] = out["fetch_bytes"] + out["write_bytes"]
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
