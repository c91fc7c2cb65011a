#!/usr/bin/env python3
"""Markdown tables for BASELINE.md from a final rehearsal's results: the
per-config bench lines (sweep/*.json, with their CPU baselines and PMC
fields) and the 1-GPU rehearsal of every rank's share (strong/inflight_*.json).
usage: python3 scripts/baseline_table.py profiles/r05/final"""
import glob
import json
import os
import sys

NAMES = {
    "c1": "C1 1 sphere 256² d1",
    "c2": "C2 3 spheres + plane, 1920×1080 d4",
    "canned": "canned.gml 1900×1200 d7 (golden)",
    "c3": "C3 cyl + cube + sphere, 4 lights, 3840×2160 d6 (**bench**)",
    "c3cone": "C3 as specified (cone, extension)",
    "c4": "C4 cube ∪ 64 spheres, 3840×2160 d8 (BVH)",
    "c4csg": "C4 as specified: cube − 64 spheres (CSG extension) d8",
    "c5": "C5 100 k spheres, 7680×4320 d8 (BVH)",
}


def pct(v):
    return "—" if v is None else "%.1f %%" % (100 * v)


def main():
    d = sys.argv[1]
    print("| config | CPU 8 thr Mrays/s | CPU all Mrays/s | 1 GPU Mrays/s | ms/frame | FP64 frac (alg.) | executed (PMC) | issue / lanes | HBM / frame |")
    print("|---|---|---|---|---|---|---|---|---|")
    for c in ["c1", "c2", "canned", "c3", "c3cone", "c4", "c4csg", "c5"]:
        p = os.path.join(d, "sweep", c + ".json")
        if not os.path.exists(p):
            continue
        j = json.load(open(p))
        r = j["roofline"]
        cb = j.get("cpu_baseline") or {}
        allc = (cb.get("all_cores") or {}).get("value")
        rows = "" if "full" in cb.get("sample", "") else " (%s)" % cb.get("sample", "").split(" of the")[0]
        il = "%.2f / %.2f" % (r["issue_util"], r["lane_util"]) if r.get("issue_util") else "—"
        tr = "%.2f GB" % (r["traffic"] / 1e9) if r.get("traffic") else "—"
        frac = r.get("frac")
        print("| %s | %s%s | %s | %s | %.4g | %s | %s | %s | %s |" % (
            NAMES[c], "%.4g" % cb["value"] if cb else "—", rows, "%.4g" % allc if allc else "—",
            "{:,.0f}".format(j["value"]).replace(",", " "), j["ms_per_step"],
            pct(frac) if frac is not None else "(%s)" % ("CSG" if c == "c4csg" else "BVH"),
            pct(r.get("executed_frac")), il, tr))
    print()
    print("| config | 1 | 2 ranks | 4 ranks | 8 ranks |")
    print("|---|---|---|---|---|")
    for p in sorted(glob.glob(os.path.join(d, "strong", "inflight_*.json"))):
        j = json.load(open(p))
        c = j["config"]
        cells = []
        for w in (1, 2, 4, 8):
            ms = j.get("w%d_f2_max_ms" % w)
            eff = j.get("w%d_f2_eff_max" % w)
            cells.append("—" if ms is None else ("%.3f ms" % ms if w == 1 else "%.3f ms (%.2f)" % (ms, eff)))
        print("| %s | %s |" % (c, " | ".join(cells)))


if __name__ == "__main__":
    main()
