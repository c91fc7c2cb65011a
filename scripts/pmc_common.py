"""Render-kernel rows of rocprofv3 --pmc counter CSVs, per frame launch.

A bench process also launches the scene-setup tile-cost estimate (the same
kernel, a few % of a frame's work) and, for C3, the c3cone companion frames
(bench.py --companion; the PMC scripts turn it off). Averages over every
rt_render dispatch would mix them in, so a dispatch counts only if its
duration is at least half the median rt_render duration of its pass.
"""
import collections
import csv
import glob
import statistics


def frame_counters(pattern, kname="rt_render"):
    """{counter: [value per kept dispatch]} over the CSVs matching pattern
    (each pass's dispatches filtered on their own durations)."""
    out = collections.defaultdict(list)
    for f in sorted(glob.glob(pattern)):
        rows = [r for r in csv.DictReader(open(f)) if kname in r["Kernel_Name"]]
        dur = {}
        for r in rows:
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if not dur:
            continue
        med = statistics.median(dur.values())
        keep = {d for d, t in dur.items() if t >= 0.5 * med}
        for r in rows:
            if r["Dispatch_Id"] in keep:
                out[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def kept_dispatches(pattern, kname="rt_render"):
    """(kept, dropped) dispatch counts, for the summaries."""
    kept = dropped = 0
    for f in sorted(glob.glob(pattern)):
        dur = {}
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if dur:
            med = statistics.median(dur.values())
            k = sum(1 for t in dur.values() if t >= 0.5 * med)
            kept += k
            dropped += len(dur) - k
    return kept, dropped
