"""GPU time per frame from a rocprofv3 kernel trace of a bench run, the
profile-side counterpart of bench.py's kernel_ms (gpu_span_ms): over the last
`steps` render-kernel dispatches (the timed region; run the bench with
--companion off), (latest end - earliest start) / steps. With frames in flight
the dispatches overlap, so this differs from rocprofv3's average duration,
which the summary also reports.
usage: python scripts/trace_span.py kernel_trace.csv|results.db steps [out.json]"""
import csv
import json
import sys


def load(path, kname):
    """Dispatches of kname from a kernel_trace.csv or a rocprofv3 results .db
    (its `kernels` view), as dicts with Start_Timestamp / End_Timestamp."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b}
                for n, a, b in con.execute("select name, start, end from kernels where name like ?",
                                           ("%" + kname + "%",))]
    return [r for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"]]


def span(path, steps, kname="rt_render_kernel"):
    rows = load(path, kname)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-steps:]
    t0 = min(int(r["Start_Timestamp"]) for r in last)
    t1 = max(int(r["End_Timestamp"]) for r in last)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last]
    # overlap: time during which two of these dispatches run at once
    ev = sorted([(int(r["Start_Timestamp"]), 1) for r in last] + [(int(r["End_Timestamp"]), -1) for r in last])
    live, prev, both = 0, None, 0
    for t, d in ev:
        if prev is not None and live >= 2:
            both += t - prev
        live += d
        prev = t
    return {"kernel": kname, "dispatches": len(last), "span_ms_per_frame": (t1 - t0) / len(last) / 1e6,
            "avg_dispatch_ms": sum(durs) / len(durs) / 1e6, "overlap_fraction_of_span": both / (t1 - t0),
            "source": path}


if __name__ == "__main__":
    d = span(sys.argv[1], int(sys.argv[2]))
    s = json.dumps(d, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)
