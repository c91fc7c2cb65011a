"""Static instruction classes per phase of the diagnostic render kernel
(-DRT_PHASE_TIMING: every PH_MARK(k) leaves "; @phase_end k" in the ISA
listing, and the code between two marks is the phase that ends at the second).
Code before the first stamp is the kernel prologue; code after the last mark
is the loop's back edge plus blocks the compiler moved out of line (cold
fix-up paths), reported apart. Feeds the C3 instruction budget.
usage: python scripts/isa_phases.py kernel_phase.s [--json out.json]"""
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_classes import classify  # noqa: E402

NAMES = ["refill", "gen", "trace_loop", "trace_unwind", "shade_surface", "light_dirs", "shadow_loops", "lighting",
         "material", "shade_unwind"]


def main():
    path = sys.argv[1]
    seg = "prologue"
    started = False
    inside = False
    table = collections.defaultdict(collections.Counter)
    pending = collections.Counter()
    for line in open(path):
        t = line.strip()
        if not inside:  # the render kernel's body only
            inside = bool(re.match(r"^_Z\w*rt_render_kernel\w*:", t))
            continue
        m = re.match(r";\s*@phase_end (\d+)", t)
        if m:
            k = int(m.group(1))
            table[NAMES[k]].update(pending)
            pending = collections.Counter()
            seg = "after_last_mark"
            continue
        if t.startswith("s_memtime") and not started:
            started = True
            table["prologue"].update(pending)
            pending = collections.Counter()
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if not re.match(r"^[vsgbfd][a-z_0-9]*$", op):
            continue
        pending[classify(op, t)] += 1
    table["out_of_line"].update(pending)
    classes = sorted({c for v in table.values() for c in v}, key=lambda c: -sum(v[c] for v in table.values()))
    order = ["prologue"] + NAMES + ["out_of_line"]
    print("%-14s" % "phase" + "".join("%9s" % c[:9] for c in classes) + "   total")
    for ph in order:
        v = table.get(ph, collections.Counter())
        print("%-14s" % ph + "".join("%9d" % v[c] for c in classes) + "%8d" % sum(v.values()))
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        json.dump({ph: dict(table.get(ph, {})) for ph in order}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
