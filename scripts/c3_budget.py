"""C3 instruction budget: dynamic instructions per phase and class.

Inputs (all measured on the same kernel build):
  * dynamic class totals per frame: rocprofv3 --pmc SQ_INSTS_VALU_{ADD,MUL,
    FMA,TRANS}_{F32,F64}, _INT32, _INT64, _CVT, SQ_INSTS_VALU, _SALU,
    _BRANCH, _SMEM, _LDS, _VMEM_RD/WR (scripts/gpu/r6_budget.sh summary);
  * the phase split of wave cycles (diagnostic build, [phase] line);
  * the static instruction mix of each phase in the ISA of the same kernel
    (scripts/isa_phases.py on the -DRT_PHASE_TIMING listing, PMC classes).
Each phase's issued instructions are taken proportional to its wave cycles
(the kernel is issue-bound: 4 x (VALU + SALU) tracks wave cycles per SIMD),
split by its static class mix, and the table is then raked (iterative
proportional fitting) so that every class column sums to its PMC total while
every phase row keeps its cycle share. Static code that runs rarely (cold
fix-up paths the compiler moves out of line) is left out of the mixes.
usage: python scripts/c3_budget.py summary.txt phase.err isa_phase.s [--json out]"""
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

PHASES = ["refill", "gen", "trace_loop", "trace_unwind", "shade_surface", "light_dirs", "shadow_loops", "lighting",
          "material", "shade_unwind"]
# PMC-aligned classes
PCLS = [
    ("fp64", r"^v_(add|mul|fma|fmac|rcp|rsq|sqrt|div_fmas)_f64"),
    ("fp32", r"^v_(pk_)?(add|sub|subrev|mul|fma|fmac|mac|rcp|rsq|sqrt|exp|log)_f32"),
    ("cvt", r"^v_cvt_"),
    ("int64", r"^v_(mad_u64_u32|mad_i64_i32|lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|add_co_u32|addc_co_u32|sub_co_u32|subb_co_u32)"),
    ("int32", r"^v_(add|sub|subrev|mul_lo|mul_hi|mad_u32|mad_i32|lshl|lshr|ashr|and|or|xor|not|bfe|bfi|alignbit|alignbyte|max_i|max_u|min_i|min_u|mbcnt|bcnt|ffbh|ffbl|add3|lshl_add|lshl_or|and_or|or3|xad|med3_i|med3_u)"),
    ("valu_other", r"^v_"),
    ("salu", r"^s_(?!load|buffer_load|store|dcache|memtime|memrealtime|waitcnt|nop|sleep|barrier|endpgm|cbranch|branch|setpc|swappc|sendmsg)"),
    ("branch", r"^s_(cbranch|branch)"),
    ("smem", r"^s_(load|buffer_load)"),
    ("lds", r"^ds_"),
    ("vmem", r"^(global|buffer|flat|scratch)_"),
]
RX = [(n, re.compile(p)) for n, p in PCLS]


def pcls(op):
    for n, rx in RX:
        if rx.search(op):
            return n
    return None


def static_mix(path):
    inside = False
    tab = collections.defaultdict(collections.Counter)
    pending = collections.Counter()
    for line in open(path):
        t = line.strip()
        if not inside:
            inside = bool(re.match(r"^_Z\w*rt_render_kernel\w*:", t))
            continue
        m = re.match(r";\s*@phase_end (\d+)", t)
        if m:
            tab[PHASES[int(m.group(1))]].update(pending)
            pending = collections.Counter()
            continue
        if t.startswith("s_memtime") and not tab and not any(pending.values()):
            pending = collections.Counter()
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = pcls(op)
        if c:
            pending[c] += 1
    return tab


def pmc_totals(path):
    a = {}
    for line in open(path):
        m = re.match(r"(\w+)\s+n=\d+\s+avg=([\d.e+-]+)", line)
        if m:
            a[m.group(1)] = float(m.group(2))
    fp64 = sum(a["SQ_INSTS_VALU_%s_F64" % k] for k in ("ADD", "MUL", "FMA", "TRANS"))
    fp32 = sum(a["SQ_INSTS_VALU_%s_F32" % k] for k in ("ADD", "MUL", "FMA", "TRANS"))
    tot = {"fp64": fp64, "fp32": fp32, "cvt": a["SQ_INSTS_VALU_CVT"], "int64": a["SQ_INSTS_VALU_INT64"],
           "int32": a["SQ_INSTS_VALU_INT32"]}
    tot["valu_other"] = a["SQ_INSTS_VALU"] - sum(tot.values())
    tot["salu"] = a["SQ_INSTS_SALU"]
    tot["branch"] = a["SQ_INSTS_BRANCH"]
    tot["smem"] = a["SQ_INSTS_SMEM"]
    tot["lds"] = a["SQ_INSTS_LDS"]
    tot["vmem"] = a.get("SQ_INSTS_VMEM_RD", 0) + a.get("SQ_INSTS_VMEM_WR", 0)
    return tot, a


def phase_shares(path):
    """The last [phase] line: the timed frames' counters (bench.py reads and
    resets them after the warm-up, then after the timed steps)."""
    last = None
    for line in open(path):
        if line.startswith("[phase]"):
            last = line
    if last is None:
        raise SystemExit("no [phase] line")
    d = dict(re.findall(r"(\w+)=([\d.e+-]+)", last))
    return {p: float(d[p]) for p in PHASES}


def main():
    summ, perr, isa = sys.argv[1:4]
    tot, raw = pmc_totals(summ)
    share = phase_shares(perr)
    mix = static_mix(isa)
    classes = list(tot)
    itot = sum(tot.values())
    # initial table: phase instructions by cycle share, split by static mix
    T = {}
    for p in PHASES:
        m = mix[p]
        n = sum(m[c] for c in classes) or 1
        for c in classes:
            T[p, c] = share[p] * itot * (m[c] / n) + 1e-9
    for _ in range(200):  # rake: columns to the PMC totals, rows to the cycle shares
        for c in classes:
            s = sum(T[p, c] for p in PHASES)
            for p in PHASES:
                T[p, c] *= tot[c] / s if s > 0 else 0.0
        for p in PHASES:
            s = sum(T[p, c] for c in classes)
            for c in classes:
                T[p, c] *= share[p] * itot / s
    print("C3 dynamic instructions per frame (millions of wave-instructions), by phase and class")
    print("%-14s" % "phase" + "".join("%9s" % c[:9] for c in classes) + "    total  cycles")
    for p in PHASES:
        row = [T[p, c] / 1e6 for c in classes]
        print("%-14s" % p + "".join("%9.1f" % v for v in row) + "%9.1f  %5.1f%%" % (sum(row), 100 * share[p]))
    print("%-14s" % "total" + "".join("%9.1f" % (tot[c] / 1e6) for c in classes) + "%9.1f" % (itot / 1e6))
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        json.dump({"classes_per_frame": tot, "phase_cycle_share": share,
                   "table_millions": {p: {c: round(T[p, c] / 1e6, 2) for c in classes} for p in PHASES},
                   "static_mix": {p: dict(mix[p]) for p in PHASES},
                   "method": __doc__.strip().splitlines()[2:17]}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
