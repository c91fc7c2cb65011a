"""Static instruction classes of a gfx950 kernel's ISA (hipcc -S output):
counts per class, optionally per code region between markers. Used for the
C3 instruction budget: which classes the VALU / SALU streams are
made of. usage: python scripts/isa_classes.py kernel.s [--top N]"""
import collections
import re
import sys

CLASSES = [
    ("fp64_divsqrt", r"^v_(div_scale|div_fmas|div_fixup|rcp|rsq|sqrt)_f64"),
    ("fp64_arith", r"^v_(add|mul|fma|ldexp|max|min|frexp_mant|frexp_exp_i32|fract|trig_preop)_f64"),
    ("fp64_cmp", r"^v_cmpx?_\w+_f64"),
    ("fp64_cvt", r"^v_cvt_\w*f64|^v_cvt_f64"),
    ("fp32", r"^v_(pk_)?(add|sub|subrev|mul|fma|fmac|mac|max|min|max3|min3|med3|rcp|rsq|sqrt|ldexp|floor|ceil|fract|exp|log)_f32"),
    ("fp32_cmp", r"^v_cmpx?_\w+_f32"),
    ("int_cmp", r"^v_cmpx?_\w+_[iu](16|32|64)"),
    ("cmp_other", r"^v_cmpx?_"),
    ("select", r"^v_cndmask"),
    ("move", r"^v_(mov|readfirstlane|accvgpr_mov)"),
    ("lane_xfer", r"^v_(readlane|writelane)"),
    ("dpp_perm", r"^v_(perm|permlane|mov_b32_dpp|bpermute)|^ds_(bpermute|permute|swizzle)"),
    ("int", r"^v_(add|sub|subrev|addc|subb|mad|mul|lshl|lshr|ashr|and|or|xor|not|bfe|bfi|alignbit|alignbyte|max|min|mbcnt|bcnt|ffbh|ffbl|cvt|lshlrev|lshrrev|ashrrev|add3|lshl_add|lshl_or|and_or|or3|xad|mad_u64|mad_i64|med3)"),
    ("v_other", r"^v_"),
    ("lds", r"^ds_"),
    ("vmem", r"^(global|buffer|flat|scratch)_"),
    ("smem", r"^s_(load|buffer_load|store|buffer_store|dcache|memtime|memrealtime)"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc|getpc)"),
    ("wait_nop", r"^s_(waitcnt|nop|sleep|barrier|sethalt|setprio|sched|endpgm|trap|sendmsg|icache|ttracedata)"),
    ("salu_exec", r"^s_(and|or|xor|andn2|orn2|nand|nor|xnor)_saveexec|^s_(and|or|andn2|xor|orn2)_b64\s+exec|^s_mov_b64\s+exec"),
    ("salu", r"^s_"),
]
RX = [(n, re.compile(p)) for n, p in CLASSES]


def classify(op, line):
    for n, rx in RX:
        if n == "salu_exec":
            if rx.search(line.strip()):
                return n
            continue
        if rx.search(op):
            return n
    return "other"


def main():
    path = sys.argv[1]
    counts = collections.Counter()
    ops = collections.Counter()
    in_text = False
    for line in open(path):
        t = line.strip()
        if t.startswith(".text") or t.startswith(".section\t.text"):
            in_text = True
        if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if not re.match(r"^[vsgbfd][a-z_0-9]*$", op):
            continue
        c = classify(op, t)
        counts[c] += 1
        ops[(c, op)] += 1
    tot = sum(counts.values())
    for c, n in counts.most_common():
        print("%-14s %6d  %5.1f%%" % (c, n, 100.0 * n / tot))
    print("total %d" % tot)
    if "--top" in sys.argv:
        k = int(sys.argv[sys.argv.index("--top") + 1])
        for (c, op), n in ops.most_common(k):
            print("  %-14s %-28s %d" % (c, op, n))


if __name__ == "__main__":
    main()
