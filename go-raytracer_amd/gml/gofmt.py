"""Go value formatting used by the RenderArgs dumps (strconv 'g' -1, %v)."""


def go_g(x):
    """strconv.FormatFloat(x, 'g', -1, 64) == fmt %v for float64."""
    if x != x:
        return "NaN"
    if x == float("inf"):
        return "+Inf"
    if x == float("-inf"):
        return "-Inf"
    if x == 0:
        return "-0" if str(x).startswith("-") else "0"
    r = repr(x)  # shortest round-trip digits
    neg = r.startswith("-")
    if neg:
        r = r[1:]
    if "e" in r:
        mant, exp = r.split("e")
        exp = int(exp)
    else:
        mant, exp = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    if fp == "0":
        fp = ""
    digits = (ip + fp).lstrip("0")
    # decimal point position relative to the digit string
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    dp = len(ip) + exp - lead_zeros
    digits = digits.rstrip("0") or "0"
    e = dp - 1
    if e < -4 or e >= 6:  # strconv ftoa.go: shortest => eprec 6
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        s = "%se%s%02d" % (m, "-" if e < 0 else "+", abs(e))
    else:
        if dp <= 0:
            s = "0." + "0" * (-dp) + digits
        elif dp >= len(digits):
            s = digits + "0" * (dp - len(digits))
        else:
            s = digits[:dp] + "." + digits[dp:]
    return ("-" if neg else "") + s


def format_float(x):
    """gml.FormatFloat (expr.go:120-128): 'g' -1 plus a trailing .0 for integers."""
    s = go_g(x)
    if any(c in s for c in ".eE") or s in ("NaN", "+Inf", "-Inf"):
        return s
    return s + ".0"


def fmt_fixed(x):
    """%+-10.2f (evaluator_test_helpers.go:31)."""
    return "%+-10.2f" % x
