#!/usr/bin/env python
"""Static instruction mix of a kernel in the gfx950 assembly (diagnostic).

usage: isa_mix.py ASM_FILE NAME_SUBSTRING [...]
Counts the instructions of the (fully unrolled) kernel body by class and
prices them with the issue costs measured by tools/probe_rates.hip at >= 4
waves per SIMD (cycles per wave-instruction per SIMD), to estimate the
VALU-issue time of one wave's work."""
import re
import sys
from collections import Counter

COST = {"valu": 2.5, "valu_half": 4.3, "trans": 8.3, "pk": 7.5, "salu": 1.0}
HALF = ("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_u32_u24", "v_mul_u32_u24", "v_mul_hi_u32_u24",
        "v_cvt_f32_u32", "v_cvt_f32_i32", "v_cvt_u32_f32", "v_cvt_i32_f32", "v_mad_i64_i32", "v_mul_i32_i24",
        "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64", "v_cvt_f64", "v_fma_f64", "v_add_f64", "v_mul_f64")
TRANS = ("v_sin_f32", "v_cos_f32", "v_log_f32", "v_exp_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32")


def classify(m):
    if m.startswith("v_pk_"):
        return "pk"
    if m.startswith(TRANS):
        return "trans"
    if m.startswith(HALF):
        return "valu_half"
    if m.startswith("v_"):
        return "valu"
    if m.startswith("s_"):
        return "salu"
    for p in ("ds_", "buffer_", "global_", "scratch_", "flat_"):
        if m.startswith(p):
            return p[:-1]
    return "other"


def main():
    text = open(sys.argv[1]).read()
    for sub in sys.argv[2:]:
        names = sorted(set(n for n in re.findall(r"^(_Z\w+):", text, re.M) if sub in n and not n.startswith(".")))
        for n in names:
            i = text.index("\n" + n + ":")
            j = text.index(".Lfunc_end", i)
            ins = [l.split()[0] for l in text[i:j].split("\n")[1:] if l.startswith("\t") and not l.startswith("\t.")
                   and not l.startswith("\t;")]
            c = Counter(classify(m) for m in ins)
            mn = Counter(m for m in ins)
            cyc = sum(COST.get(k, 0) * v for k, v in c.items())
            print("%s\n  total %d  %s\n  VALU-issue estimate %.0f cycles/wave  top: %s" % (
                n[:90], len(ins), dict(c), cyc, mn.most_common(12)))


if __name__ == "__main__":
    main()
