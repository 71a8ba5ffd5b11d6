#!/usr/bin/env python
"""Static instruction mix of a kernel in the gfx950 assembly (diagnostic).

usage: isa_mix.py ASM_FILE NAME_SUBSTRING [...]
(ASM_FILE: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize
 --cuda-device-only -S -o pss.s psrsigsim_amd/csrc/pss_fourstep.hip: the C3 kernels; other units for the other paths)

For each matching kernel: the per-class count of the (fully unrolled)
kernel body, per phase (the code between workgroup barriers) and in total,
priced with the issue costs tools/probe_rates.hip measured at >= 4 waves per
SIMD (cycles per wave-instruction per SIMD) to estimate the VALU-issue time
of one wave's work.  Classes: float arithmetic (add/sub/mul/fma), integer /
address / bit arithmetic, conversions, transcendentals, data moves / selects
/ compares, packed f32, LDS, global/buffer memory, scalar.  Static counts:
loops that are not unrolled count once."""
import re
import sys
from collections import Counter, OrderedDict

COST = {"f_arith": 2.5, "int": 2.5, "int_half": 4.3, "cvt": 4.3, "trans": 8.3, "move": 2.5, "pk": 7.5}
TRANS = ("v_sin_f32", "v_cos_f32", "v_log_f32", "v_exp_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32")
HALF_INT = ("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_i64_i32", "v_lshlrev_b64", "v_lshrrev_b64",
            "v_ashrrev_i64")
F_ARITH = ("v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32",
           "v_fmaak_f32", "v_mac_f32", "v_min_f32", "v_max_f32", "v_ldexp_f32", "v_div_", "v_fma_f64", "v_add_f64",
           "v_mul_f64")
MOVE = ("v_mov_", "v_cndmask", "v_cmp", "v_readlane", "v_readfirstlane", "v_writelane", "v_accvgpr", "v_perm",
        "v_swap")


def classify(m):
    if m.startswith("v_pk_"):
        return "pk"
    if m.startswith(TRANS):
        return "trans"
    if m.startswith("v_cvt"):
        return "cvt"
    if m.startswith(F_ARITH):
        return "f_arith"
    if m.startswith(MOVE):
        return "move"
    if m.startswith(HALF_INT):
        return "int_half"
    if m.startswith("v_"):
        return "int"
    if m.startswith("s_"):
        return "salu"
    for p in ("ds_", "buffer_", "global_", "scratch_", "flat_"):
        if m.startswith(p):
            return p[:-1]
    return "other"


def kernel_body(text, name):
    i = text.index("\n" + name + ":")
    j = text.index(".Lfunc_end", i)
    return [l.split()[0] for l in text[i:j].split("\n")[1:]
            if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]


def report(name, ins):
    phases, cur = [], []
    for m in ins:
        if m == "s_barrier":
            phases.append(cur)
            cur = []
        else:
            cur.append(m)
    phases.append(cur)
    keys = ["f_arith", "int", "int_half", "cvt", "trans", "move", "pk", "ds", "buffer", "global", "scratch", "salu"]
    out = ["%s" % name[:110], "  %-8s %s %8s" % ("phase", " ".join("%8s" % k for k in keys), "VALUcyc")]
    tot = Counter()
    for pi, ph in enumerate(phases):
        c = Counter(classify(m) for m in ph)
        tot += c
        if sum(c.values()) < 12:
            continue
        cyc = sum(COST.get(k, 0) * v for k, v in c.items())
        out.append("  %-8s %s %8.0f" % ("p%d" % pi, " ".join("%8d" % c.get(k, 0) for k in keys), cyc))
    cyc = sum(COST.get(k, 0) * v for k, v in tot.items())
    valu = sum(tot.get(k, 0) for k in ("f_arith", "int", "int_half", "cvt", "trans", "move", "pk"))
    out.append("  %-8s %s %8.0f" % ("total", " ".join("%8d" % tot.get(k, 0) for k in keys), cyc))
    out.append("  VALU instructions %d, of which float arithmetic %.0f%%, integer/address %.0f%%, "
               "moves/selects/compares %.0f%%, conversions %.0f%%, transcendentals %.0f%%"
               % (valu, 100.0 * tot["f_arith"] / valu, 100.0 * (tot["int"] + tot["int_half"]) / valu,
                  100.0 * tot["move"] / valu, 100.0 * tot["cvt"] / valu, 100.0 * tot["trans"] / valu))
    out.append("  top: %s" % Counter(ins).most_common(14))
    return "\n".join(out)


def main():
    text = open(sys.argv[1]).read()
    for sub in sys.argv[2:]:
        names = sorted(set(n for n in re.findall(r"^(_Z\w+):", text, re.M) if sub in n and not n.startswith(".")))
        for n in names:
            print(report(n, kernel_body(text, n)))
            print()


if __name__ == "__main__":
    main()
