"""Delayed-null ambiguity band and flips per replay case, with the packed
paths' float64 decisions (default) and without them (PSS_FLAG_NULL_F32):
tests/replay.py STATS for the null cases of tests/test_gpu_parity.py and the
golden replays.  GPU box only (diagnostic).  usage: tools/null_band_r4.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import replay  # noqa: E402
import test_gpu_parity as P  # noqa: E402
from psrsigsim_amd import _lib  # noqa: E402


def cases():
    yield "c4_gauss_null", P._c4_case(2, True), 2
    yield "c4_b1855_null", P._c4_case(2, True, ("b1855", 2)), 2
    c = P._big_case(0, 3, null=True)
    c["ops"][1] = ("make_pulses", (10006 + 0.5) * 20.48e-6, "pulses")
    yield "bluestein_10006", c, 10009
    c = P._big_case(0, 2, null=True)
    c["ops"][1] = ("make_pulses", (100002 + 0.5) * 20.48e-6, "pulses")
    yield "bluestein_100002", c, 100004
    yield "golden_northstar_mini", None, None
    yield "golden_fold_sublen", None, None


def main():
    L = _lib.lib()
    for refined in (True, False):
        replay.REFINED = refined
        old = L.pss_set_flags(0 if refined else _lib.FLAG_NULL_F32)
        try:
            for name, case, seed in cases():
                replay.STATS.clear()
                note = ""
                errs = {}
                try:
                    if case is None:
                        errs = replay.run_case(name.replace("golden_", ""), fused=True)
                    else:
                        errs = replay.run_case(None, fused=True, case=case, seed=seed)
                except AssertionError as e:
                    note = " ASSERT: %s" % e
                worst = max(errs.values()) if errs else float("nan")
                print("%-8s %-22s path=%-8s band=%.3g flipped=%.3g worst_err=%.3g" % (
                    "f64" if refined else "f32", name, replay.STATS.get("ambiguous_path"),
                    replay.STATS.get("ambiguous_band_frac", float("nan")),
                    replay.STATS.get("null_flipped_frac", float("nan")), worst) + note, flush=True)
        finally:
            L.pss_set_flags(old)


if __name__ == "__main__":
    main()
