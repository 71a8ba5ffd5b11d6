"""Ambiguity-band and flip statistics of the delayed-null parity cases
(tests/replay.py STATS) on the GPU: C4 with a null on the fallback path, and
the four-step table path for comparison.  usage: python tools/null_band.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import replay
from tests.test_gpu_parity import _c4_case, _big_case

for name, case, seed in [("c4 null gauss 2ch", _c4_case(2, True), 2),
                         ("c4 null b1855 2ch", _c4_case(2, True, ("b1855", 2)), 2),
                         ("2^16 null table", _big_case(16, 3, null=True), 16)]:
    replay.STATS.clear()
    try:
        errs = replay.run_case(None, fused=True, case=case, seed=seed)
        worst = "worst err %.3g" % max(errs.values())
    except AssertionError as e:
        worst = "FAILED: %s" % e
    print(name, worst, {k: (round(v, 6) if isinstance(v, float) else v) for k, v in replay.STATS.items()})
