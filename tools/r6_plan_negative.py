"""One-off check: the plan assertions of the parity tests
fail when the expected kernels are wrong.  Runs the C3-geometry fast-path
oracle test with a wrong expected split (2048 x 2048) and then a wrong pass C
(C:generic expected), each of which must raise AssertionError.  GPU box."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_fastpath_oracle as T  # noqa: E402

good = T.PLANS["c3"]
for wrong in (("fourstep", "2048x2048", "A:fast"), ("fourstep", "1024x4096", "C:generic")):
    T.PLANS["c3"] = wrong
    try:
        T.test_fast_path_channels_vs_oracle("c3", None)
    except AssertionError as e:
        print("expected %s: raised as it should: %s" % (wrong, str(e)[:200]))
    else:
        print("expected %s: NOT raised" % (wrong,))
        sys.exit(1)
T.PLANS["c3"] = good
T.test_fast_path_channels_vs_oracle("c3", None)
print("right plan: passes")
