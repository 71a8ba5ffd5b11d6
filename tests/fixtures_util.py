"""Loader for the golden fixtures recorded from the reference
(tests/golden/make_golden.py).  Plain npz (allow_pickle=False) + json."""
import json
import os

import numpy as np

FIXDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")


def load(name):
    with open(os.path.join(FIXDIR, name + ".json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(FIXDIR, name + ".npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    draws = [(d["kind"], d["df"], arrays["draw%02d" % i]) for i, d in enumerate(meta["draws"])]
    return meta, arrays, draws


def names():
    return sorted(f[:-5] for f in os.listdir(FIXDIR) if f.endswith(".json"))
