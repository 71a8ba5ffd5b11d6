"""Host (Python / ctypes) cost of a workload's steps with the device calls
stubbed out -- a CPU-only view of the per-step API overhead (no GPU needed):
pss_run and the other launches return at once, device tensors are CPU tensors.
usage: tools/host_cpu_profile.py t2|t1|c4|c3 [steps] [--prof]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import logging  # noqa: E402
logging.disable(logging.WARNING)

import psrsigsim_amd as pss  # noqa: E402
from psrsigsim_amd import _engine, _lib  # noqa: E402

_real = _lib.load()


class _Stub(object):
    """The library with its device entry points replaced by no-ops."""
    def __getattr__(self, name):
        if name.startswith("pss_host_") or name in ("pss_workspace_bytes", "pss_filter_workspace_bytes",
                                                       "pss_last_error", "pss_plan_collect"):
            return getattr(_real, name)
        return lambda *a: 0


_stub = _Stub()
_lib.lib = lambda: _stub
_engine.device = lambda: torch.device("meta")
_engine.to_dev = lambda a, dtype=None: torch.as_tensor(np.ascontiguousarray(a)) if dtype is None else \
    torch.as_tensor(np.ascontiguousarray(a)).to(dtype)
_engine.stream_ptr = lambda: None
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "t2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 50
step = {"c4": lambda: bench.c4_step(pss, 2048, None, False),
        "c3": lambda: bench.c3_step(pss, 2048, None, 22),
        "t1": lambda: bench.tutorial_step(pss, "t1", 128, None),
        "t2": lambda: bench.tutorial_step(pss, "t2", 64, None)}[wl]
for _ in range(3):
    step()
t = time.perf_counter()
for _ in range(steps):
    step()
print("%s: host %.3f ms/step (device calls stubbed)" % (wl, (time.perf_counter() - t) / steps * 1e3))
if "--prof" in sys.argv:
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    pr.disable()
    pstats.Stats(pr).sort_stats(sys.argv[-1] if sys.argv[-1] in ("tottime", "cumtime") else "cumtime").print_stats(40)
