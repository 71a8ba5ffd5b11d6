import numpy as np, sys
sys.path.insert(0, '.')
from tools.diag_fast import run
from psrsigsim_amd import _lib
L = _lib.lib()
for log2n in (14, 16):
    fast = run(2, log2n, False, False, 1e-3)
    old = L.pss_set_flags(_lib.FLAG_NO_FAST)
    gen = run(2, log2n, False, False, 1e-3)
    L.pss_set_flags(old)
    d = np.abs(fast - gen)
    print(log2n, 'n diff', int((d > 0).sum()), 'max', d.max())
    for r in range(2):
        idx = np.argsort(d[r])[::-1][:12]
        print(' row', r, [(int(i), float(d[r, i]), float(gen[r, i])) for i in sorted(idx)])
    # relative difference histogram where gen != 0
    rel = d / np.maximum(np.abs(gen), 1e-30)
    print(' rel quantiles', np.quantile(rel[d > 0], [0.5, 0.9, 0.99, 1.0]))
