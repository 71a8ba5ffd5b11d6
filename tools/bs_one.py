"""One Bluestein geometry for rocprofv3 (kernel stats): shift_t on 512 rows
of 2^20 - 2 samples (tools/bs_time.py's headline case), 5 timed calls."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from psrsigsim_amd.utils import shift_t

R, N = int(sys.argv[1]) if len(sys.argv) > 1 else 512, int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 20) - 2
x = torch.rand((R, N), device="cuda")
s = np.linspace(0.3, 1234.5, R)
for _ in range(6):
    shift_t(x, s, dt=1.0)
torch.cuda.synchronize()
print("done", R, N)
