#!/usr/bin/env python
"""Diagnostic (GPU): how many positions of the delayed-null mask table are
f-dependent (k_mask_table's compacted root-record count) for the C3 signal
geometry (2^22 samples, DM 100, null(0.1)); the table is channel-independent,
so a 2-channel run of the C3 step builds the same table.
usage: tools/mask_count.py [log2n] [nchan] [DUMP_PREFIX]
(DUMP_PREFIX: also saves the last rep's root records and output rows, to
compare two builds bit for bit)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def al(b):
    return (b + 255) // 256 * 256


def main():
    import torch
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    nchan = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    import bench
    import psrsigsim_amd as pss
    from psrsigsim_amd import _engine
    pss.seed(1776)
    dump = sys.argv[3] if len(sys.argv) > 3 else None
    for rep in range(3):
        sig = bench.c3_step(pss, nchan, None, log2n)
        torch.cuda.synchronize()
        N = 1 << log2n
        npairs = (nchan + 2) // 2
        misc = al(npairs * N * 8) + al(N * 8) + al(6 * N * 8) + al(12 * N * 4) + al(N // 32 * 8) + \
            al(N // 32 * 4) + al(N * 16 * 4)
        ws = _engine._ws[(torch.cuda.current_device(), "main")]
        cnt = int(ws[misc:misc + 4].cpu().numpy().view(np.uint32)[0])
        nw = int(ws[misc + 8:misc + 12].cpu().numpy().view(np.uint32)[0])
        if dump and rep == 2:
            coef = misc - al(N * 16 * 4)
            np.save(dump + "_rec.npy", ws[coef:coef + cnt * 64].cpu().numpy())
            d = sig.data
            np.save(dump + "_data.npy", d.cpu().numpy() if hasattr(d, "cpu") else np.asarray(d))
        print("rep %d: N=%d f-dependent positions %d (%.2f%%), listed table words %d of %d (%.1f%%)"
              % (rep, N, cnt, 100.0 * cnt / N, nw, N // 32, 100.0 * nw / (N // 32)))


if __name__ == "__main__":
    main()
