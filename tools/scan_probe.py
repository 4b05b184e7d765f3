"""Diagnostic: one encode of the many-tile inputs of tests/test_gpu_worklist.py::test_scan_many_tiles,
step by step with progress lines (which launch shape / scan path stalls).
usage: scan_probe.py SW NTILE"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import deflate_compression_amd as D

sw, ntile = int(sys.argv[1]), int(sys.argv[2])
nblk = ntile * 256 - 100
rng = np.random.default_rng(5 + ntile)
a = np.zeros(nblk * sw - sw // 3, dtype=np.uint8)
text = D.gen_text(64 * sw, 5 + ntile)
for s in range(0, nblk - 64, 331):
    k = int(rng.integers(1, 32))
    if rng.integers(0, 2):
        a[s * sw:(s + k) * sw] = text[:k * sw]
    else:
        a[s * sw:(s + k) * sw] = rng.integers(0, 256, k * sw, dtype=np.uint8)
print("input", a.size, "blocks", nblk, flush=True)
fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
e = D.Encoder(0, a.size, sw=sw)
t = torch.from_numpy(a).cuda()
for flg in (0, D.DMX_F_STORE_CHECK):
    for v in (1, 0):
        e.set_hook("scan3", v)
        for rep in range(2):
            t0 = time.time()
            z, r = e.compress_tensor(t, opts=D.Opts(sw, 4, D.DMX_ZLIB | D.DMX_F_LAZY | flg, 0))
            print("store_check", bool(flg), "scan3", v, "rep", rep, "status", r.status, "len", int(r.out_len),
                  "s", round(time.time() - t0, 3), flush=True)
e.close()
