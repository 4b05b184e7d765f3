"""Diagnostic: back-to-back encode_async throughput (bench.py's N = 1 timed loop: no sync
between steps) of one configuration, optionally with a kernel variant (DMX_LIBV).
usage: pipe_time.py [MB] [K] [flags: l s d c e] [text|random|zeros] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import deflate_compression_amd as D

if os.environ.get("DMX_LIBV"):
    D.LIB_PATH = os.environ["DMX_LIBV"]

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 1073.741824
k = int(sys.argv[2]) if len(sys.argv) > 2 else 7
fs = sys.argv[3] if len(sys.argv) > 3 else "lce"
kind = sys.argv[4] if len(sys.argv) > 4 else "random"
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
flags = D.DMX_ZLIB | (D.DMX_F_LAZY if "l" in fs else 0) | (D.DMX_F_SPLIT if "s" in fs else 0) | \
    (D.DMX_F_DICT if "d" in fs else 0) | (D.DMX_F_STORE_CHECK if "c" in fs else 0) | \
    (D.DMX_F_DEEP if "e" in fs else 0)
n = int(mb * 1e6)
host = {"text": lambda: D.gen_text(n, 0xE5818), "random": lambda: D.gen_random(n, 0x5EED),
        "zeros": lambda: __import__("numpy").zeros(n, __import__("numpy").uint8)}[kind]()
d_in = torch.from_numpy(host).cuda()
cap = D.max_compressed(n)
d_out = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
e = D.Encoder(0, n, max_chain=k, flags=flags)
stream = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    e.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
torch.cuda.synchronize()
best = None
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(steps):
        e.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    best = dt if best is None else min(best, dt)
r = e.result(stream)
print({"lib": os.path.basename(D.LIB_PATH), "config": f"{mb} MB K={k} {fs} {kind}", "GBps": round(n / best / 1e9, 1),
       "ms_per_step": round(best * 1e3, 4), "out_len": int(r.out_len), "status": int(r.status)}, flush=True)
e.close()
