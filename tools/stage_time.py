"""Diagnostic: HIP-event stage times (ms) of one encode configuration on cuda:0, averaged
over a few encodes (no verification -- for experiments on a kernel variant).
usage: stage_time.py [MB] [K] [flags: any of l(azy) s(plit) d(ict) c(store check) e (deep)] [text|random|zeros] [nowl|list|plain]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import deflate_compression_amd as D

if os.environ.get("DMX_LIBV"):   # a kernel variant built beside libdmx.so
    D.LIB_PATH = os.environ["DMX_LIBV"]

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 100
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
fs = sys.argv[3] if len(sys.argv) > 3 else "lc"
flags = D.DMX_ZLIB | (D.DMX_F_LAZY if "l" in fs else 0) | (D.DMX_F_SPLIT if "s" in fs else 0) | \
    (D.DMX_F_DICT if "d" in fs else 0) | (D.DMX_F_STORE_CHECK if "c" in fs else 0) | \
    (D.DMX_F_DEEP if "e" in fs else 0)
n = int(mb * 1e6)
kind = sys.argv[4] if len(sys.argv) > 4 else "text"
if len(sys.argv) > 5:   # DMX_WORKLIST: 0 = no work lists, list / plain = that launch shape
    os.environ["DMX_WORKLIST"] = {"nowl": "0"}.get(sys.argv[5], sys.argv[5])
host = {"text": lambda: D.gen_text(n, 0xE5818), "random": lambda: D.gen_random(n, 0x5EED),
        "zeros": lambda: __import__("numpy").zeros(n, __import__("numpy").uint8)}[kind]()
t = torch.from_numpy(host).cuda()
e = D.Encoder(0, n, max_chain=k, flags=flags)
for _ in range(2):
    e.compress_tensor(t)
torch.cuda.synchronize()
e.set_timing(True)   # mean ms per launch of each stage over the timed encodes
import time
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    e.compress_tensor(t)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 5
st, cnt = e.stage_times()
import hashlib
o, r = e.compress_tensor(t)
h = hashlib.sha1(o.cpu().numpy().tobytes()).hexdigest()[:16]
print({"config": f"{mb} MB K={k} {fs} {kind}{' wl=' + os.environ['DMX_WORKLIST'] if os.environ.get('DMX_WORKLIST') else ''}", "encodes": cnt, "GBps_wall": round(n / wall / 1e9, 2), "stage_ms": {a: round(b, 4) for a, b in st.items()},
       "out_len": int(r.out_len), "sha1": h})
e.close()
