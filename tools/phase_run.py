"""Diagnostic: one text encode on cuda:0 for per-phase SQ counters of the match kernel.
Run under rocprofv3 --pmc with DMX_LIBV = a -DDMX_DEBUG_STOP=1|2|3 library variant (end
blocks after P0 / P1 / P2; the stream is then not the input's) or unset (the whole kernel).  usage: phase_run.py [MB] [K] [lazy] [dict]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import deflate_compression_amd as D

if os.environ.get("DMX_LIBV"):
    D.LIB_PATH = os.environ["DMX_LIBV"]

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 20
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
lazy = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dct = int(sys.argv[4]) if len(sys.argv) > 4 else 0
n = int(mb * 1e6)
t = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
e = D.Encoder(0, n, max_chain=k, flags=D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0) | (D.DMX_F_DICT if dct else 0))
for _ in range(2):
    out, r = e.compress_tensor(t)
torch.cuda.synchronize()
print(f"lib={os.path.basename(D.LIB_PATH)} blocks={r.nblocks} out={r.out_len}")
e.close()
