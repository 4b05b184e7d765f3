"""Diagnostic: exhaustive-parse tokens of the GPU vs the oracle at several block sizes."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import deflate_compression_amd as D
from oracle import oracle as O
text = D.gen_text(120000, 17).tobytes()
for sw, n, fl in [(w, 20000, 0) for w in (300, 500, 999, 1000, 1001, 1024, 1500, 3000, 5000)]:
    data = text[:n]
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = D.Encoder(0, 1 << 20)
    out, r = enc.compress_tensor(t, opts=D.Opts(sw, 0, D.DMX_ZLIB | fl, 0))
    a = np.frombuffer(data, np.uint8)
    bad = []
    for b in range(r.nblocks):
        g = enc.tokens(b)
        o = O.parse_block(a[b*sw:(b+1)*sw], 0)
        if not np.array_equal(g, o):
            bad.append(b)
    print("sw", sw, "exact" if fl else "", "bad blocks", bad, "of", r.nblocks)
    enc.close()
