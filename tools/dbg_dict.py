import sys, numpy as np
sys.path.insert(0, '/root/repo')
import deflate_compression_amd as D
import os
if os.environ.get("DMX_LIBV"): D.LIB_PATH = os.environ["DMX_LIBV"]
from oracle import oracle as O
import torch
text = D.gen_text(300000, 21).tobytes()
e = D.Encoder(0, 8 << 20)
for K in (0, 1, 8):
    for lazy in (False, True):
        fl = D.DMX_ZLIB | D.DMX_F_DICT | (D.DMX_F_LAZY if lazy else 0)
        z, r = e.compress_bytes(text, max_chain=K, flags=fl)
        ref = O.parse(text, max_chain=K, lazy=lazy, dict=True)
        bad = [b for b in range(len(ref)) if not np.array_equal(e.tokens(b), ref[b])]
        print(K, lazy, "bad blocks", bad[:10])
        if bad:
            b = bad[0]; g = e.tokens(b); o = ref[b]
            m = min(len(g), len(o)); d = np.nonzero(g[:m] != o[:m])[0]
            k = int(d[0]) if len(d) else m
            pos = int(sum(1 if (t >> 9) == 0 else (t & 0x1FF) for t in o[:k]))
            print("  first diff tok", k, "pos", pos, "gpu", [(int(t)>>9, int(t)&0x1FF) for t in g[k:k+3]], "ora", [(int(t)>>9, int(t)&0x1FF) for t in o[k:k+3]])
