"""Diagnostic: per-phase cycle totals of the indexed GPU inflate (a DMX_INF_STAMPS build).
usage: DMX_LIBV=deflate_compression_amd/libdmx_st.so python3 tools/inf_stamps.py [MB]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import deflate_compression_amd as D

D.LIB_PATH = os.environ["DMX_LIBV"]
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 100
n = mb * 1_000_000
data = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
enc = D.Encoder(0, n, max_chain=7, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_DEEP)
out, r = enc.compress_tensor(data)
ix, nb = enc.block_index()
L = D.lib()
L.dmx_inflate_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
s = torch.cuda.current_stream()
dec = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.zeros(16, dtype=torch.uint8, device="cuda")
for _ in range(2):
    assert L.dmx_inflate_async(out.data_ptr(), out.numel(), ix.data_ptr(), nb, dec.data_ptr(), n, st.data_ptr(),
                               s.cuda_stream) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
assert L.dmx_inflate_async(out.data_ptr(), out.numel(), ix.data_ptr(), nb, dec.data_ptr(), n, st.data_ptr(),
                           s.cuda_stream) == 0
e1.record(s)
torch.cuda.synchronize()
a = np.zeros((nb, 16), np.uint64)
assert L.dmx_inflate_stamps(a.ctypes.data, a.nbytes) == 0
a = a.astype(np.float64)
tot = a[:, 0] + a[:, 1]
print(json.dumps({"lib": os.path.basename(D.LIB_PATH), "ms": round(e0.elapsed_time(e1), 3),
                  "bit_exact": bool(torch.equal(dec, data)), "blocks": nb,
                  "hdr_tables_kcyc": round(a[:, 0].mean() / 1e3, 1), "symbols_kcyc": round(a[:, 1].mean() / 1e3, 1),
                  "flush_kcyc": round(a[:, 2].mean() / 1e3, 1), "cpp_path_matches": round(a[:, 3].mean(), 1),
                  "cpp_path_far": round(a[:, 4].mean(), 1), "deflate_blocks": round(a[:, 6].mean(), 2),
                  "cl_table_kcyc": round(a[:, 7].mean() / 1e3, 1),
                  "header_to_ll_table_kcyc": round(a[:, 8].mean() / 1e3, 1),
                  "ll_table_kcyc": round(a[:, 9].mean() / 1e3, 1), "dist_table_kcyc": round(a[:, 10].mean() / 1e3, 1),
                  "asm_runs": round(a[:, 5].mean(), 1),
                  "exits": {k: round(a[:, 11 + j].mean(), 1) for j, k in enumerate(["sym", "seg", "lim", "dist", "match"])},
                  "total_kcyc_max": round(tot.max() / 1e3, 1)}))
enc.close()
