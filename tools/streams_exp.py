"""Experiment: consecutive encodes on 1 vs 2 HIP streams (two contexts, two output buffers),
so one encode's Huffman/scan/pack can overlap the next one's match kernel."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import deflate_compression_amd as D
n = 100_000_000
host = D.gen_text(n, 0xE5818)
dev = torch.device("cuda:0")
d_in = torch.from_numpy(host).to(dev)
cap = D.max_compressed(n)
fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
for ns in (1, 2, 3):
    encs = [D.Encoder(0, n, 32768, 8, fl) for _ in range(ns)]
    outs = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(ns)]
    strs = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    def run(k):
        for i in range(k):
            j = i % ns
            encs[j].encode_async(d_in.data_ptr(), n, outs[j].data_ptr(), cap, strs[j].cuda_stream)
    run(2 * ns)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); run(30); torch.cuda.synchronize(); t1 = time.perf_counter()
    z = [outs[j][:int(encs[j].result(strs[j].cuda_stream).out_len)].cpu().numpy().tobytes() for j in range(ns)]
    print(ns, "streams:", round(n * 30 / (t1 - t0) / 1e9, 2), "GB/s", "same" if all(x == z[0] for x in z) else "DIFF", flush=True)
    for e in encs: e.close()
