"""Diagnostic: the cost of a wrong launch-shape hint.  The work-list
shapes of an encode follow the previous encode on the same context; after a
switch from noise to text (or back) the first encode runs with the other input's shapes.
One context alternates inputs; every encode is timed alone with HIP events on its stream,
and the first encode after each switch is reported against the steady state of that input.
usage: hint_switch.py [text_MB] [noise_MB] [reps]   (defaults: 100 MB C3 text, 1 GiB C4 noise;
and 16 MiB chunks of each, the fd path's chunk size)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import deflate_compression_amd as D

if os.environ.get("DMX_LIBV"):
    D.LIB_PATH = os.environ["DMX_LIBV"]

tmb = float(sys.argv[1]) if len(sys.argv) > 1 else 100
nmb = float(sys.argv[2]) if len(sys.argv) > 2 else 1073.741824
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP


def run(sizes):
    nt, nn = sizes
    text = torch.from_numpy(D.gen_text(nt, 0xE5818)).cuda()
    noise = torch.from_numpy(D.gen_random(nn, 0x5EED)).cuda()
    n = max(nt, nn)
    cap = D.max_compressed(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    e = D.Encoder(0, n, max_chain=7, flags=fl)
    s = torch.cuda.Stream()   # (a stream of its own: handle 0 would mean the context's stream to the encoder)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def once(t):
        ev[0].record(s)
        e.encode_async(t.data_ptr(), t.numel(), out.data_ptr(), cap, s.cuda_stream)
        ev[1].record(s)
        ev[1].synchronize()
        r = e.result(s.cuda_stream)
        assert r.status == 0
        return ev[0].elapsed_time(ev[1])

    for t in (text, noise, text):   # warm both inputs' kernels
        once(t)
    res = {}
    for name, a, b in (("noise->text", noise, text), ("text->noise", text, noise)):
        firsts, steady = [], []
        for _ in range(reps):
            for _ in range(3):
                once(a)   # the context's hint is now a's
            firsts.append(once(b))   # b with a's shapes
            steady += [once(b) for _ in range(3)]   # b with its own
        st = sorted(steady)[len(steady) // 2]
        fm = sorted(firsts)[len(firsts) // 2]
        res[name] = {"first_ms_median": round(fm, 4), "steady_ms_median": round(st, 4),
                     "first_over_steady": round(fm / st, 3), "firsts_ms": [round(x, 4) for x in firsts]}
    e.close()
    return {"text_bytes": nt, "noise_bytes": nn, **res}


out = {"whole": run((int(tmb * 1e6), int(nmb * 1e6))), "chunks_16MiB": run((16 << 20, 16 << 20))}
print(json.dumps(out), flush=True)
