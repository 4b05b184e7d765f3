"""GPU inflate throughput: indexed parallel mode on the bench workload
(C3 text, 100 MB, K=8 lazy) and single-workgroup stream mode on a zlib-6 stream.

Prints one JSON line.  Output bytes / kernel time, inputs resident in HBM, timed with
events on the launch stream over K back-to-back launches.
"""
import argparse
import json
import os
import sys
import zlib

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deflate_compression_amd as D
if os.environ.get("DMX_LIB"):   # a variant build (tools/inflate_variants.sh)
    D.LIB_PATH = os.environ["DMX_LIB"]


def _time(fn, k, stream):
    s = torch.cuda.Stream(stream=stream) if isinstance(stream, int) else stream
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(k):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=100)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--stream-mb", type=int, default=4)
    ap.add_argument("--chained", type=int, default=0, help="1: a DMX_F_DICT stream, the chained decode")
    a = ap.parse_args()
    if a.chained:
        return chained(a)
    n = a.mb * 1_000_000
    data = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    enc = D.Encoder(0, n, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    out, r = enc.compress_tensor(data)
    ix, nb = enc.block_index()
    L = D.lib()
    s = torch.cuda.current_stream()
    dec = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(16, dtype=torch.uint8, device="cuda")

    def idx():
        rc = L.dmx_inflate_async(out.data_ptr(), out.numel(), ix.data_ptr(), nb, dec.data_ptr(), n,
                                 st.data_ptr(), s.cuda_stream)
        assert rc == 0

    ms = _time(idx, a.steps, s)
    ok_idx = torch.equal(dec, data)

    m = a.stream_mb * 1_000_000
    raw = data[:m].cpu().numpy().tobytes()
    z = torch.frombuffer(bytearray(zlib.compress(raw, 6)), dtype=torch.uint8).cuda()
    dec2 = torch.empty(m, dtype=torch.uint8, device="cuda")

    def strm():
        rc = L.dmx_inflate_async(z.data_ptr(), z.numel(), None, 0, dec2.data_ptr(), m,
                                 st.data_ptr(), s.cuda_stream)
        assert rc == 0

    ms2 = _time(strm, 2, s)
    ok_strm = torch.equal(dec2, data[:m])
    enc.close()
    print(json.dumps({
        "indexed": {"bytes_out": n, "bytes_in": int(out.numel()), "blocks": nb, "ms": round(ms, 4),
                    "GBps_out": round(n / ms / 1e6, 2), "bit_exact": ok_idx},
        "stream_zlib6": {"bytes_out": m, "ms": round(ms2, 3), "GBps_out": round(m / ms2 / 1e6, 4),
                         "bit_exact": ok_strm},
    }))


def chained(a):
    """The chained decode of a dictionary stream (K=6 lazy, DMX_F_DICT): output bytes / time."""
    n = a.mb * 1_000_000
    data = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    enc = D.Encoder(0, n, max_chain=6, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_DICT)
    out, r = enc.compress_tensor(data)
    ix, nb = enc.block_index()
    L = D.lib()
    s = torch.cuda.current_stream()
    dec = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(16, dtype=torch.uint8, device="cuda")
    wb = int(L.dmx_inflate_chained_work(n, nb))
    work = torch.empty(wb + 256, dtype=torch.uint8, device="cuda")
    wptr = (work.data_ptr() + 255) & ~255

    def run():
        rc = L.dmx_inflate_chained_async(out.data_ptr(), out.numel(), ix.data_ptr(), nb, dec.data_ptr(), n, wptr, wb,
                                         st.data_ptr(), s.cuda_stream)
        assert rc == 0

    ms = _time(run, a.steps, s)
    ok = torch.equal(dec, data) and int(st[:4].view(torch.int32).item()) == 0
    enc.close()
    print(json.dumps({"chained": {"bytes_out": n, "blocks": nb, "ms": round(ms, 4), "GBps_out": round(n / ms / 1e6, 2),
                                  "bit_exact": ok}}))


if __name__ == "__main__":
    main()
