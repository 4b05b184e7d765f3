"""GPU encode rate of small-alphabet inputs at several chain depths (DMX_F_DEEP's cost).
    python tools/deep_bench.py [MB]"""
import binascii
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import deflate_compression_amd as D  # noqa: E402
from tests.deep_inputs import bitdump  # noqa: E402

if os.environ.get("DMX_LIBV"):   # a variant built beside libdmx.so (tools/build_var.sh)
    D.LIB_PATH = os.environ["DMX_LIBV"]


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    n = mb << 20
    rng = np.random.default_rng(3)
    text = D.gen_text(n, 0xE5818).tobytes()
    ins = {"text": text, "bitdump": bitdump(n, 4), "hex": binascii.hexlify(text[:n // 2]),
           "dna": rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()}
    stream = torch.cuda.current_stream().cuda_stream
    for name, data in ins.items():
        a = np.frombuffer(data, dtype=np.uint8)
        d_in = torch.from_numpy(a.copy()).cuda()
        cap = D.max_compressed(a.size)
        d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        row = []
        # (K, DMX_F_DEEP, deep_chain): the bench's K=7 alone, and with the adaptive depth at
        # the depths VERDICT r4 #6 asks for
        cfgs = [(7, 0, 0)] + [(7, D.DMX_F_DEEP, dk) for dk in (16, 24, 32, 64)]
        for k, fl, dk in cfgs:
            e = D.Encoder(0, a.size, 32768, k, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | fl)
            e.opts.deep_chain = dk
            e.encode_async(d_in.data_ptr(), a.size, d_out.data_ptr(), cap, stream)
            ln = int(e.result(stream).out_len)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                e.encode_async(d_in.data_ptr(), a.size, d_out.data_ptr(), cap, stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            e.close()
            row.append(f"K={k}{f'+deep{dk}' if fl else ''}: {a.size / dt / 1e9:7.2f} GB/s ratio {ln / a.size:.4f}")
        print(f"{name:8s} " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
