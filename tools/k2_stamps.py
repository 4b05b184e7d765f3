"""Diagnostic: K2 (dmx_huff_kernel) phase cycles per block from a -DDMX_K2_STAMPS build
(build/var/libdmx_k2st.so).  python tools/k2_stamps.py [MB]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deflate_compression_amd as D  # noqa: E402

D.LIB_PATH = os.environ.get("DMX_LIBV", os.path.join(os.path.dirname(D.LIB_PATH), "..", "build", "var",
                                                      "libdmx_k2st.so"))
import torch  # noqa: E402


def main():
    n = int(sys.argv[1] if len(sys.argv) > 1 else 20) * 1_000_000
    t = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    e = D.Encoder(0, n, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_DEEP)
    e.compress_tensor(t)
    st = (ctypes.c_ulonglong * 16)()
    L = D.lib()
    L.dmx_k2_stamps(st, 1)
    e.compress_tensor(t)
    torch.cuda.synchronize()
    L.dmx_k2_stamps(st, 1)
    e.close()
    v = list(st)
    nb = max(v[7], 1)
    names = ["rank", "merge", "depth+len", "canon", "rle", "header", "total", None, "load", "plan", "emit"]
    print({k: round(v[i] / nb / 1e3, 1) for i, k in enumerate(names) if k}, "K cycles per block over", nb, "blocks")


if __name__ == "__main__":
    main()
