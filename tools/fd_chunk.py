"""Diagnostic: the drop-in fd path into /dev/null (bench.py's end_to_end sink_devnull leg; with
FD_SINK_FILE=1 into a file next to the input) at several DMX_CHUNK_MB values, with the bench's
parse settings; best of 5 per chunk size.
    python tools/fd_chunk.py [MB] [chunk_mb ...]"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deflate_compression_amd as D

if os.environ.get("DMX_LIBV"):   # a variant built beside libdmx.so (tools/build_var.sh)
    D.LIB_PATH = os.environ["DMX_LIBV"]


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 100
    chunks = [int(x) for x in sys.argv[2:]] or [4, 8, 12, 16, 24, 32]
    n = int(mb * 1e6)
    os.environ.update({"DMX_MAX_CHAIN": "7", "DMX_LAZY": "1", "DMX_SPLIT": "0", "DMX_DICT": "0",
                       "DMX_STORE_CHECK": "1", "DMX_DEEP": "1"})
    host = D.gen_text(n, 0xE5818)
    td = tempfile.mkdtemp(dir="/tmp")
    fi = os.path.join(td, "in")
    host.tofile(fi)
    try:
        for cm in chunks:
            os.environ["DMX_CHUNK_MB"] = str(cm)
            best, st = None, None
            for _ in range(5):
                a = os.open(fi, os.O_RDONLY)
                b = os.open(os.devnull, os.O_WRONLY) if not os.environ.get("FD_SINK_FILE") else \
                    os.open(os.path.join(td, "out"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                t0 = time.perf_counter()
                rc = D.deflate_compress(a, b, -1, 32768, 0)
                t1 = time.perf_counter()
                os.close(a)
                os.close(b)
                assert rc == 0, rc
                if best is None or t1 - t0 < best:
                    best, st = t1 - t0, D.fd_last_stats()
            print(json.dumps({"lib": os.path.basename(D.LIB_PATH), "chunk_mb": cm, "GBps": round(n / best / 1e9, 3), "ms": round(best * 1e3, 3),
                              "stages": st}), flush=True)
    finally:
        for f in os.listdir(td):
            os.remove(os.path.join(td, f))
        os.rmdir(td)


if __name__ == "__main__":
    main()
