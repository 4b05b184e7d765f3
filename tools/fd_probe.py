"""Host-side rates that bound the drop-in fd path (diagnostic): page-cache reads into pinned
memory with T threads, H2D / D2H over PCIe, and writes of the stream to a file.
    python tools/fd_probe.py [MB]"""
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch


def par(fn, n, T):
    piece = (n + T - 1) // T
    th = [threading.Thread(target=fn, args=(k * piece, min(n, (k + 1) * piece))) for k in range(T) if k * piece < n]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return time.perf_counter() - t0


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    where = sys.argv[2] if len(sys.argv) > 2 else "/tmp"
    n = mb * 1_000_000
    td = tempfile.mkdtemp(dir=where)
    fi = os.path.join(td, "in")
    np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8).tofile(fi)
    pin = torch.empty(n, dtype=torch.uint8).pin_memory()
    mv = memoryview(pin.numpy())
    fd = os.open(fi, os.O_RDONLY)
    res = {}
    for T in (1, 2, 4, 8, 16):
        def rd(lo, hi):
            o = lo
            while o < hi:
                k = os.preadv(fd, [mv[o:hi]], o)
                if k <= 0:
                    break
                o += k
        dt = min(par(rd, n, T) for _ in range(3))
        res[f"pread_T{T}"] = round(n / dt / 1e9, 2)
    os.close(fd)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()
        h2d = time.perf_counter() - t0
        t0 = time.perf_counter()
        pin.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
        d2h = time.perf_counter() - t0
    res["h2d"] = round(n / h2d / 1e9, 2)
    res["d2h"] = round(n / d2h / 1e9, 2)
    fo = os.path.join(td, "out")
    m = int(n * 0.45)
    for T in (1, 4, 8):
        fdo = os.open(fo, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)

        def wr(lo, hi):
            o = lo
            while o < hi:
                o += os.pwritev(fdo, [mv[o:hi]], o)
        dt = par(wr, m, T)
        os.close(fdo)
        res[f"pwrite_T{T}"] = round(m / dt / 1e9, 2)
    # the output through a shared mapping of the file (ftruncate + mmap), T threads copying
    import ctypes
    import mmap
    src = torch.from_numpy(pin.numpy()[:m])
    for T in (1, 4, 8, 16):
        fdo = os.open(fo, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
        t0 = time.perf_counter()
        os.ftruncate(fdo, m)
        mm = mmap.mmap(fdo, m, mmap.MAP_SHARED, mmap.PROT_WRITE | mmap.PROT_READ)
        dst = torch.from_numpy(np.frombuffer(mm, dtype=np.uint8))

        def cp(lo, hi):
            dst[lo:hi].copy_(src[lo:hi])
        par(cp, m, T)
        del dst
        mm.close()
        os.close(fdo)
        res[f"mmap_write_T{T}"] = round(m / (time.perf_counter() - t0) / 1e9, 2)
    # D2H straight into the mapped file pages (hipHostRegister of the mapping)
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        fdo = os.open(fo, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
        t0 = time.perf_counter()
        os.ftruncate(fdo, m)
        mm = mmap.mmap(fdo, m, mmap.MAP_SHARED, mmap.PROT_WRITE | mmap.PROT_READ)
        buf = (ctypes.c_char * m).from_buffer(mm)
        ptr = ctypes.addressof(buf)
        t1 = time.perf_counter()
        rc = hip.hipHostRegister(ctypes.c_void_p(ptr), ctypes.c_size_t(m), 0)
        t2 = time.perf_counter()
        rc2 = hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(m), 2)
        t3 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(ptr))
        t4 = time.perf_counter()
        del buf
        mm.close()
        os.close(fdo)
        res["reg_d2h"] = {"rc": (rc, rc2), "map_ms": round((t1 - t0) * 1e3, 2), "register_ms": round((t2 - t1) * 1e3, 2),
                          "d2h_ms": round((t3 - t2) * 1e3, 2), "unregister_ms": round((t4 - t3) * 1e3, 2),
                          "GBps_total": round(m / (t4 - t0) / 1e9, 2)}
    except Exception as e:  # pragma: no cover
        res["reg_d2h"] = repr(e)
    print("fs of", where, ":", os.popen("stat -f -c %T " + where).read().strip())
    os.remove(fi)
    os.remove(fo)
    os.rmdir(td)
    print(res)


if __name__ == "__main__":
    main()
