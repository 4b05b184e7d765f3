"""deflate_compression_amd -- MI355X-native DEFLATE encoder (host mirror of the
reference's codec API, src/include/deflate_ext.h of mparker97/deflate_compression).

The compute path is libdmx.so (hand-written HIP kernels for gfx950 behind a C ABI,
include/dmx.h).  This module is a thin ctypes layer:

    deflate_compress(fd_in, fd_out, fd_stats=-1, sw=32768, ops=0) -> int
        deflate_ext.h:17 / deflate_compress.c:362 -- 0 or -E_* (no exceptions, like C)
    deflate_decompress(data, ops=0) -> bytes
        deflate_ext.h:16 -- raises DeflateError(code) on a negative return
    compress(data, sw=32768, max_chain=0) -> bytes        host buffer convenience
    Encoder                                               device-resident encodes

There is no CPU fallback: if libdmx.so is missing the import of this module fails,
and on a machine without an MI355X every encode fails with -E_NEXIST.
"""
from __future__ import annotations

import ctypes
import os
import struct

__all__ = [
    "DeflateError", "Opts", "Result", "Encoder", "lib", "compress", "deflate_compress",
    "deflate_decompress", "max_compressed", "adler32_combine", "gen_text", "gen_random",
    "COMPRESS_STATS", "E", "DMX_F_HEADER", "DMX_F_TRAILER", "DMX_F_FINAL", "DMX_ZLIB", "DMX_F_LAZY", "DMX_F_EXACT_SORT", "DMX_F_SPLIT", "DMX_F_DICT", "DMX_F_STORE_CHECK", "DMX_F_DEEP", "inflate_gpu", "inflate_gpu_chained", "ref_estimates",
]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdmx.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "dmx.h")

DEFLATE_NULLTERM = 1
DMX_F_HEADER, DMX_F_TRAILER, DMX_F_FINAL = 1, 2, 4
DMX_ZLIB = 7
DMX_F_LAZY = 8
DMX_F_EXACT_SORT = 16
DMX_F_SPLIT = 32
DMX_F_DICT = 64
DMX_F_STORE_CHECK = 128
DMX_F_DEEP = 256
_M = 1 << 24
# src/include/global_errors.h:24-35 and src/include/deflate_errors.h:9-22
E = {
    "E_LEN": 1, "E_MALLOC": 2, "E_FORK": 3, "E_PIPE": 4, "E_CRC": 5, "E_SZ": 6, "E_EXIST": 7,
    "E_NEXIST": 8, "E_NONULL": 9, "E_RANGE": 10, "E_INVAL": 11, "E_RESERV": 12,
    "E_HUFAMB": _M + 1, "E_HUFINV": _M + 2, "E_HUFVAL": _M + 3, "E_HUFDIS": _M + 4,
    "E_ZADL32": _M + 5, "E_ZHEAD": _M + 6, "E_ZFCHCK": _M + 7, "E_ZCMPMT": _M + 8,
    "E_ZSLWIN": _M + 9, "E_ZPDICT": _M + 10, "E_ZBSZ": _M + 11, "E_ZNLEN": _M + 12,
    "E_ZINV": _M + 13, "E_ZBTYPE": _M + 14, "E_DEVICE": _M + 64,
}
_ENAME = {v: k for k, v in E.items()}

# struct compress_stats (deflate_ext.h:19-31): six little-endian int32
COMPRESS_STATS = struct.Struct("<6i")


class DeflateError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what or 'dmx'} failed: -{_ENAME.get(-code, str(-code))} ({code})")


class Opts(ctypes.Structure):
    _fields_ = [("sw", ctypes.c_int32), ("max_chain", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("deep_chain", ctypes.c_int32), ("dict", ctypes.c_void_p), ("dict_len", ctypes.c_uint64)]


class Result(ctypes.Structure):
    _fields_ = [("out_len", ctypes.c_uint64), ("end_bits", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("ntokens", ctypes.c_uint64), ("adler", ctypes.c_uint32), ("status", ctypes.c_int32),
                ("nblocks", ctypes.c_uint32), ("nstored", ctypes.c_uint32), ("nfixed", ctypes.c_uint32),
                ("ndynamic", ctypes.c_uint32), ("nsortfallback", ctypes.c_uint32),
                ("nsortfallback_total", ctypes.c_uint32)]


class FdStats(ctypes.Structure):
    _fields_ = [("chunks", ctypes.c_uint64), ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64),
                ("wall_ms", ctypes.c_double), ("read_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("encode_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double), ("write_ms", ctypes.c_double)]


class _StringLen(ctypes.Structure):
    _fields_ = [("str", ctypes.POINTER(ctypes.c_ubyte)), ("len", ctypes.c_size_t)]


_lib = None
_libc = ctypes.CDLL(None)
_libc.free.argtypes = [ctypes.c_void_p]
_libc.free.restype = None


def lib() -> ctypes.CDLL:
    """Load libdmx.so (built by __graft_entry__.build() / `make -C deflate_compression_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                          "g.build()'` (the encoder has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    sig = {
        "deflate_compress": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_ushort, ctypes.c_int], ctypes.c_int),
        "deflate_decompress": ([ctypes.POINTER(_StringLen), ctypes.POINTER(_StringLen), ctypes.c_int], ctypes.c_int),
        "spawn_deflate_compr_t": ([], vp),
        "deflate_compr_init": ([vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_ushort], None),
        "deflate_compr_deinit": ([vp], None),
        "dmx_ctx_create": ([ctypes.c_int, u64, ctypes.POINTER(vp)], ctypes.c_int),
        "dmx_ctx_destroy": ([vp], None),
        "dmx_ctx_reserve": ([vp, u64, i32], ctypes.c_int),
        "dmx_ctx_reserve_flags": ([vp, u64, i32, u32], ctypes.c_int),
        "dmx_fault_set": ([ctypes.c_char_p], ctypes.c_int),
        "dmx_encode_fd_multi": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(Opts), u64,
                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
        "dmx_max_compressed": ([u64, i32], u64),
        "dmx_fd_last_stats": ([ctypes.POINTER(FdStats)], ctypes.c_int),
        "dmx_encode_async": ([vp, vp, u64, vp, u64, ctypes.POINTER(Opts), vp], ctypes.c_int),
        "dmx_encode_result": ([vp, ctypes.POINTER(Result), vp], ctypes.c_int),
        "dmx_encode_result_async": ([vp, vp, vp], ctypes.c_int),
        "dmx_encode_host": ([vp, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(Opts)], ctypes.c_int),
        "dmx_last_blocks": ([vp, u32p, u8p, u32p, u32], ctypes.c_int),
        "dmx_last_tokens": ([vp, u32, u32p, u32], ctypes.c_int),
        "dmx_last_code_lengths": ([vp, u32, u8p], ctypes.c_int),
        "dmx_last_subblock": ([vp, u32, u32, u32p, u32p, u32p, u8p], ctypes.c_int),
        "dmx_ctx_set_timing": ([vp, ctypes.c_int], ctypes.c_int),
        "dmx_ctx_set_hook": ([vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "dmx_ctx_stage_times": ([vp, ctypes.POINTER(ctypes.c_double), u32p], ctypes.c_int),
        "dmx_adler32_combine": ([u32, u32, u64], u32),
        "dmx_debug_stamps": ([vp, ctypes.POINTER(u64), u32], ctypes.c_int),
        "dmx_block_index": ([vp, vp, u32, vp], ctypes.c_int),
        "dmx_inflate_async": ([vp, u64, vp, u32, vp, u64, vp, vp], ctypes.c_int),
        "dmx_gen_text": ([vp, u64, u64], None),
        "dmx_gen_random": ([vp, u64, u64], None),
        "dmx_inflate_chained_async": ([vp, u64, vp, u32, vp, u64, vp, u64, vp, vp], ctypes.c_int),
        "dmx_inflate_chained_lists": ([vp, u32p, u32, vp], ctypes.c_int),
        "dmx_inflate_chained_work": ([u64, u32], u64),
        "dmx_refest_create": ([], vp),
        "dmx_refest_destroy": ([vp], None),
        "dmx_refest_feed": ([vp, u32p, u32, vp, u32p], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(r: int, what: str) -> None:
    if r != 0:
        raise DeflateError(r, what)


def _buf(data):
    """(ctypes pointer, length, keepalive) for bytes / bytearray / memoryview / numpy."""
    try:
        import numpy as np
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            return ctypes.c_void_p(a.ctypes.data), a.size, a
    except ImportError:  # pragma: no cover
        pass
    b = bytes(data)
    cb = ctypes.create_string_buffer(b, len(b) or 1)
    return ctypes.cast(cb, ctypes.c_void_p), len(b), cb


def fd_last_stats() -> dict | None:
    """Per-stage busy time of the last single-device fd-path call (dmx_fd_last_stats):
    wall, read, h2d, encode, d2h, write in ms, plus chunks and bytes; None before any."""
    st = FdStats()
    if lib().dmx_fd_last_stats(ctypes.byref(st)) != 0:
        return None
    return {k: (round(getattr(st, k), 3) if isinstance(getattr(st, k), float) else int(getattr(st, k)))
            for k, _ in FdStats._fields_}


def max_compressed(n: int, sw: int = 32768) -> int:
    return int(lib().dmx_max_compressed(n, sw))


def compress(data, sw: int = 32768, max_chain: int = 0, flags: int = DMX_ZLIB, lazy: bool = False,
             split: bool = False, dict: bool = False, pre=None, store_check: bool = False,
             deep: bool = False) -> bytes:
    """Encode a host buffer on the GPU; returns the zlib stream (or raw DEFLATE with flags).
    lazy = f2 lazy parse (DMX_F_LAZY), split = f3 adaptive block splitting (DMX_F_SPLIT),
    dict = f1 cross-block dictionary (DMX_F_DICT; pre = the bytes before `data`),
    store_check = noise blocks stored without a parse (DMX_F_STORE_CHECK),
    deep = adaptive chain depth of small-alphabet blocks (DMX_F_DEEP)."""
    L = lib()
    p, n, keep = _buf(data)
    cap = max_compressed(n, sw)
    out = ctypes.create_string_buffer(cap)
    olen = ctypes.c_uint64(0)
    o = Opts(sw, max_chain, flags | (DMX_F_LAZY if lazy else 0) | (DMX_F_SPLIT if split else 0) |
             (DMX_F_DICT if dict else 0) | (DMX_F_STORE_CHECK if store_check else 0) | (DMX_F_DEEP if deep else 0), 0)
    pk = None
    if dict and pre is not None and len(pre):
        pk = ctypes.create_string_buffer(bytes(pre), len(pre))
        o.dict, o.dict_len = ctypes.cast(pk, ctypes.c_void_p), len(pre)
    _check(L.dmx_encode_host(p, n, out, cap, ctypes.byref(olen), ctypes.byref(o)), "dmx_encode_host")
    del keep, pk
    return out.raw[:olen.value]


def deflate_compress(fd_in: int, fd_out: int, fd_stats: int = -1, sw: int = 32768, ops: int = 0) -> int:
    """deflate_ext.h:17 -- returns 0 or -E_* exactly like the C entry point."""
    return int(lib().deflate_compress(fd_in, fd_out, fd_stats, sw & 0xFFFF, ops))


def deflate_decompress(data, ops: int = 0) -> bytes:
    """deflate_ext.h:16 -- inflate a zlib stream; raises DeflateError on -E_*."""
    L = lib()
    b = bytes(data)
    src = (ctypes.c_ubyte * max(len(b), 1)).from_buffer_copy(b or b"\0")
    cin = _StringLen(ctypes.cast(src, ctypes.POINTER(ctypes.c_ubyte)), len(b))
    cout = _StringLen()
    r = L.deflate_decompress(ctypes.byref(cout), ctypes.byref(cin), ops)
    if r != 0:
        raise DeflateError(r, "deflate_decompress")
    n = cout.len + (1 if ops & DEFLATE_NULLTERM else 0)
    res = ctypes.string_at(cout.str, n)
    _libc.free(ctypes.cast(cout.str, ctypes.c_void_p))
    return res


def inflate_gpu(z, out_cap: int, index=None, nblk: int = 0, stream=None):
    """Inflate on the GPU (csrc/dmx_inflate_dev.hip).  z: uint8 CUDA tensor.  index=None:
    z is a whole zlib stream, decoded in one workgroup with the Adler-32 check.  index:
    the encoder's block index (Encoder.block_index), every block decoded in parallel.
    Returns (uint8 tensor of out_len bytes, status) -- status 0 or -E_*."""
    import numpy as np
    import torch
    L = lib()
    dev = z.device
    out = torch.empty(max(out_cap, 1), dtype=torch.uint8, device=dev)
    st = torch.zeros(16, dtype=torch.uint8, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    r = L.dmx_inflate_async(z.data_ptr(), z.numel(), index.data_ptr() if index is not None else None,
                            nblk, out.data_ptr(), out_cap, st.data_ptr(), s)
    _check(r, "dmx_inflate_async")
    torch.cuda.synchronize(dev)
    h = st.cpu().numpy()
    status = int(np.frombuffer(h[:4].tobytes(), np.int32)[0])
    olen = int(np.frombuffer(h[8:16].tobytes(), np.uint64)[0])
    return out[:olen], status


def inflate_gpu_chained(z, out_cap: int, index, nblk: int, stream=None, work=None):
    """Inflate on the GPU a stream whose blocks may reference the block before them
    (DMX_F_DICT streams), all blocks in parallel: each decodes into 16-bit cells with
    references for the bytes before it, then pointer jumping resolves the references
    (dmx_inflate_chained_async).  index: Encoder.block_index().  work: optional uint8 CUDA
    scratch of dmx_inflate_chained_work(out_cap, nblk) bytes.  Returns (uint8 tensor, status)."""
    import numpy as np
    import torch
    L = lib()
    dev = z.device
    out = torch.empty(max(out_cap, 1), dtype=torch.uint8, device=dev)
    st = torch.zeros(16, dtype=torch.uint8, device=dev)
    wb = int(L.dmx_inflate_chained_work(out_cap, nblk))
    if work is None or work.numel() < wb:
        work = torch.empty(wb + 256, dtype=torch.uint8, device=dev)
    wp = (work.data_ptr() + 255) & ~255
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    r = L.dmx_inflate_chained_async(z.data_ptr(), z.numel(), index.data_ptr(), nblk, out.data_ptr(), out_cap,
                                    wp, work.numel() - (wp - work.data_ptr()), st.data_ptr(), s)
    _check(r, "dmx_inflate_chained_async")
    torch.cuda.synchronize(dev)
    h = st.cpu().numpy()
    status = int(np.frombuffer(h[:4].tobytes(), np.int32)[0])
    olen = int(np.frombuffer(h[8:16].tobytes(), np.uint64)[0])
    return out[:olen], status


def fault_set(spec: str | None) -> int:
    """Fault injection (tests): "malloc:N" / "launch:N" / None (dmx_fault_set)."""
    return int(lib().dmx_fault_set(spec.encode() if spec else None))


def ref_estimates(tokens, state=None):
    """The reference's estimate fields (tree_bits, ll_bits, d_bits) of every token's
    compress_stats record (deflate_compress.c:290-298), from libdmx's host restatement of its
    adaptive Huffman trees (csrc/dmx_refstats.c).  tokens: uint32 (byte | dist << 9 | len) in
    stream order.  Returns int32[ntok, 3].  Pure host code: no GPU needed."""
    import numpy as np
    t = np.ascontiguousarray(tokens, dtype=np.uint32)
    L = lib()
    e = L.dmx_refest_create() if state is None else state
    rec = np.zeros((t.size, 6), dtype=np.int32)
    nf = ctypes.c_uint32(0)
    try:
        r = L.dmx_refest_feed(e, t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), t.size,
                              ctypes.c_void_p(rec.ctypes.data), ctypes.byref(nf))
    finally:
        if state is None:
            L.dmx_refest_destroy(e)
    _check(r, "dmx_refest_feed")
    return rec[:, 1:4].copy()


def adler32_combine(a: int, b: int, len_b: int) -> int:
    return int(lib().dmx_adler32_combine(a, b, len_b))


def gen_text(n: int, seed: int = 0xE5818):
    import numpy as np
    a = np.empty(n, dtype=np.uint8)
    lib().dmx_gen_text(ctypes.c_void_p(a.ctypes.data), n, seed)
    return a


def gen_random(n: int, seed: int = 0x5EED):
    import numpy as np
    a = np.empty(n, dtype=np.uint8)
    lib().dmx_gen_random(ctypes.c_void_p(a.ctypes.data), n, seed)
    return a


class Encoder:
    """Device-resident encoder on one GPU (a dmx_ctx: own HIP stream + HBM workspace).

    encode_async(d_in, n, d_out, cap, stream=None) takes raw device pointers (ints),
    e.g. torch tensors' .data_ptr(); nothing is allocated or synchronised per call.
    """

    def __init__(self, device: int = 0, max_input: int = 1 << 20, sw: int = 32768, max_chain: int = 0,
                 flags: int = DMX_ZLIB):
        self._L = lib()
        self.device = device
        self.opts = Opts(sw, max_chain, flags, 0)
        self._ctx = ctypes.c_void_p()
        _check(self._L.dmx_ctx_create(device, max_input, ctypes.byref(self._ctx)), "dmx_ctx_create")
        if flags & (DMX_F_SPLIT | DMX_F_DICT):   # the block options' scratch (no allocation per encode)
            try:
                self.reserve(max_input, sw, flags)
            except DeflateError:
                self.close()
                raise

    def close(self) -> None:
        if self._ctx:
            self._L.dmx_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, n: int, sw: int = 32768, flags: int = 0) -> None:
        """Workspace for n bytes of sw-byte blocks, plus the scratch of DMX_F_SPLIT / DMX_F_DICT
        (dmx_ctx_reserve_flags; synchronises only when it allocates)."""
        _check(self._L.dmx_ctx_reserve_flags(self._ctx, n, sw, flags), "dmx_ctx_reserve_flags")

    def encode_async(self, d_in: int, n: int, d_out: int, cap: int, stream: int | None = None,
                     opts: Opts | None = None) -> None:
        o = opts or self.opts
        _check(self._L.dmx_encode_async(self._ctx, ctypes.c_void_p(d_in), n, ctypes.c_void_p(d_out), cap,
                                        ctypes.byref(o), ctypes.c_void_p(stream or 0)), "dmx_encode_async")

    def result(self, stream: int | None = None) -> Result:
        r = Result()
        _check(self._L.dmx_encode_result(self._ctx, ctypes.byref(r), ctypes.c_void_p(stream or 0)),
               "dmx_encode_result")
        if r.status:
            raise DeflateError(r.status, "encode")
        return r

    def result_async(self, host_ptr: int, stream: int | None = None) -> None:
        """Enqueue the D2H copy of the last encode's 64 B dmx_result into host_ptr (pinned
        memory, e.g. a pin_memory uint8 tensor); read it after the stream or an event."""
        _check(self._L.dmx_encode_result_async(self._ctx, ctypes.c_void_p(host_ptr), ctypes.c_void_p(stream or 0)),
               "dmx_encode_result_async")

    # -- introspection of the last encode (tests / stats) --
    def blocks(self, nblk: int):
        import numpy as np
        nt = np.zeros(nblk, np.uint32)
        bt = np.zeros(nblk, np.uint8)
        hb = np.zeros(nblk, np.uint32)
        r = self._L.dmx_last_blocks(self._ctx, nt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    bt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                    hb.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), nblk)
        if r < 0:
            raise DeflateError(r, "dmx_last_blocks")
        return nt[:r], bt[:r], hb[:r]

    def tokens(self, blk: int):
        import numpy as np
        t = np.zeros(32768, np.uint32)
        r = self._L.dmx_last_tokens(self._ctx, blk, t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 32768)
        if r < 0:
            raise DeflateError(r, "dmx_last_tokens")
        return t[:r].copy()

    def code_lengths(self, blk: int):
        import numpy as np
        ln = np.zeros(316, np.uint8)
        _check(self._L.dmx_last_code_lengths(self._ctx, blk, ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))),
               "dmx_last_code_lengths")
        return ln

    def subblocks(self, blk: int):
        """DEFLATE blocks of sw block `blk` in the last encode (f3 split: up to 4):
        list of (t0, t1, btype, hdr_bits, code lengths[316])."""
        import numpy as np
        out = []
        nsub, k = 1, 0
        while k < nsub:
            rg = np.zeros(2, np.uint32)
            bt = np.zeros(1, np.uint32)
            hb = np.zeros(1, np.uint32)
            ln = np.zeros(316, np.uint8)
            P = ctypes.POINTER(ctypes.c_uint32)
            nsub = self._L.dmx_last_subblock(self._ctx, blk, k, rg.ctypes.data_as(P), bt.ctypes.data_as(P),
                                             hb.ctypes.data_as(P), ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
            if nsub < 0:
                raise DeflateError(nsub, "dmx_last_subblock")
            out.append((int(rg[0]), int(rg[1]), int(bt[0]), int(hb[0]), ln))
            k += 1
        return out

    def stamps(self, nblk: int):
        """[nblk, 16] match-kernel phase cycles (needs DMX_STAMPS=1): P0, search, walk+compaction,
        deferred extension, search steps, W1, W1-W3, total, then P0 sub-phase ends (staged,
        pass 1, pass 2) relative to the kernel start."""
        import numpy as np
        a = np.zeros((nblk, 16), np.uint64)
        _check(self._L.dmx_debug_stamps(self._ctx, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nblk),
               "dmx_debug_stamps")
        return a

    def block_index(self, stream=None):
        """Device block index of the last encode (uint8 tensor of nblk x 24 B dmx_iblock
        records) for inflate_gpu's parallel mode."""
        import torch
        n = self.last_nblk()
        ix = torch.empty(max(n, 1) * 24, dtype=torch.uint8, device=f"cuda:{self.device}")
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        r = self._L.dmx_block_index(self._ctx, ix.data_ptr(), n, s)
        if r < 0:
            raise DeflateError(r, "dmx_block_index")
        return ix, n

    def last_nblk(self) -> int:
        return int(self._L.dmx_last_blocks(self._ctx, None, None, None, 1 << 30))

    STAGES = ("pre", "match", "huff", "scan", "pack")

    HOOKS = {"worklist": 1, "dedupe": 2, "scan3": 3}   # DMX_HOOK_* (include/dmx.h)
    WORKLIST = {None: -1, "0": 0, "list": 1, "plain": 2}

    def set_hook(self, name: str, value) -> None:
        """Test hooks of this context (dmx_ctx_set_hook): "worklist" None (adaptive) / "0" /
        "list" / "plain"; "dedupe" None / 0 / 1; "scan3" 0 / 1.  Every setting must give the
        same stream; they pick launch shapes only."""
        if name == "worklist":
            v = self.WORKLIST[value]
        elif name == "dedupe":
            v = -1 if value is None else int(value)
        else:
            v = int(value)
        _check(self._L.dmx_ctx_set_hook(self._ctx, self.HOOKS[name], v), "dmx_ctx_set_hook")

    def set_timing(self, on: bool, stage: str | None = None, every: int = 1) -> None:
        """HIP-event stage times of the following encodes: every stage boundary, or with
        `stage` only that stage's two events (a timed loop then pays two event records per
        encode; the other stages read 0), on every `every`-th encode (1..255)."""
        if not 1 <= every <= 255:
            raise ValueError("every must be 1..255")
        mode = 0 if not on else (1 if stage is None else 0x100 | self.STAGES.index(stage) | (every << 12))
        self._L.dmx_ctx_set_timing(self._ctx, mode)

    def stage_times(self):
        ms = (ctypes.c_double * 6)()
        cnt = ctypes.c_uint32(0)
        self._L.dmx_ctx_stage_times(self._ctx, ms, ctypes.byref(cnt))
        return {k: v for k, v in zip(["pre", "match", "huff", "scan", "pack", "total"], list(ms))}, cnt.value

    # -- host convenience on this context via torch tensors --
    def compress_tensor(self, t_in, stream=None, opts: Opts | None = None):
        """Encode a uint8 CUDA tensor; returns (uint8 CUDA tensor of the stream, Result)."""
        import torch
        o = opts or self.opts
        n = t_in.numel()
        self.reserve(n, o.sw, o.flags)
        cap = max_compressed(n, o.sw)
        out = torch.empty(cap, dtype=torch.uint8, device=t_in.device)
        s = stream if stream is not None else torch.cuda.current_stream(t_in.device).cuda_stream
        self.encode_async(t_in.data_ptr() if n else out.data_ptr(), n, out.data_ptr(), cap, s, o)
        r = self.result(s)
        return out[:r.out_len], r

    def compress_bytes(self, data, sw: int = 32768, max_chain: int = 0, flags: int = DMX_ZLIB, pre=None):
        """Host bytes -> HBM -> encode -> host bytes, on this context (keeps introspection).
        pre: DMX_F_DICT history of block 0 (host bytes, staged in HBM here)."""
        import numpy as np
        import torch
        dev = f"cuda:{self.device}"
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        t = torch.from_numpy(a.copy()).to(dev) if a.size else torch.empty(0, dtype=torch.uint8, device=dev)
        self.reserve(a.size, sw, flags)
        o = Opts(sw, max_chain, flags, 0)
        if pre is not None and len(pre):
            tp = torch.from_numpy(np.frombuffer(bytes(pre), dtype=np.uint8).copy()).to(dev)
            o.dict, o.dict_len = tp.data_ptr(), tp.numel()
        out, r = self.compress_tensor(t, opts=o)
        return out.cpu().numpy().tobytes(), r
