"""ctypes bindings for the CPU oracle (oracle/dmx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  Never imported by deflate_compression_amd/.

Also drives oracle/_ref/ref_tokens (the reference encoder compiled from
/root/reference by Makefile.ref) when it exists -- only in the build container.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_tokens")

HASH_MUL = 0
HASH_MORTON = 1

_lib = None


def build() -> None:
    """Compile liboracle.so (gcc); idempotent."""
    src = os.path.join(HERE, "dmx_oracle.c")
    if os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= os.path.getmtime(src):
        return
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.dmx_oracle_parse_block_ex.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p]
        L.dmx_oracle_parse_block_ex.restype = ctypes.c_int
        L.dmx_oracle_huff_lengths.argtypes = [u32p, ctypes.c_int, ctypes.c_int, u8p]
        L.dmx_oracle_huff_lengths.restype = ctypes.c_int
        L.dmx_oracle_adler32.argtypes = [u8p, ctypes.c_size_t]
        L.dmx_oracle_adler32.restype = ctypes.c_uint32
        L.dmx_oracle_compress_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t, u8p]
        L.dmx_oracle_compress_ex.restype = ctypes.c_longlong
        L.dmx_oracle_compress_ex2.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t, u8p]
        L.dmx_oracle_compress_ex2.restype = ctypes.c_longlong
        L.dmx_oracle_compress_ex3.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t,
                                              u8p, ctypes.c_size_t, u8p]
        L.dmx_oracle_compress_ex3.restype = ctypes.c_longlong
        L.dmx_oracle_compress_framed.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t,
                                                 ctypes.c_int, u8p, ctypes.c_size_t, u8p]
        L.dmx_oracle_compress_framed.restype = ctypes.c_longlong
        L.dmx_oracle_compress_par.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              u8p, ctypes.c_size_t]
        L.dmx_oracle_compress_par.restype = ctypes.c_longlong
        L.dmx_oracle_parse_block_hist.argtypes = [u8p, ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, u32p]
        L.dmx_oracle_parse_block_hist.restype = ctypes.c_int
        L.dmx_oracle_store_check.argtypes = [u8p, ctypes.c_int]
        L.dmx_oracle_store_check.restype = ctypes.c_int
        L.dmx_oracle_plan.argtypes = [u32p, ctypes.c_int, ctypes.c_int, u64p, u8p, u8p]
        L.dmx_oracle_plan.restype = ctypes.c_int
        L.dmx_oracle_set_deep_chain.argtypes = [ctypes.c_int]
        L.dmx_oracle_set_deep_chain.restype = None
        L.dmx_oracle_block_chain.argtypes = [u8p, ctypes.c_int, ctypes.c_int]
        L.dmx_oracle_block_chain.restype = ctypes.c_int
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _lz(lazy: bool, deep: bool) -> int:
    """The oracle's `lazy` argument: bit 0 = lazy evaluation (f2), bit 1 = DMX_F_DEEP."""
    return int(bool(lazy)) | (2 if deep else 0)


def set_deep_chain(k: int) -> None:
    """The depth DMX_F_DEEP gives small-alphabet blocks (0 = 32), as dmx_opts.deep_chain."""
    lib().dmx_oracle_set_deep_chain(int(k))


def block_chain(block, max_chain: int) -> int:
    """DMX_F_DEEP: the chain depth the block's own search uses (dmx_oracle_block_chain)."""
    a = _as_u8(block)
    return int(lib().dmx_oracle_block_chain(_u8(a), a.size, max_chain))


def _as_u8(data) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8)) if not isinstance(
        data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)


def parse_block(data, max_chain: int = 0, hash_kind: int = HASH_MUL, lazy: bool = False,
                hist=None, deep: bool = False) -> np.ndarray:
    """Token stream (uint32, see dmx_oracle.c header) of one block (<= 32768 bytes).
    hist: the bytes before the block as a dictionary (f1), or None.
    deep: the adaptive chain depth (DMX_F_DEEP; dmx_oracle_block_chain)."""
    a = _as_u8(data)
    assert a.size <= 32768
    tok = np.zeros(max(a.size, 1), dtype=np.uint32)
    h = _as_u8(hist if hist is not None else b"")
    n = lib().dmx_oracle_parse_block_hist(_u8(h), h.size, _u8(a), a.size, max_chain, hash_kind, _lz(lazy, deep),
                                          tok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return tok[:n].copy()


def parse(data, sw: int = 32768, max_chain: int = 0, hash_kind: int = HASH_MUL, lazy: bool = False,
          dict: bool = False, deep: bool = False) -> list:
    a = _as_u8(data)
    return [parse_block(a[o:o + sw], max_chain, hash_kind, lazy, a[o - sw:o] if dict and o else None, deep)
            for o in range(0, a.size, sw)]


def huff_lengths(freq, maxbits: int) -> np.ndarray:
    f = np.ascontiguousarray(freq, dtype=np.uint32)
    out = np.zeros(f.size, dtype=np.uint8)
    lib().dmx_oracle_huff_lengths(f.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), f.size,
                                  maxbits, _u8(out))
    return out


def adler32(data) -> int:
    a = _as_u8(data)
    return int(lib().dmx_oracle_adler32(_u8(a), a.size))


F_HEADER, F_TRAILER, F_FINAL = 1, 2, 4   # include/dmx.h framing bits (DMX_ZLIB = 7)


def compress(data, sw: int = 32768, max_chain: int = 0, hash_kind: int = HASH_MUL,
             want_btypes: bool = False, lazy: bool = False, split: bool = False, dict: bool = False,
             pre=None, store_check: bool = False, flags: int = 7, deep: bool = False):
    """zlib stream of `data`; lazy = f2 parse, split = f3 adaptive block splitting,
    dict = f1 cross-block dictionary (pre: the bytes before `data`, history of block 0),
    store_check = blocks that pass the DESIGN.md §4.7 noise check are stored unparsed.
    flags = the framing (F_HEADER | F_TRAILER | F_FINAL = a zlib stream; a shard of one
    otherwise, DESIGN.md §6: no BFINAL -> ends with a sync flush)."""
    a = _as_u8(data)
    nblk = (a.size + sw - 1) // sw
    cap = a.size + 5 * (nblk + 1) + 64
    out = np.zeros(cap, dtype=np.uint8)
    bt = np.zeros(max(nblk, 1), dtype=np.uint8)
    pa = _as_u8(pre if pre is not None else b"")
    r = lib().dmx_oracle_compress_framed(_u8(a), a.size, sw, max_chain, hash_kind, _lz(lazy, deep),
                                         int(split) | (2 if store_check else 0), int(dict), _u8(pa), pa.size,
                                         flags, _u8(out), cap, _u8(bt))
    if r < 0:
        raise RuntimeError(f"oracle compress failed: {r}")
    z = out[:r].tobytes()
    return (z, bt[:nblk].copy()) if want_btypes else z


def compress_par(data, sw: int = 32768, max_chain: int = 0, lazy: bool = False, split: bool = False,
                 dict: bool = False, store_check: bool = False, flags: int = 7, threads: int = 0,
                 deep: bool = False) -> bytes:
    """The same stream as compress(), blocks encoded in parallel by `threads` OpenMP threads
    (dmx_oracle_compress_par; the all-cores CPU baseline)."""
    a = _as_u8(data)
    nblk = (a.size + sw - 1) // sw
    cap = a.size + 5 * (nblk + 1) + 64
    out = np.zeros(cap, dtype=np.uint8)
    r = lib().dmx_oracle_compress_par(_u8(a), a.size, sw, max_chain, HASH_MUL, _lz(lazy, deep),
                                      int(split) | (2 if store_check else 0), int(dict), flags, threads, _u8(out), cap)
    if r < 0:
        raise RuntimeError(f"oracle compress_par failed: {r}")
    return out[:r].tobytes()


def store_check(block) -> bool:
    """would DMX_F_STORE_CHECK emit this block stored without a parse?"""
    a = _as_u8(block)
    return bool(lib().dmx_oracle_store_check(_u8(a), a.size))


def plan(tokens: np.ndarray, n: int):
    """(btype, (stored, fixed, dynamic) bit costs, litlen lengths, dist lengths)."""
    t = np.ascontiguousarray(tokens, dtype=np.uint32)
    costs = np.zeros(3, dtype=np.uint64)
    lll = np.zeros(286, dtype=np.uint8)
    ld = np.zeros(30, dtype=np.uint8)
    bt = lib().dmx_oracle_plan(t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), t.size, n,
                               costs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                               _u8(lll), _u8(ld))
    return bt, tuple(int(c) for c in costs), lll, ld


def replay(tokens) -> bytes:
    """check_lld's replay contract (tests/check_lld.c:20-39): rebuild the block."""
    out = bytearray()
    for t in np.asarray(tokens, dtype=np.uint32).tolist():
        d = t >> 9
        if d == 0:
            out.append(t & 0xFF)
        else:
            ln = t & 0x1FF
            s = len(out) - d
            assert s >= 0, "distance beyond block start"
            for k in range(ln):
                out.append(out[s + k])
    return bytes(out)


# ---- the reference itself (only where oracle/_ref was built, i.e. this container) ----

def ref_available() -> bool:
    return os.path.exists(REF_BIN)


def ref_stats(block: bytes) -> np.ndarray:
    """Run the reference encoder on one block; returns its int32[k,6] compress_stats."""
    assert 0 < len(block) <= 32768
    with tempfile.TemporaryDirectory() as td:
        fi, fs = os.path.join(td, "in"), os.path.join(td, "st")
        with open(fi, "wb") as f:
            f.write(block)
        subprocess.check_call([REF_BIN, fi, fs])
        return np.fromfile(fs, dtype="<i4").reshape(-1, 6)


def ref_tokens(block: bytes) -> np.ndarray:
    """Reference token stream in the oracle's uint32 encoding (ll, d) -> token."""
    st = ref_stats(block)
    ll = st[:, 4].astype(np.uint32)
    d = st[:, 5].astype(np.uint32)
    return np.where(d == 0, ll & 0xFF, (d << 9) | ll).astype(np.uint32)
