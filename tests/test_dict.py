"""SURVEY §8 f1, cross-block dictionary (DMX_F_DICT), CPU side: the oracle's history
parse (oracle/dmx_oracle.c dmx_oracle_parse_block_hist) pinned against an independent
Python statement of DESIGN.md §4.6, and its streams checked with zlib.

The reference intends this (README.md:6-14, the A/B two-window design of
src/deflate_compress.c:14-62) but its multi-window path is broken, so
there is no reference output to pin against: the rule is the project's own and these
tests state it a second time, independently of the C code ("parity unpinned" against
the reference; pinned against the specification).
"""
import zlib
from collections import defaultdict

import numpy as np
import pytest

from oracle import oracle as O


def _h(b: bytes, i: int) -> int:
    t = b[i] | (b[i + 1] << 8) | (b[i + 2] << 16)
    return ((t * 0x9E3779B1) & 0xFFFFFFFF) >> 19


def _common(src: bytes, s: int, dst: bytes, i: int, lim: int) -> int:
    t = 0
    while t < lim and src[s + t] == dst[i + t]:
        t += 1
    return t


def _dict_parse(hist: bytes, d: bytes, K: int, lazy: bool) -> np.ndarray:
    """DESIGN.md §4.6 restated: best(i) = the block's own longest match (K newest entries of
    its bucket chain, ties to the nearest); a history match (the K newest history entries of
    the bucket with q + 2 < hn and distance <= 32768, ties to the nearest) replaces it only
    when strictly longer; then greedy or lazy evaluation over best()."""
    hn, n = len(hist), len(d)
    hb = defaultdict(list)
    for q in range(hn - 2):
        hb[_h(hist, q)].append(q)
    ib = defaultdict(list)
    for p in range(n - 2):
        ib[_h(d, p)].append(p)
    cat = hist + d
    cache = {}

    def best(i):
        if i in cache:
            return cache[i]
        lim = min(258, n - i)
        res = (0, 0)
        if lim >= 3:
            h = _h(d, i)
            own = [p for p in ib[h] if p < i][::-1]
            if K:
                own = own[:K]
            bl, bd = 0, 0
            for p in own:
                t = _common(d, p, d, i, lim)
                if t >= 3 and t > bl:
                    bl, bd = t, i - p
            hc = hb[h][::-1]
            if K:
                hc = hc[:K]
            hl, hd = 0, 0
            for q in hc:
                if hn - q + i > 32768:
                    break
                t = _common(cat, q, d, i, lim)
                if t >= 3 and t > hl:
                    hl, hd = t, hn - q + i
            res = (hl, hd) if hl > bl else (bl, bd)
        cache[i] = res
        return res

    toks, i = [], 0
    while i < n:
        ln, dist = best(i)
        if ln >= 3 and lazy and i + 1 < n and best(i + 1)[0] > ln:
            ln = 0
        if ln >= 3:
            toks.append((dist << 9) | ln)
            i += ln
        else:
            toks.append(d[i])
            i += 1
    return np.array(toks, dtype=np.uint32)


def _replay(hist: bytes, toks) -> bytes:
    out = bytearray(hist)
    for t in np.asarray(toks, dtype=np.uint32).tolist():
        if t >> 9 == 0:
            out.append(t & 0xFF)
        else:
            s = len(out) - (t >> 9)
            assert s >= 0 and (t >> 9) <= 32768
            for k in range(t & 0x1FF):
                out.append(out[s + k])
    return bytes(out[len(hist):])


def _text(n, seed):
    import deflate_compression_amd as D
    return D.gen_text(n, seed).tobytes()


CASES = {
    # full 32 KiB windows: the distance limit (q >= i) is active
    "text32k": lambda: (_text(65536, 11)[:32768], _text(65536, 11)[32768:]),
    "bee": lambda: (None, None),
    "zeros": lambda: (bytes(32768), bytes(5000)),
    "runs_boundary": lambda: (b"xyz" * 10000 + b"abcdefgh" * 345, b"abcdefgh" * 600 + b"tail"),
    "short_hist": lambda: (b"hello world, hello dictionary", b"hello dictionary world, hello world!"),
    "tiny_hist": lambda: (b"ab", b"abababab"),
}


@pytest.mark.parametrize("name", ["text32k", "bee", "zeros", "runs_boundary", "short_hist", "tiny_hist"])
@pytest.mark.parametrize("K", [1, 4, 8])
@pytest.mark.parametrize("lazy", [False, True])
def test_hist_parse_matches_restatement(golden_cases, name, K, lazy):
    if name == "bee":
        hist, d = golden_cases["bee0"], golden_cases["bee1"][:12000]
    else:
        hist, d = CASES[name]()
    t = O.parse_block(d, K, lazy=lazy, hist=hist)
    assert np.array_equal(t, _dict_parse(hist, d, K, lazy)), (name, K, lazy)
    assert _replay(hist, t) == d


def test_hist_parse_exhaustive_matches_restatement():
    hist, d = _text(12000, 5)[:6000], _text(12000, 5)[6000:9000]
    for lazy in (False, True):
        assert np.array_equal(O.parse_block(d, 0, lazy=lazy, hist=hist), _dict_parse(hist, d, 0, lazy))


def test_no_history_is_the_plain_parse(golden_cases):
    d = golden_cases["bee0"]
    for K in (0, 8):
        assert np.array_equal(O.parse_block(d, K, hist=b""), O.parse_block(d, K))


@pytest.mark.parametrize("sw", [32768, 4096, 1000, 17])
@pytest.mark.parametrize("K", [0, 8])
def test_dict_stream_inflates(sw, K):
    d = _text(150000, 3) + bytes(40000) + _text(30000, 3)
    for lazy in (False, True):
        z = O.compress(d, sw=sw, max_chain=K, lazy=lazy, dict=True)
        assert zlib.decompress(z) == d
        zs = O.compress(d, sw=sw, max_chain=K, lazy=lazy, dict=True, split=True)
        assert zlib.decompress(zs) == d


def test_dict_with_pre_history():
    """Block 0 takes the caller's preceding bytes as history (shards of one stream)."""
    full = _text(200000, 9)
    pre, d = full[:65536], full[65536:]
    z = O.compress(d, max_chain=8, lazy=True, dict=True, pre=pre)
    dec = zlib.decompressobj(wbits=-15, zdict=pre[-32768:])   # raw inflate with the preset window
    assert dec.decompress(z[2:-4]) + dec.flush() == d
    assert int.from_bytes(z[-4:], "big") == zlib.adler32(d)
    # == the tail of the stream over pre||d, block for block
    t0 = O.parse_block(d[:32768], 8, lazy=True, hist=pre[-32768:])
    assert np.array_equal(t0, O.parse(full, max_chain=8, lazy=True, dict=True)[2])


def test_dict_is_smaller():
    d = _text(1 << 20, 4)
    for K in (4, 8):
        a = len(O.compress(d, max_chain=K, lazy=True))
        b = len(O.compress(d, max_chain=K, lazy=True, dict=True))
        assert b < 0.97 * a, (K, a, b)
