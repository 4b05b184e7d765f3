"""DMX_F_SPLIT (adaptive block splitting) on the MI355X.

Bar: the GPU stream equals the oracle's split stream byte for byte (same quarter cut
points, same per-group Huffman plans, same cheapest-cut choice and tie-break), it inflates
with zlib, our CPU inflate and the GPU inflate, and it is never larger than the unsplit
stream.  In DMX_STATS=exact the compress_stats side channel follows every DEFLATE block's
own codes and header, in running sums over the whole stream.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def enc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = D.Encoder(0, 8 << 20)
    yield e
    e.close()


def _het(n_pieces=24, seed=3):
    """Text, random and zero pieces of 8 KiB: the statistics change inside a block."""
    text = D.gen_text(n_pieces * 8192, seed).tobytes()
    rnd = D.gen_random(n_pieces * 8192, seed + 1).tobytes()
    out = []
    for i in range(n_pieces):
        k = (i * 7 + seed) % 4
        out.append(text[i * 8192:(i + 1) * 8192] if k in (0, 3) else
                   rnd[i * 4096:i * 4096 + 8192] if k == 1 else bytes(8192))
    return b"".join(out)


_LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131,
          163, 195, 227, 258]
_LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
_DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049,
          3073, 4097, 6145, 8193, 12289, 16385, 24577]


def _len_sym(n):   # RFC 1951 3.2.5: (symbol, extra bits)
    i = max(k for k in range(29) if _LBASE[k] <= n)
    return 257 + i, _LEXT[i]


def _dist_sym(d):
    i = max(k for k in range(30) if _DBASE[k] <= d)
    return i, 0 if i < 4 else i // 2 - 1


def _check(z, data):
    assert zlib.decompress(z) == data
    assert D.deflate_decompress(z) == data


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("k", [0, 8])
def test_split_parity(enc, golden_cases, k, lazy):
    f = D.DMX_ZLIB | D.DMX_F_SPLIT | (D.DMX_F_LAZY if lazy else 0)
    for data in (golden_cases["bee0"] + golden_cases["bee1"], _het(), D.gen_text(150000, 9).tobytes(),
                 bytes(70000), D.gen_random(40000, 2).tobytes() + bytes(30000)):
        z, _ = enc.compress_bytes(data, max_chain=k, flags=f)
        assert z == O.compress(data, max_chain=k, lazy=lazy, split=True)
        _check(z, data)
        z1, _ = enc.compress_bytes(data, max_chain=k, flags=f & ~D.DMX_F_SPLIT)
        assert len(z) <= len(z1)


@pytest.mark.parametrize("sw", [1, 3, 7, 64, 1000, 32768])
def test_split_edges(enc, golden_cases, sw):
    base = (golden_cases["bee0"] + golden_cases["runs32k"])
    for n in (0, 1, 2, 3, 4, 5, 9, 100, 4097, 32768, 32771, 70001):
        data = (base * 3)[:n]
        if sw < 64 and n > 5000:
            continue
        z, _ = enc.compress_bytes(data, sw=sw, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT)
        assert z == O.compress(data, sw=sw, max_chain=8, split=True), (sw, n)
        _check(z, data)


def test_split_heterogeneous_blocks(enc):
    data = _het(32, 5)
    z, r = enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT | D.DMX_F_LAZY)
    z1, _ = enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    assert len(z) < len(z1) * 0.99   # mixed statistics inside a block: splitting pays
    enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT | D.DMX_F_LAZY)
    nsplit = 0
    for b in range(r.nblocks):
        subs = enc.subblocks(b)
        nt = enc.tokens(b).size
        assert 1 <= len(subs) <= 4
        assert subs[0][0] == 0 and subs[-1][1] == nt
        for s0, s1 in zip(subs, subs[1:]):
            assert s0[1] == s1[0] and s0[1] > s0[0]
        nsplit += len(subs) > 1
    assert nsplit > 0


def test_split_gpu_inflate(enc, golden_cases):
    """The indexed GPU inflate decodes every sw block's DEFLATE blocks in one workgroup."""
    data = _het(40, 11) + golden_cases["bee0"]
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    e = D.Encoder(0, len(data), max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT | D.DMX_F_LAZY)
    try:
        out, r = e.compress_tensor(t)
        assert out.cpu().numpy().tobytes() == O.compress(data, max_chain=8, lazy=True, split=True)
        ix, nb = e.block_index()
        dec, st = D.inflate_gpu(out, len(data), ix, nb)
        assert st == 0 and torch.equal(dec, t)
        dec2, st2 = D.inflate_gpu(out, len(data) + 16)   # whole-stream mode
        assert st2 == 0 and torch.equal(dec2, t)
    finally:
        e.close()


def test_split_stats(tmp_path, enc, monkeypatch):
    """fd API with DMX_SPLIT=1: the stream equals the oracle's split stream and the
    compress_stats records follow each DEFLATE block's own codes and header, in running sums
    over the whole stream (dmx_host.c write_stats)."""
    data = _het(10, 7)
    fi, fo, fs = tmp_path / "in", tmp_path / "out", tmp_path / "st"
    fi.write_bytes(data)
    monkeypatch.setenv("DMX_SPLIT", "1")
    monkeypatch.setenv("DMX_MAX_CHAIN", "8")
    monkeypatch.setenv("DMX_STATS", "exact")
    with open(fi, "rb") as a, open(fo, "wb") as b, open(fs, "wb") as c:
        assert D.deflate_compress(a.fileno(), b.fileno(), c.fileno(), 32768, 0) == 0
    assert fo.read_bytes() == O.compress(data, max_chain=8, split=True)
    st = np.frombuffer(fs.read_bytes(), dtype="<i4").reshape(-1, 6)
    # expected records from the same encode on our own context
    enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT)
    nblk = (len(data) + 32767) // 32768
    row = 0
    tree = ll = dd = 0
    for b in range(nblk):
        toks = enc.tokens(b)
        for (t0, t1, bt, hb, ln) in enc.subblocks(b):
            tree += hb if bt == 2 else 3
            for k in range(t0, t1):
                t = int(toks[k])
                if t >> 9 == 0:
                    ll += 8 if bt == 0 else int(ln[t & 0xFF])
                else:
                    L, dist = t & 0x1FF, t >> 9
                    if bt == 0:
                        ll += 8 * L
                    else:
                        s, eb = _len_sym(L)
                        ll += int(ln[s]) + eb
                        s, eb = _dist_sym(dist)
                        dd += int(ln[286 + s]) + eb
                assert st[row, 1] == tree
                assert st[row, 2] == ll and st[row, 3] == dd, (b, k)
                row += 1
    assert row == st.shape[0]
