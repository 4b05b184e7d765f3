"""HIP path vs the CPU oracle (and the reference's golden tokens) on the MI355X.

Bar: bit-exact.  Token streams equal the reference's (tests/golden, exhaustive
mode); compressed bytes equal the oracle's stream byte for byte; every stream
inflates to the input with zlib and with our own deflate_decompress.
"""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from oracle import oracle as O  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLD, "manifest.json")))


@pytest.fixture(scope="module")
def enc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = D.Encoder(0, 8 << 20)
    yield e
    e.close()


def check_stream(z: bytes, data: bytes):
    assert zlib.decompress(z) == data
    assert D.deflate_decompress(z) == data


def test_golden_tokens_exact(enc, golden_cases, golden_tokens):
    """Per block: GPU tokens == the reference encoder's tokens; bytes == oracle bytes."""
    for name, data in golden_cases.items():
        z, r = enc.compress_bytes(data)
        assert r.nblocks == 1
        t = enc.tokens(0)
        assert np.array_equal(t, golden_tokens[name]), name
        assert hashlib.sha256(t.astype("<u4").tobytes()).hexdigest() == MAN["cases"][name]["tokens_sha256"]
        assert z == O.compress(data), name
        check_stream(z, data)


def test_code_lengths_match_oracle(enc, golden_cases):
    for name in ("bee0", "alldist", "px_sunrise_a", "abcd32k", "zeros32k"):
        data = golden_cases[name]
        enc.compress_bytes(data)
        bt, costs, lll, ld = O.plan(O.parse_block(data), len(data))
        _, gbt, _ = enc.blocks(1)
        assert int(gbt[0]) == bt, name
        if bt == 2:
            ln = enc.code_lengths(0)
            assert np.array_equal(ln[:286], lll) and np.array_equal(ln[286:], ld), name


@pytest.mark.parametrize("kind,n", [("bee", 57641), ("text", 1 << 20), ("zeros", 1 << 20), ("random", 300000),
                                    ("text", 3 * 32768 + 17), ("mixed", 400000)])
def test_multiblock_stream_identical(enc, golden_cases, kind, n):
    if kind == "bee":
        data = golden_cases["bee0"] + golden_cases["bee1"]
    elif kind == "text":
        data = D.gen_text(n, 0xE5818).tobytes()
    elif kind == "zeros":
        data = bytes(n)
    elif kind == "random":
        data = D.gen_random(n, 0x5EED).tobytes()
    else:
        a = D.gen_text(n, 7)
        a[100000:150000] = 0
        a[200000:260000] = D.gen_random(60000, 9)
        data = a.tobytes()
    z, r = enc.compress_bytes(data)
    zo = O.compress(data)
    assert z == zo
    assert r.adler == zlib.adler32(data)
    check_stream(z, data)


def test_config_c1_size(enc, golden_cases):
    bee = golden_cases["bee0"] + golden_cases["bee1"]
    z, _ = enc.compress_bytes(bee)
    assert len(z) == 24895   # S_ref of C1: 0 % size penalty


def test_config_c2_zeros(enc):
    """C2: 1 MiB of zeros = 32 blocks: literal, 127 x (258, 1), literal/short per block."""
    data = bytes(1 << 20)
    z, r = enc.compress_bytes(data)
    assert r.nblocks == 32
    for b in (0, 31):
        t = enc.tokens(b)
        assert np.array_equal(t, O.parse_block(data[:32768]))
    check_stream(z, data)
    assert len(z) <= 1.02 * 1466


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 16, 64])
def test_bounded_chain_parity(enc, k):
    data = D.gen_text(300000, 11).tobytes()
    z, _ = enc.compress_bytes(data, max_chain=k)
    assert z == O.compress(data, max_chain=k)
    check_stream(z, data)


@pytest.mark.parametrize("k", [0, 1, 4, 6, 7, 8, 16])
def test_lazy_parity(enc, golden_cases, k):
    """DMX_F_LAZY: byte-identical to the oracle's sequential lazy parse."""
    data = (golden_cases["bee0"] + D.gen_text(200000, 12).tobytes() + bytes(5000)
            + golden_cases["period7"] + D.gen_random(3000, 4).tobytes())
    z, _ = enc.compress_bytes(data, max_chain=k, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    assert z == O.compress(data, max_chain=k, lazy=True)
    check_stream(z, data)


@pytest.mark.parametrize("k", [0, 6, 7, 8, 16])
def test_exact_sort_fallback_parity(enc, golden_cases, k):
    """The match-any sort (the fallback if lane-ordered LDS atomics ever misorder) gives the
    same stream as the fast sort and the oracle.  dmx_result.nsortfallback counts the
    fallbacks: none on the fast path, at least one per searched block under the test hook
    (which forces the fallback), and the context total adds them up."""
    data = golden_cases["bee0"] + D.gen_text(150000, 21).tobytes() + bytes(3000) + golden_cases["runs32k"]
    for lazy in (False, True):
        f = D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0)
        z_fast, r_fast = enc.compress_bytes(data, max_chain=k, flags=f)
        tot0 = r_fast.nsortfallback_total
        z_exact, r_ex = enc.compress_bytes(data, max_chain=k, flags=f | D.DMX_F_EXACT_SORT)
        assert z_fast == z_exact == O.compress(data, max_chain=k, lazy=lazy)
        assert r_fast.nsortfallback == 0
        assert r_ex.nsortfallback >= r_ex.nblocks == 7
        assert r_ex.nsortfallback_total == tot0 + r_ex.nsortfallback


def test_lazy_tokens_and_edges(enc, golden_cases):
    for n in (0, 1, 2, 3, 4, 9, 258, 259, 32767, 32768, 32771):
        data = ((golden_cases["bee0"] + golden_cases["bee1"]) * 2)[:n]
        z, r = enc.compress_bytes(data, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
        assert z == O.compress(data, lazy=True), n
        check_stream(z, data)
    blk = golden_cases["bee0"]
    enc.compress_bytes(blk, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    assert np.array_equal(enc.tokens(0), O.parse_block(blk, max_chain=8, lazy=True))


@pytest.mark.parametrize("sw", [1, 2, 3, 64, 1000, 4095, 4096, 32767, 32768])
def test_window_sizes(enc, sw):
    data = D.gen_text(70000 if sw >= 64 else 3000, 5).tobytes()
    z, _ = enc.compress_bytes(data, sw=sw)
    assert z == O.compress(data, sw=sw)
    check_stream(z, data)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 63, 64, 65, 257, 258, 259, 32766, 32767, 32768, 32769, 65541])
def test_edge_sizes(enc, golden_cases, n):
    base = (golden_cases["bee0"] + golden_cases["bee1"]) * 2
    data = base[:n]
    z, _ = enc.compress_bytes(data)
    assert z == O.compress(data)
    check_stream(z, data)


def test_runs_and_periodic(enc):
    rng = np.random.default_rng(3)
    parts = []
    for _ in range(200):
        parts.append(bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 700)))
        parts.append((b"xyz" * 200)[: int(rng.integers(1, 500))])
    data = b"".join(parts)
    z, _ = enc.compress_bytes(data)
    assert z == O.compress(data)
    check_stream(z, data)


def test_shards_stitch(enc):
    """Multi-GPU shard framing: raw shards ending in a sync flush, concatenated,
    header on the first, BFINAL on the last, Adler combined on the host."""
    data = D.gen_text(5 * 32768 + 999, 21).tobytes()
    cut = [0, 2 * 32768, 4 * 32768, len(data)]
    pieces, adl = [], None
    for i in range(3):
        part = data[cut[i]:cut[i + 1]]
        fl = (D.DMX_F_HEADER if i == 0 else 0) | (D.DMX_F_FINAL if i == 2 else 0)
        z, r = enc.compress_bytes(part, flags=fl)
        pieces.append(z)
        adl = r.adler if adl is None else D.adler32_combine(adl, r.adler, len(part))
    stream = b"".join(pieces) + adl.to_bytes(4, "big")
    check_stream(stream, data)
    assert adl == zlib.adler32(data)


def test_fixed_blocks_high_literals(enc):
    """Fixed-Huffman blocks with literals 144..255 (9-bit codes, RFC 1951 3.2.6): the
    canonical assignment must count the 8-bit codes 280..287 too."""
    cases = [bytes([195]), bytes([143, 144, 255, 0, 200]), bytes(range(256)), bytes(range(255, -1, -1)) * 2,
             bytes([250]) * 5 + bytes([7, 251])]
    for data in cases:
        for sw in (1, 2, 7, 32768):
            for f in (D.DMX_ZLIB, D.DMX_ZLIB | D.DMX_F_LAZY):
                z, _ = enc.compress_bytes(data, sw=sw, max_chain=8, flags=f)
                assert z == O.compress(data, sw=sw, max_chain=8, lazy=bool(f & D.DMX_F_LAZY)), (list(data[:4]), sw)
                check_stream(z, data)


def test_raw_deflate_flags(enc):
    data = D.gen_text(100000, 4).tobytes()
    z, _ = enc.compress_bytes(data, flags=D.DMX_F_FINAL)
    assert zlib.decompressobj(-15).decompress(z) == data
    assert zlib.decompress(b"\x78\x9c" + z + zlib.adler32(data).to_bytes(4, "big")) == data


def test_fd_api_and_stats(tmp_path, golden_cases):
    """deflate_compress(fd_in, fd_out, fd_stats, sw, ops) drop-in: file in, zlib out,
    one compress_stats record per token; the check_lld replay contract on the records."""
    data = golden_cases["bee0"] + golden_cases["bee1"]
    fi, fo, fs = tmp_path / "in", tmp_path / "out", tmp_path / "st"
    fi.write_bytes(data)
    with open(fi, "rb") as a, open(fo, "wb") as b, open(fs, "wb") as c:
        assert D.deflate_compress(a.fileno(), b.fileno(), c.fileno(), 32768, 0) == 0
    z = fo.read_bytes()
    assert z == O.compress(data)
    st = np.frombuffer(fs.read_bytes(), dtype="<i4").reshape(-1, 6)
    toks = np.concatenate(O.parse(data))
    assert st.shape[0] == toks.size
    ll, d = st[:, 4].astype(np.uint32), st[:, 5].astype(np.uint32)
    rt = np.where(d == 0, ll, (d << 9) | ll).astype(np.uint32)
    assert np.array_equal(rt, toks)
    # bytes = 1 + token start offset (deflate_compress.c:235, :313)
    assert st[0, 0] == 1 and st[1, 0] == 2
    # replay block by block (tests/check_lld.c:20-39)
    assert O.replay(rt[: O.parse_block(data[:32768]).size]) == data[:32768]


def test_fd_api_stats_concurrent(tmp_path, golden_cases):
    """Two threads calling deflate_compress with fd_stats at once: the cached context is
    held across each call's encode and its token read-back, so every call's records are
    its own input's tokens."""
    import threading
    inputs = [golden_cases["bee0"] + golden_cases["bee1"], D.gen_text(70000, 91).tobytes()]
    res = [None, None]

    def run(j):
        fi, fo, fs = tmp_path / f"in{j}", tmp_path / f"out{j}", tmp_path / f"st{j}"
        fi.write_bytes(inputs[j])
        for _ in range(4):
            with open(fi, "rb") as a, open(fo, "wb") as b, open(fs, "wb") as c:
                rc = D.deflate_compress(a.fileno(), b.fileno(), c.fileno(), 32768, 0)
            st = np.frombuffer(fs.read_bytes(), dtype="<i4").reshape(-1, 6)
            ll, d = st[:, 4].astype(np.uint32), st[:, 5].astype(np.uint32)
            rt = np.where(d == 0, ll, (d << 9) | ll).astype(np.uint32)
            ok = rc == 0 and fo.read_bytes() == O.compress(inputs[j]) and \
                np.array_equal(rt, np.concatenate(O.parse(inputs[j])))
            if not ok:
                res[j] = False
                return
        res[j] = True

    th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert res == [True, True]


def test_fd_api_errors(tmp_path):
    fi = tmp_path / "in"
    fi.write_bytes(b"abc")
    with open(fi, "rb") as a:
        assert D.deflate_compress(a.fileno(), -1, -1, 40000 & 0xFFFF, 0) == -D.E["E_RANGE"]


def test_c3_scale_roundtrip(enc):
    """C3 size (100 000 000 B of enwik-style text): the whole stream equals the oracle's
    (its OpenMP form) at the reference parse (exhaustive) and at the bench's headline parse
    (K=7, lazy, adaptive depth, noise check), and both inflate."""
    n = 100_000_000
    a = D.gen_text(n, 0xE5818)
    t = torch.from_numpy(a).cuda()
    enc.reserve(n)
    out, r = enc.compress_tensor(t)
    z = out.cpu().numpy().tobytes()
    assert r.nblocks == 3052 and r.adler == zlib.adler32(a)
    assert 0.3 < len(z) / n < 0.5
    assert z == O.compress_par(a, max_chain=0, threads=16)
    assert zlib.decompress(z) == a.tobytes()
    for b in (0, 1526, 3051):
        blk = a[b * 32768:(b + 1) * 32768].tobytes()
        assert np.array_equal(enc.tokens(b), O.parse_block(blk))
    o = D.Opts(32768, 7, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_DEEP | D.DMX_F_STORE_CHECK, 0)
    out, r = enc.compress_tensor(t, opts=o)
    z = out.cpu().numpy().tobytes()
    assert z == O.compress_par(a, max_chain=7, lazy=True, deep=True, store_check=True, threads=16)
    assert zlib.decompress(z) == a.tobytes()


def _run_heavy(seed=7):
    rng = np.random.default_rng(seed)
    parts = []
    while sum(map(len, parts)) < 200000:
        r = rng.random()
        if r < 0.6:   # a run, lengths around and beyond the 258 cap and the block edges
            parts.append(bytes([int(rng.integers(0, 4))]) * int(rng.choice([1, 2, 3, 12, 13, 255, 258, 259, 300, 5000])))
        elif r < 0.8:
            parts.append(bytes(int(rng.integers(0, 256)) for _ in range(int(rng.integers(1, 20)))))
        else:
            parts.append((b"ab" * 400)[: int(rng.integers(2, 700))])
    return b"".join(parts)


@pytest.mark.parametrize("k", [1, 2, 4, 6, 7, 8])
@pytest.mark.parametrize("lazy", [False, True])
def test_run_dominated_blocks(enc, k, lazy):
    """Run-dominated blocks search with the change bitmap (run_len, bounded mode K <= 8):
    byte-identical to the oracle, also mixed with text blocks, with the dict, and on the
    exact-sort fallback (which rebuilds the bitmap)."""
    text = D.gen_text(100000, 3).tobytes()
    for data in (_run_heavy(), bytes(100000), text[:40000] + _run_heavy(9)[:70000] + text[40000:],
                 b"\x00" * 32767 + b"\x01" + b"\x00" * 40000):
        f = D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0)
        z, _ = enc.compress_bytes(data, max_chain=k, flags=f)
        assert z == O.compress(data, max_chain=k, lazy=lazy)
        check_stream(z, data)
        z2, _ = enc.compress_bytes(data, max_chain=k, flags=f | D.DMX_F_EXACT_SORT)
        assert z2 == z
        zd, _ = enc.compress_bytes(data, max_chain=k, flags=f | D.DMX_F_DICT)
        assert zd == O.compress(data, max_chain=k, lazy=lazy, dict=True)
    for sw in (16, 100, 1000, 4096):
        data = _run_heavy(11)[:50000]
        z, _ = enc.compress_bytes(data, sw=sw, max_chain=k, flags=D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0))
        assert z == O.compress(data, sw=sw, max_chain=k, lazy=lazy), sw


@pytest.mark.parametrize("n", [0, 1, 100000, 1 << 20, (1 << 20) + 1, 3 << 20, (3 << 20) + 777])
@pytest.mark.parametrize("mode", ["exhaustive", "k8_lazy", "k8_lazy_dict"])
def test_fd_api_streaming_chunks(tmp_path, n, mode):
    """deflate_compress without fd_stats streams the file in chunks (DMX_CHUNK_MB) through
    pinned buffers: one chunk is byte-identical to the one-shot stream; several chunks form
    one zlib stream (sync flushes, host Adler-32 combine; a one-byte lookahead makes an input
    that ends on a chunk boundary one chunk); with DMX_F_DICT the parse equals the one-shot one."""
    import os
    text = D.gen_text(max(n, 1), 31).tobytes()[:n]
    fi, fo = tmp_path / "in", tmp_path / "out"
    fi.write_bytes(text)
    env = {"DMX_CHUNK_MB": "1", "DMX_MAX_CHAIN": "0" if mode == "exhaustive" else "8",
           "DMX_LAZY": "0" if mode == "exhaustive" else "1", "DMX_DICT": "1" if "dict" in mode else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with open(fi, "rb") as a, open(fo, "wb") as b:
            assert D.deflate_compress(a.fileno(), b.fileno(), -1, 32768, 0) == 0
    finally:
        for k, v in old.items():
            os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)
    z = fo.read_bytes()
    assert zlib.decompress(z) == text
    assert D.deflate_decompress(z) == text
    kw = dict(max_chain=0 if mode == "exhaustive" else 8, lazy=mode != "exhaustive", dict="dict" in mode)
    if n <= 1 << 20:
        assert z == O.compress(text, **kw)
    else:   # the parse is the one-shot parse: the chunks' tokens equal the oracle's blocks
        one = O.compress(text, **kw)
        nchunks = (n + (1 << 20) - 1) >> 20
        assert abs(len(z) - len(one)) <= 8 * nchunks


@pytest.mark.parametrize("n", [0, 5000, 1 << 20, (5 << 19) + 3])
def test_fd_api_streaming_pipes_and_offsets(tmp_path, n):
    """The streaming fd path on pipes (read() + one-byte lookahead, output through a pipe)
    and on a regular file read from a non-zero offset (parallel preads from there; the
    offset is left at EOF, as read() would leave it)."""
    import os
    import threading
    text = D.gen_text(max(n, 1), 77).tobytes()[:n]
    env = {"DMX_CHUNK_MB": "1", "DMX_MAX_CHAIN": "8", "DMX_LAZY": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        # pipes in and out
        ri, wi = os.pipe()
        ro, wo = os.pipe()
        got = []
        feeder = threading.Thread(target=lambda: (os.write(wi, text) if text else None, os.close(wi)))
        reader = threading.Thread(target=lambda: got.append(b"".join(iter(lambda: os.read(ro, 1 << 16), b""))))
        feeder.start()
        reader.start()
        rc = D.deflate_compress(ri, wo, -1, 32768, 0)
        os.close(wo)
        feeder.join()
        reader.join()
        os.close(ri)
        os.close(ro)
        assert rc == 0
        assert zlib.decompress(got[0]) == text
        # regular file from an offset
        fi, fo = tmp_path / "in", tmp_path / "out"
        fi.write_bytes(b"HEADER----" + text)
        with open(fi, "rb") as a, open(fo, "wb") as b:
            assert os.read(a.fileno(), 10) == b"HEADER----"
            assert D.deflate_compress(a.fileno(), b.fileno(), -1, 32768, 0) == 0
            assert os.lseek(a.fileno(), 0, os.SEEK_CUR) == 10 + n
        z = fo.read_bytes()
        assert zlib.decompress(z) == text
        assert z == got[0]   # same framing whichever reader ran
        if n <= 1 << 20:
            assert z == O.compress(text, max_chain=8, lazy=True)
    finally:
        for k, v in old.items():
            os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)


@pytest.mark.parametrize("check", [False, True])
@pytest.mark.parametrize("k,lazy", [(0, False), (6, True), (7, True), (8, False), (16, True)])
def test_uniform_blocks_closed_form(enc, check, k, lazy):
    """Blocks of one repeated byte take a closed-form parse (K1's uniform path, or K0's with
    DMX_F_STORE_CHECK): byte-identical to the oracle's search for every remainder of
    (n - 1) mod 258 around the 3-byte threshold, several byte values, short and full blocks,
    uniform blocks next to text and runs that are almost uniform."""
    fl = D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0) | (D.DMX_F_STORE_CHECK if check else 0)
    for c in (0x00, 0x41, 0xFF):
        for n in (1, 2, 3, 4, 5, 258, 259, 260, 261, 262, 516, 517, 518, 4095, 4096, 4097, 32767, 32768):
            data = bytes([c]) * n
            z, _ = enc.compress_bytes(data, max_chain=k, flags=fl)
            assert z == O.compress(data, max_chain=k, lazy=lazy, store_check=check), (c, n)
    almost = bytearray(32768)
    almost[20000] = 1   # one odd byte: not uniform
    data = bytes(32768) + D.gen_text(40000, 3).tobytes() + bytes([7]) * 32768 + bytes(almost) + bytes([9]) * 1000
    z, _ = enc.compress_bytes(data, max_chain=k, flags=fl)
    assert z == O.compress(data, max_chain=k, lazy=lazy, store_check=check)
    assert zlib.decompress(z) == data


@pytest.mark.parametrize("n", [5000, (9 << 20) + 123])
def test_fd_api_output_offset_and_append(tmp_path, n):
    """fd_out is written from its current offset (positioned parallel writes on a regular file)
    and left at the stream's end, as write() would; an O_APPEND fd takes write() and appends."""
    import os
    text = D.gen_text(n, 93).tobytes()
    fi = tmp_path / "in"
    fi.write_bytes(text)
    env = {"DMX_CHUNK_MB": "4", "DMX_MAX_CHAIN": "7", "DMX_LAZY": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        fo = tmp_path / "out"
        with open(fi, "rb") as a:
            b = os.open(fo, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            os.write(b, b"HDR")
            assert D.deflate_compress(a.fileno(), b, -1, 32768, 0) == 0
            end = os.lseek(b, 0, os.SEEK_CUR)
            os.write(b, b"END")
            os.close(b)
        got = fo.read_bytes()
        assert got[:3] == b"HDR" and got[-3:] == b"END" and end == len(got) - 3
        z = got[3:-3]
        assert zlib.decompress(z) == text
        fa = tmp_path / "app"
        fa.write_bytes(b"PRE")
        with open(fi, "rb") as a:
            b = os.open(fa, os.O_WRONLY | os.O_APPEND)
            assert D.deflate_compress(a.fileno(), b, -1, 32768, 0) == 0
            os.close(b)
        assert fa.read_bytes() == b"PRE" + z
    finally:
        for k, v in old.items():
            os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)
