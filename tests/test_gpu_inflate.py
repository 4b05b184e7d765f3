"""GPU inflate (csrc/dmx_inflate_dev.hip): bit-exact round trips on device.

Indexed mode decodes every block of a dmx stream in parallel from the encoder's block
index; stream mode decodes any zlib stream (here: ours, and zlib's own at several levels,
which use cross-block references and stored blocks) in one workgroup with the Adler-32
check.  Corrupted input must end with an error status, never a hang or a fault.
"""
import zlib

import numpy as np
import pytest
import torch

import deflate_compression_amd as D

pytestmark = pytest.mark.gpu


def _dev(b: bytes):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda() if b else torch.zeros(1, dtype=torch.uint8).cuda()


def _inputs(golden_cases):
    return {
        "text": D.gen_text(400_000, 31).tobytes(),
        "bee": golden_cases["bee0"] + golden_cases["bee1"],
        "zeros": bytes(200_000),
        "random": D.gen_random(100_000, 5).tobytes(),
        "mixed": golden_cases["runs32k"] + D.gen_random(5000, 2).tobytes() + golden_cases["period7"] + bytes(70000),
        "tiny": b"ab",
        "one": b"x",
        "high": bytes([195, 250, 144, 143, 255]),   # fixed block, 9-bit literal codes
    }


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("k", [0, 8])
def test_indexed_roundtrip(golden_cases, k, lazy):
    enc = D.Encoder(0, 1 << 20)
    try:
        for name, data in _inputs(golden_cases).items():
            t = _dev(data)
            flags = D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0)
            opts = D.Opts(32768, k, flags, 0)
            out, r = enc.compress_tensor(t[:len(data)], opts=opts)
            ix, n = enc.block_index()
            dec, st = D.inflate_gpu(out, len(data), ix, n)
            assert st == 0, (name, st)
            assert dec.cpu().numpy().tobytes() == data, name
    finally:
        enc.close()


def test_stream_mode_ours(golden_cases):
    for name, data in _inputs(golden_cases).items():
        z = D.compress(data, max_chain=8, lazy=True)
        dec, st = D.inflate_gpu(_dev(z), len(data) + 16)
        assert st == 0, (name, st)
        assert dec.cpu().numpy().tobytes() == data, name


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_stream_mode_zlib(golden_cases, level):
    """zlib's streams: history across blocks, stored blocks (level 0), all code shapes."""
    for name, data in _inputs(golden_cases).items():
        z = zlib.compress(data, level)
        dec, st = D.inflate_gpu(_dev(z), len(data) + 16)
        assert st == 0, (name, level, st)
        assert dec.cpu().numpy().tobytes() == data, (name, level)


def test_stream_mode_png_idat():
    """The reference's own inflate consumer: PNG IDAT streams (tests/golden/idat)."""
    import glob
    import os
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "idat", "*.zlib")))
    assert files
    for f in files:
        z = open(f, "rb").read()
        want = zlib.decompress(z)
        dec, st = D.inflate_gpu(_dev(z), len(want) + 16)
        assert st == 0, (f, st)
        assert dec.cpu().numpy().tobytes() == want, f


def test_errors_terminate(golden_cases):
    data = golden_cases["bee0"]
    z = bytearray(zlib.compress(data, 6))
    rng = np.random.default_rng(7)
    bad = 0
    for trial in range(40):
        c = bytearray(z)
        for _ in range(1 + trial % 4):
            c[int(rng.integers(2, len(c)))] ^= 1 << int(rng.integers(0, 8))
        dec, st = D.inflate_gpu(_dev(bytes(c)), len(data) + 16)
        if st != 0:
            bad += 1
        else:   # a flip can survive decoding only if the output still matches Adler-32
            assert dec.cpu().numpy().tobytes() == data
    assert bad > 30
    for z2 in (b"", b"\x78", b"\x78\x9c", b"\x79\x9c\x03\x00", bytes(z[:20])):
        _, st = D.inflate_gpu(_dev(z2), 100000)
        assert st < 0
    _, st = D.inflate_gpu(_dev(bytes(z)), 100)   # output cap too small
    assert st == -D.E["E_SZ"]


def test_indexed_matches_bulk_decode_at_scale():
    n = 20_000_000
    data = D.gen_text(n, 41)
    t = torch.from_numpy(data).cuda()
    enc = D.Encoder(0, n, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    try:
        out, r = enc.compress_tensor(t)
        ix, nb = enc.block_index()
        dec, st = D.inflate_gpu(out, n, ix, nb)
        assert st == 0 and dec.numel() == n
        assert torch.equal(dec, t)
    finally:
        enc.close()


def _ring_edge_inputs():
    """Inputs aimed at the symbol loop's paths (isym_run): sources at and across the indexed
    ring's edge (8 KiB) and the stream ring's (32 KiB), short periods 1..63 and periods 64..257
    under 258-byte matches, and a skewed literal alphabet whose rare literals get codes longer
    than the 10-bit first-level table (the slow path)."""
    rng = np.random.default_rng(77)
    out = {}
    for d in (4095, 4096, 4097, 8191, 8192, 8193, 16384, 24576, 32767):
        head = rng.integers(0, 256, d, dtype=np.uint8).tobytes()
        out[f"dist{d}"] = head + head[:32768 - d] + head[:1000]
    per = b""
    for p in list(range(1, 64)) + [64, 65, 100, 129, 200, 257]:
        unit = rng.integers(0, 256, p, dtype=np.uint8).tobytes()
        per += rng.integers(0, 256, 7, dtype=np.uint8).tobytes() + (unit * (600 // p + 2))[:600]
    out["periods"] = per
    geo = np.minimum(rng.geometric(0.18, 120_000), 255).astype(np.uint8)   # literal codes up to 15 bits
    out["skewed"] = geo.tobytes()
    words = [bytes(rng.integers(97, 123, rng.integers(2, 9), dtype=np.uint8)) for _ in range(300)]
    out["skewed_text"] = b" ".join(words[min(int(rng.geometric(0.02)), 299)] for _ in range(30000))
    return out


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("k", [0, 8])
def test_indexed_ring_edges(k, lazy):
    enc = D.Encoder(0, 1 << 20)
    try:
        for name, data in _ring_edge_inputs().items():
            t = _dev(data)
            opts = D.Opts(32768, k, D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0), 0)
            out, r = enc.compress_tensor(t[:len(data)], opts=opts)
            assert zlib.decompress(out.cpu().numpy().tobytes()) == data, name
            ix, n = enc.block_index()
            dec, st = D.inflate_gpu(out, len(data), ix, n)
            assert st == 0, (name, st)
            assert dec.cpu().numpy().tobytes() == data, name
    finally:
        enc.close()


@pytest.mark.parametrize("level", [1, 9])
def test_stream_ring_edges(level):
    for name, data in _ring_edge_inputs().items():
        z = zlib.compress(data, level)
        dec, st = D.inflate_gpu(_dev(z), len(data) + 16)
        assert st == 0, (name, level, st)
        assert dec.cpu().numpy().tobytes() == data, (name, level)


def _max_code_lengths(z: bytes, raw_offset: int = 2):
    """(longest literal/length code, longest distance code) of the first DEFLATE block of a
    zlib stream (RFC 1951 §3.2.7 header), or None if that block is not dynamic."""
    pos = raw_offset * 8

    def bits(n):
        nonlocal pos
        v = 0
        for i in range(n):
            v |= ((z[(pos + i) >> 3] >> ((pos + i) & 7)) & 1) << i
        pos += n
        return v

    bits(1)
    if bits(2) != 2:
        return None
    hlit, hdist, hclen = bits(5) + 257, bits(5) + 1, bits(4) + 4
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl = [0] * 19
    for k in range(hclen):
        cl[order[k]] = bits(3)
    # canonical decode of the code-length code (codes read MSB first)
    codes, code, nxt = {}, 0, {}
    for L in range(1, 8):
        code = (code + sum(1 for x in cl if x == L - 1 and L > 1)) << 1 if L > 1 else 0
        nxt[L] = code
    for s in range(19):
        if cl[s]:
            codes[(cl[s], nxt[cl[s]])] = s
            nxt[cl[s]] += 1
    lens = []
    while len(lens) < hlit + hdist:
        c, L = 0, 0
        while (L, c) not in codes or L == 0:
            c = (c << 1) | bits(1)
            L += 1
        s = codes[(L, c)]
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (3 + bits(2))
        elif s == 17:
            lens += [0] * (3 + bits(3))
        else:
            lens += [0] * (11 + bits(7))
    return max(lens[:hlit]), max(lens[hlit:])


def _long_code_input() -> bytes:
    """Text with rare literals (each once: long literal codes), one long repeat (a rare length
    symbol) and a few far repeats (rare distance codes)."""
    rng = np.random.default_rng(77)
    t = bytearray(D.gen_text(30000, 41).tobytes())
    for k, p in enumerate(rng.choice(len(t), 60, replace=False)):
        t[int(p)] = 128 + k
    t[20000:20230] = t[3000:3230]                          # a 230-byte match
    for d, p in ((5, 9000), (6, 9100), (9, 9200), (13, 9300)):
        t[p:p + 5] = t[p - d:p - d + 5]                     # short-distance matches: distance codes 4..7
    return bytes(t)


def test_long_codes_inside_the_run():
    """Literal/length and distance codes longer than the 10-bit first-level tables: decoded
    inside the asm run from the canonical arrays.  Checked on our
    streams (indexed, one block) and zlib's (stream mode); the headers are parsed to show the
    codes really are longer than 10 bits."""
    data = _long_code_input()
    enc = D.Encoder(0, 1 << 20)
    try:
        for k, lazy in ((0, False), (8, True)):
            z = D.compress(data, max_chain=k, lazy=lazy)
            ll, dl = _max_code_lengths(z)
            assert ll > 10 and dl > 10, (k, ll, dl)
            out, r = enc.compress_tensor(_dev(data), opts=D.Opts(32768, k, D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0), 0))
            ix, n = enc.block_index()
            dec, st = D.inflate_gpu(out, len(data), ix, n)
            assert st == 0 and dec.cpu().numpy().tobytes() == data, (k, st)
            dec, st = D.inflate_gpu(_dev(z), len(data) + 16)
            assert st == 0 and dec.cpu().numpy().tobytes() == data, (k, st)
    finally:
        enc.close()
    for level in (6, 9):
        z = zlib.compress(data, level)
        dec, st = D.inflate_gpu(_dev(z), len(data) + 16)
        assert st == 0 and dec.cpu().numpy().tobytes() == data, (level, st)


def test_many_short_lived_streams(golden_cases):
    """dmx_inflate_async on more than 64 short-lived streams (created and dropped
    per call) and on two threads' default streams returns 0 every time and decodes bit-exact:
    the table scratch is a stream-ordered pool allocation per call, not a per-stream cache."""
    import threading
    data = golden_cases["bee0"] + D.gen_text(50_000, 3).tobytes()
    enc = D.Encoder(0, 1 << 20)
    try:
        out, r = enc.compress_tensor(_dev(data)[:len(data)], opts=D.Opts(32768, 8, D.DMX_ZLIB | D.DMX_F_LAZY, 0))
        ix, n = enc.block_index()
        torch.cuda.synchronize()
        for k in range(80):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                dec, st = D.inflate_gpu(out, len(data), ix, n, stream=s.cuda_stream)
            s.synchronize()
            assert st == 0, (k, st)
            assert dec.cpu().numpy().tobytes() == data, k
            del s
        res = [None, None]

        def run(j):
            d2, st2 = D.inflate_gpu(out, len(data), ix, n)
            torch.cuda.synchronize()
            res[j] = st2 == 0 and d2.cpu().numpy().tobytes() == data

        th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert res == [True, True]
    finally:
        enc.close()
