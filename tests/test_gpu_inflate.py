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
