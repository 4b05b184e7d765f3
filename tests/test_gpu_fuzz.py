"""Seeded fuzz: mixtures of text, noise, runs, uniform blocks and repeats at ragged sizes and
windows, through every parse/block option the encoder has, byte-identical to the oracle.
Bounded to a few seconds on the MI355X (-m gpu)."""
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from oracle import oracle as O  # noqa: E402


def piece(rng):
    kind = int(rng.integers(0, 6))
    n = int(rng.integers(1, 40000))
    if kind == 0:
        return D.gen_text(n, int(rng.integers(0, 1 << 30))).tobytes()
    if kind == 1:
        return D.gen_random(n, int(rng.integers(0, 1 << 30))).tobytes()
    if kind == 2:
        return bytes([int(rng.integers(0, 256))]) * n
    if kind == 3:   # short runs
        return b"".join(bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 300)) for _ in range(max(1, n // 150)))
    if kind == 4:   # a period
        per = bytes(rng.integers(0, 256, int(rng.integers(1, 50)), dtype=np.uint8))
        return (per * (n // len(per) + 1))[:n]
    return bytes(rng.integers(0, 8, n, dtype=np.uint8))   # small alphabet


@pytest.fixture(scope="module")
def enc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = D.Encoder(0, 4 << 20)
    yield e
    e.close()


# 40 seeds by default (DMX_FUZZ_N=300 ran clean once, profiles/ round 1)
@pytest.mark.parametrize("seed", range(int(os.environ.get("DMX_FUZZ_N", "40"))))
def test_fuzz_parity(enc, seed):
    rng = np.random.default_rng(1000 + seed)
    data = b"".join(piece(rng) for _ in range(int(rng.integers(1, 12))))[: 3 << 20]
    sw = int(rng.choice([32768, 32768, 32768, 4096, 12345, 65]))
    k = int(rng.choice([0, 1, 4, 6, 8, 16]))
    lazy = bool(rng.integers(0, 2))
    split = bool(rng.integers(0, 2))
    dct = bool(rng.integers(0, 2)) and sw >= 258
    chk = bool(rng.integers(0, 2))
    fl = (D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0) | (D.DMX_F_SPLIT if split else 0)
          | (D.DMX_F_DICT if dct else 0) | (D.DMX_F_STORE_CHECK if chk else 0))
    z, r = enc.compress_bytes(data, sw=sw, max_chain=k, flags=fl)
    zo = O.compress(data, sw=sw, max_chain=k, lazy=lazy, split=split, dict=dct, store_check=chk)
    assert z == zo, dict(n=len(data), sw=sw, k=k, lazy=lazy, split=split, dict=dct, check=chk)
    assert zlib.decompress(z) == data


@pytest.mark.parametrize("seed", range(int(os.environ.get("DMX_FUZZ_N", "40")) // 2))
def test_fuzz_inflate(enc, seed):
    """GPU inflate on the same mixtures: zlib's own streams (levels, strategies, window
    sizes) through the whole-stream decoder, and our streams through the block index."""
    rng = np.random.default_rng(5000 + seed)
    data = b"".join(piece(rng) for _ in range(int(rng.integers(1, 8))))[: 1 << 20]
    lvl = int(rng.integers(0, 10))
    strat = int(rng.choice([zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]))
    wbits = int(rng.integers(9, 16))
    co = zlib.compressobj(lvl, zlib.DEFLATED, wbits, 8, strat)
    zz = co.compress(data) + co.flush()
    if wbits == 15:   # the stream decoder reads zlib headers of window 32 KiB
        t = torch.frombuffer(bytearray(zz), dtype=torch.uint8).cuda()
        out, st = D.inflate_gpu(t, len(data) + 16)
        assert st == 0 and out.cpu().numpy().tobytes() == data
    fl = D.DMX_ZLIB | (D.DMX_F_LAZY if seed & 1 else 0) | (D.DMX_F_SPLIT if seed & 2 else 0) | D.DMX_F_STORE_CHECK
    zt, r = enc.compress_tensor(torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda(),
                                opts=D.Opts(32768, 6, fl, 0))
    ix, nb = enc.block_index()
    out, st = D.inflate_gpu(zt, len(data), index=ix, nblk=nb)
    assert st == 0 and out.cpu().numpy().tobytes() == data
