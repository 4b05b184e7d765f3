"""The exhaustive parse (max_chain = 0, the reference's semantics) on 4-byte chains
(DESIGN.md §3, P0'): every match of 4 or more bytes is searched among positions with the same
first 4 bytes, a match of exactly 3 comes from the nearest earlier position with the same
trigram.  Tokens must equal the oracle's (the reference's parse, pinned by its golden blocks)
at every block size -- small blocks put many positions near the block end, where a 4-byte
gram runs into the zero padding -- and on inputs where trigram buckets collide."""
import numpy as np
import pytest
import torch

import deflate_compression_amd as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _check(data: bytes, sw: int, lazy: bool = False):
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    enc = D.Encoder(0, 1 << 20)
    try:
        out, r = enc.compress_tensor(t, opts=D.Opts(sw, 0, D.DMX_ZLIB | (D.DMX_F_LAZY if lazy else 0), 0))
        a = np.frombuffer(data, np.uint8)
        for b in range(r.nblocks):
            o = O.parse_block(a[b * sw:(b + 1) * sw], 0, lazy=lazy)
            assert np.array_equal(enc.tokens(b), o), (sw, b)
    finally:
        enc.close()


@pytest.mark.parametrize("sw", [300, 999, 1000, 1001, 4096, 32768])
def test_exhaustive_tokens_block_sizes(sw):
    _check(D.gen_text(60000, 17).tobytes(), sw)


@pytest.mark.parametrize("lazy", [False, True])
def test_exhaustive_tokens_collisions_and_ends(golden_cases, lazy):
    rng = np.random.default_rng(5)
    # few distinct trigrams in long runs of one (chains cross many collisions), grams that
    # differ only in their 4th / 5th byte, and blocks ending inside repeats
    alpha = rng.integers(0, 256, (40, 3), dtype=np.uint8)
    grams = b"".join(bytes(alpha[rng.integers(0, 40)]) + bytes([rng.integers(0, 4)]) for _ in range(20000))
    data = golden_cases["bee0"] + grams + D.gen_text(30000, 3).tobytes() + b"abcabcabx" * 500
    _check(data, 32768, lazy)
    _check(data[:70001], 7000, lazy)


def _colliding_trigram(a: bytes) -> bytes:
    """A trigram of printable bytes in the same 13-bit bucket as `a` (dmx_hash), a != it."""
    ta = a[0] | a[1] << 8 | a[2] << 16
    h = ((ta * 0x9E3779B1) & 0xFFFFFFFF) >> 19
    for x in range(65, 123):
        for y in range(65, 123):
            for z in range(65, 123):
                t = x | y << 8 | z << 16
                if t != ta and ((t * 0x9E3779B1) & 0xFFFFFFFF) >> 19 == h:
                    return bytes([x, y, z])
    raise AssertionError("no collision")


@pytest.mark.parametrize("lazy", [False, True])
def test_exhaustive_deferred_walks(lazy):
    """A rare trigram in the bucket of a common one: the nearest earlier entry with the same
    trigram lies hundreds of bucket entries down, so the gram pass lists the walk and walks it
    a wave per entry (the path that hung in round 4 when its work counter was claimed by lane 0
    only).  Tokens equal the oracle's."""
    rng = np.random.default_rng(9)
    a = b"qzv"
    b = _colliding_trigram(a)
    parts = []
    for n in range(3000):
        parts.append(a + bytes([int(rng.integers(48, 58))]))
        if n % 150 == 75:
            parts.append(b + bytes([int(rng.integers(97, 123))]))
    data = b"".join(parts)
    _check(data, 32768, lazy)
    _check(data, 4096, lazy)
