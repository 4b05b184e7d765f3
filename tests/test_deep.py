"""DMX_F_DEEP on the CPU: the oracle's adaptive chain depth (dmx_oracle_block_chain) against
an independent numpy statement of the rule, and its effect on size."""
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from tests.deep_inputs import bitdump, inputs

DEEP_K = 32   # DMX_DEEP_CHAIN (round 5; 64 before)


def rule(block: bytes, k: int) -> int:
    """Independent statement: D distinct 13-bit buckets among the trigram positions p < n - 2
    with p mod 2048 < 256; the block searches DEEP_K deep when 4 D < samples."""
    if k <= 0 or k >= DEEP_K:
        return k
    a = np.frombuffer(block, dtype=np.uint8).astype(np.uint64)
    nv = max(a.size - 2, 0)
    p = np.arange(nv)
    p = p[(p % 2048) < 256]
    if p.size == 0:
        return k
    t = a[p] | (a[p + 1] << np.uint64(8)) | (a[p + 2] << np.uint64(16))
    h = ((t * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)) >> np.uint64(19)
    return DEEP_K if 4 * np.unique(h).size < p.size else k


@pytest.mark.parametrize("name", sorted(inputs()))
@pytest.mark.parametrize("k", [1, 6, 8, 32, 63, 64, 0])
def test_block_chain_rule(name, k):
    data = inputs()[name]
    for o in range(0, len(data), 32768):
        blk = data[o:o + 32768]
        assert O.block_chain(blk, k) == rule(blk, k), (name, o)


def test_rule_selects_small_alphabets_only():
    d = inputs()
    for name in ("bitdump", "bin01", "dna", "hex"):
        assert O.block_chain(d[name][:32768], 8) == DEEP_K, name
    assert O.block_chain(d["text"][:32768], 8) == 8
    bee = open("tests/golden/bee_movie_script.txt", "rb").read()
    assert O.block_chain(bee[:32768], 8) == 8


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 256, 257, 258, 259, 2048, 2050, 2304, 4096, 32767, 32768])
def test_block_chain_edge_sizes(n):
    blk = bitdump(n, 9)
    assert O.block_chain(blk, 8) == rule(blk, 8), n
    txt = (b"the quick brown fox jumps over the lazy dog " * 800)[:n]
    assert O.block_chain(txt, 6) == rule(txt, 6), n


@pytest.mark.parametrize("lazy", [False, True])
def test_deep_parse_equals_deep_k_on_deep_blocks(lazy):
    """A deep block's parse is the K = DEEP_K parse; a text block's is the K parse."""
    d = inputs()
    for name in ("bitdump", "text"):
        blk = d[name][:32768]
        k = O.block_chain(blk, 8)
        assert np.array_equal(O.parse_block(blk, 8, lazy=lazy, deep=True), O.parse_block(blk, k, lazy=lazy))


def test_deep_streams_inflate_and_shrink():
    d = inputs()
    for name in ("bitdump", "hex", "mixed"):
        data = d[name]
        z8 = O.compress(data, max_chain=8, lazy=True)
        zd = O.compress(data, max_chain=8, lazy=True, deep=True)
        assert zlib.decompress(zd) == data
        assert len(zd) < len(z8), name
        if name != "mixed":   # every block deep: the K = DEEP_K stream
            assert zd == O.compress(data, max_chain=DEEP_K, lazy=True), name
    # with dict and split too
    data = d["mixed"]
    for kw in (dict(dict=True), dict(split=True), dict(store_check=True)):
        z = O.compress(data, max_chain=8, lazy=True, deep=True, **kw)
        assert zlib.decompress(z) == data
        assert z == O.compress_par(data, max_chain=8, lazy=True, deep=True, threads=4, **kw)


def test_oracle_deep_chain_setting():
    """dmx_oracle_set_deep_chain (the GPU's dmx_opts.deep_chain): a deep block gets that depth,
    0 restores DEEP_K; K >= the depth is left alone."""
    from tests.deep_inputs import inputs
    blk = inputs()["bitdump"][:32768]
    try:
        assert O.block_chain(blk, 7) == DEEP_K
        O.set_deep_chain(24)
        assert O.block_chain(blk, 7) == 24
        assert O.block_chain(blk, 30) == 30
    finally:
        O.set_deep_chain(0)
    assert O.block_chain(blk, 7) == DEEP_K
