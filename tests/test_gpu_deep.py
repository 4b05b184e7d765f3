"""DMX_F_DEEP on the MI355X: the adaptive chain depth through the C-ABI.

Bar: bit-exact.  Streams byte-identical to the oracle's (tests/test_deep.py pins the
oracle's block rule against an independent numpy statement); tokens per block equal the
oracle's parse at the block's depth; every stream inflates.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.deep_inputs import inputs  # noqa: E402


@pytest.fixture(scope="module")
def enc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = D.Encoder(0, 8 << 20)
    yield e
    e.close()


@pytest.mark.parametrize("name", sorted(inputs()))
@pytest.mark.parametrize("k,lazy", [(8, True), (8, False), (6, True), (7, True), (4, False), (1, True), (32, True)])
def test_deep_streams_match_oracle(enc, name, k, lazy):
    data = inputs()[name]
    fl = D.DMX_ZLIB | D.DMX_F_DEEP | (D.DMX_F_LAZY if lazy else 0)
    z, r = enc.compress_bytes(data, max_chain=k, flags=fl)
    assert z == O.compress(data, max_chain=k, lazy=lazy, deep=True), (name, k, lazy)
    assert zlib.decompress(z) == data


@pytest.mark.parametrize("name", sorted(inputs()))
def test_deep_headline_parse(enc, name):
    """The bench's parse: K=7, lazy, adaptive depth and the noise check together."""
    data = inputs()[name]
    fl = D.DMX_ZLIB | D.DMX_F_DEEP | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
    z, r = enc.compress_bytes(data, max_chain=7, flags=fl)
    assert z == O.compress(data, max_chain=7, lazy=True, deep=True, store_check=True), name
    assert zlib.decompress(z) == data


def test_deep_tokens_per_block(enc):
    data = inputs()["mixed"]
    enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_DEEP | D.DMX_F_LAZY)
    depths = set()
    for b, o in enumerate(range(0, len(data), 32768)):
        blk = data[o:o + 32768]
        depths.add(O.block_chain(blk, 8))
        assert np.array_equal(enc.tokens(b), O.parse_block(blk, 8, lazy=True, deep=True)), b
    assert depths == {8, 32}   # both kinds of block in one launch (DMX_DEEP_CHAIN = 32)


@pytest.mark.parametrize("sw", [4096, 2049, 300])
def test_deep_small_windows(enc, sw):
    data = inputs()["mixed"][:120000]
    fl = D.DMX_ZLIB | D.DMX_F_DEEP | D.DMX_F_LAZY
    z, _ = enc.compress_bytes(data, sw=sw, max_chain=8, flags=fl)
    assert z == O.compress(data, sw=sw, max_chain=8, lazy=True, deep=True)


@pytest.mark.parametrize("extra", ["dict", "split", "store_check", "exact_sort"])
def test_deep_with_block_options(enc, extra):
    data = inputs()["mixed"]
    fl = D.DMX_ZLIB | D.DMX_F_DEEP | D.DMX_F_LAZY
    kw = {}
    if extra == "dict":
        fl |= D.DMX_F_DICT
        kw["dict"] = True
    elif extra == "split":
        fl |= D.DMX_F_SPLIT
        kw["split"] = True
    elif extra == "store_check":
        fl |= D.DMX_F_STORE_CHECK
        kw["store_check"] = True
    else:
        fl |= D.DMX_F_EXACT_SORT
    z, _ = enc.compress_bytes(data, max_chain=8, flags=fl)
    assert z == O.compress(data, max_chain=8, lazy=True, deep=True, **kw), extra
    assert zlib.decompress(z) == data


def test_deep_off_for_exhaustive_and_long_chains(enc):
    """max_chain 0 (the reference parse) and K >= the depth (32) ignore the flag."""
    data = inputs()["bitdump"][:70000]
    for k in (0, 32, 64, 100):
        z, _ = enc.compress_bytes(data, max_chain=k, flags=D.DMX_ZLIB | D.DMX_F_DEEP)
        assert z == O.compress(data, max_chain=k), k


@pytest.mark.parametrize("depth", [16, 24, 48, 64])
def test_deep_chain_depths(enc, depth):
    """dmx_opts.deep_chain: small-alphabet blocks search `depth` deep (the oracle at the same
    depth, dmx_oracle_set_deep_chain), at the headline parse."""
    data = inputs()["mixed"]
    fl = D.DMX_ZLIB | D.DMX_F_DEEP | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    O.set_deep_chain(depth)
    try:
        z, _ = enc.compress_tensor(t, opts=D.Opts(32768, 7, fl, depth))
        assert z.cpu().numpy().tobytes() == O.compress(data, max_chain=7, lazy=True, deep=True, store_check=True)
    finally:
        O.set_deep_chain(0)
