"""C5's shape on one MI355X: the input cut into 8 block-aligned shards
(shard_range), each encoded by the HIP path with the multi-GPU framing (shard_flags: zlib
header on shard 0, sync flush after every shard but the last, BFINAL on the last), byte-equal
to the oracle's shard stream with the same framing, stitched with the combined Adler-32 and
inflated by zlib and by our deflate_decompress.  One GPU encodes the shards one after the
other -- exactly what each rank of `bench.py --gpus 8 --workload enwik9` encodes.
Also C4 at its stated size (1 GiB, 32 768 blocks) through the stored path."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from deflate_compression_amd import shard as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

WORLD = 8


def _encode_shards(host: np.ndarray, max_chain: int, flags: int, dict_halo: bool, enc):
    """Per shard: (gpu chunk bytes, adler, length) with the shard framing."""
    n = host.size
    d_all = torch.from_numpy(host).cuda()
    out = []
    for r in range(WORLD):
        lo, hi = S.shard_range(n, r, WORLD)
        o = D.Opts(32768, max_chain, flags | S.shard_flags(r, WORLD), 0)
        if dict_halo and lo > 0:   # the block before the shard: exchange_history's bytes
            o.dict, o.dict_len = d_all[lo - min(32768, lo):lo].data_ptr(), min(32768, lo)
        t = d_all[lo:hi] if hi > lo else torch.empty(0, dtype=torch.uint8, device="cuda")
        z, res = enc.compress_tensor(t, opts=o)
        out.append((z.cpu().numpy().tobytes(), int(res.adler), hi - lo))
    return out


def _stitch(parts):
    return b"".join(p[0] for p in parts) + S.trailer(S.combine_adler([p[1] for p in parts], [p[2] for p in parts]))


@pytest.mark.parametrize("cfg", ["bench", "exhaustive", "dict", "split"])
def test_c5_shape_8_shards_vs_oracle(cfg):
    n = 8 * 3 * 32768 + 12345   # 25 blocks: shards of 3 or 4 blocks, a short tail
    host = D.gen_text(n, 0xE5819)
    kw = {"bench": dict(max_chain=7, lazy=True, store_check=True, deep=True), "exhaustive": dict(max_chain=0),
          "dict": dict(max_chain=6, lazy=True, dict=True), "split": dict(max_chain=8, lazy=True, split=True)}[cfg]
    flags = (D.DMX_F_LAZY if kw.get("lazy") else 0) | (D.DMX_F_STORE_CHECK if kw.get("store_check") else 0) | \
            (D.DMX_F_DICT if kw.get("dict") else 0) | (D.DMX_F_SPLIT if kw.get("split") else 0) | \
            (D.DMX_F_DEEP if kw.get("deep") else 0)
    e = D.Encoder(0, n)
    try:
        parts = _encode_shards(host, kw["max_chain"], flags, bool(kw.get("dict")), e)
    finally:
        e.close()
    for r, (z, ad, ln) in enumerate(parts):
        lo, hi = S.shard_range(n, r, WORLD)
        pre = host[max(0, lo - 32768):lo] if kw.get("dict") else None
        zo = O.compress(host[lo:hi], flags=S.shard_flags(r, WORLD), pre=pre, **kw)
        assert z == zo, (cfg, r, len(z), len(zo))
        assert ad == zlib.adler32(host[lo:hi].tobytes())
    stream = _stitch(parts)
    data = host.tobytes()
    assert zlib.decompress(stream) == data
    assert D.deflate_decompress(stream) == data


def test_c5_full_size_8_shards():
    """C5 at its stated size: 1 000 000 000 B of enwik9-style text, 8 shards (3 815 blocks
    each, the last 3 814 with the 18 944 B tail) at the bench parse: K=7 lazy + adaptive
    depth + store check; every shard byte-equal to the oracle's (its OpenMP form), the
    stitched stream inflates."""
    n = 1_000_000_000
    host = D.gen_text(n, 0xE5819)
    flags = D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    e = D.Encoder(0, n // WORLD + 32768)
    try:
        parts = _encode_shards(host, 7, flags, False, e)
    finally:
        e.close()
    for r, (z, _, _) in enumerate(parts):
        lo, hi = S.shard_range(n, r, WORLD)
        assert z == O.compress_par(host[lo:hi], max_chain=7, lazy=True, store_check=True, deep=True,
                                   flags=S.shard_flags(r, WORLD), threads=16), r
    d = zlib.decompressobj()
    out = d.decompress(_stitch(parts)) + d.flush()
    assert d.eof and out == host.tobytes()


def test_c4_full_size_1gib_round_trip():
    """C4 at its stated size: 1 GiB of splitmix64 (32 768 blocks), every block stored by the
    noise check: stream length = 2 + 32 768 x (32 768 + 5) + 4, zlib round trip, and the
    indexed GPU inflate of all 32 768 blocks bit-exact."""
    n = 1 << 30
    host = D.gen_random(n, 0x5EED)
    e = D.Encoder(0, n)
    try:
        d_in = torch.from_numpy(host).to("cuda:0")
        o = D.Opts(32768, 6, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK, 0)
        z_t, res = e.compress_tensor(d_in, opts=o)
        nblk = n // 32768
        assert res.nblocks == nblk and res.nstored == nblk
        assert res.out_len == 2 + nblk * (32768 + 5) + 4
        z = z_t[:res.out_len].cpu().numpy().tobytes()
        assert zlib.decompress(z) == host.tobytes()
        ix, nb = e.block_index()
        assert nb == nblk
        out, st = D.inflate_gpu(z_t[:res.out_len], n, index=ix, nblk=nb)
        assert st == 0 and out.numel() == n
        assert torch.equal(out, d_in)
    finally:
        e.close()
