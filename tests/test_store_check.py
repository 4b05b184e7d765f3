"""DMX_F_STORE_CHECK: noise blocks are emitted stored without a parse.

CPU: the oracle's rule (oracle/dmx_oracle.c, dmx_oracle_store_check) against an
independent numpy statement of the same integer rule; streams with the check inflate
and differ from the unchecked stream only in the blocks the rule stores.
GPU (-m gpu): streams byte-identical to the oracle's with the check, on inputs built to
land on both sides of each test (flat/skewed histograms, few/many 4-byte repeats, short
blocks), with lazy, split and dict; the fd API; GPU inflate; 256 MiB noise round trip.
"""
import os
import zlib

import numpy as np
import pytest

import deflate_compression_amd as D
from oracle import oracle as O


def np_store_check(block) -> bool:
    """The §4.7 rule, restated in numpy (independent of the C oracle)."""
    b = np.frombuffer(bytes(block), dtype=np.uint8)
    n = b.size
    if n < 4096:
        return False
    bits = np.unpackbits(b[:4096, None], axis=1)
    if np.any(8 * np.abs(2 * bits.sum(axis=0).astype(np.int64) - 4096) > 4096):
        return False
    sh = 3 if n >= 32768 else 2 if n >= 16384 else 1 if n >= 8192 else 0
    h = np.bincount(b[0::1 << sh], minlength=256).astype(np.uint64)
    s2 = int((h * h).sum())
    m = (n + (1 << sh) - 1) >> sh
    if 256 * s2 > m * m + ((m * m) >> 4) + 256 * m:
        return False
    w = (b[:-3].astype(np.uint64) | b[1:-2].astype(np.uint64) << 8 | b[2:-1].astype(np.uint64) << 16
         | b[3:].astype(np.uint64) << 24)
    x = (w * 0x9E3779B1) & 0xFFFFFFFF
    g = x[(x & (7 << 11)) == 0] >> 15
    q = g.size
    coll = q - np.unique(g).size
    return 16 * q >= n and 64 * coll <= 4 * q


def _noise(n, seed, alphabet=256):
    r = np.random.default_rng(seed)
    return r.integers(0, alphabet, n, dtype=np.uint16).astype(np.uint8).tobytes()


def _noise_with_repeats(n, seed, frac):
    """Noise in which a fraction `frac` of the bytes are copies of earlier 64-byte pieces."""
    a = bytearray(_noise(n, seed))
    r = np.random.default_rng(seed + 1)
    for _ in range(int(n * frac) // 64):
        src = int(r.integers(0, n - 64))
        dst = int(r.integers(0, n - 64))
        a[dst:dst + 64] = a[src:src + 64]
    return bytes(a)


def cases():
    """Blocks chosen to sit on both sides of each test of the rule."""
    text = D.gen_text(40000, 5).tobytes()
    return {
        "noise": _noise(32768, 1),
        "noise_248": _noise(32768, 2, 248),       # flat enough (256/248 = 1.032)
        "noise_232": _noise(32768, 3, 232),       # too skewed (256/232 = 1.10)
        "noise_rep1": _noise_with_repeats(32768, 4, 0.01),
        "noise_rep8": _noise_with_repeats(32768, 5, 0.08),
        "cycle": bytes(range(256)) * 128,         # flat histogram, all repeats
        "noise_7bit": _noise(32768, 9, 128),      # bit 7 never set: fails the bit-plane test
        "noise_hi": bytes(x | 0x40 if i % 3 == 0 else x for i, x in enumerate(_noise(32768, 10))),
        "zeros": bytes(32768),
        "text": text[:32768],
        "short_4095": _noise(4095, 6),
        "short_4096": _noise(4096, 7),
        "short_9000": _noise(9000, 8),
    }


def test_rule_matches_numpy_statement():
    seen = set()
    for name, blk in cases().items():
        a, b = O.store_check(blk), np_store_check(blk)
        assert a == b, name
        seen.add(a)
    assert seen == {True, False}
    for seed in range(20):   # many noise blocks: all pass, with margin on both statistics
        assert O.store_check(_noise(32768, 100 + seed))


def test_expected_decisions():
    c = cases()
    want = {"noise": True, "noise_248": True, "noise_232": False, "noise_rep1": True, "noise_rep8": False,
            "cycle": False, "noise_7bit": False, "noise_hi": False, "zeros": False, "text": False, "short_4095": False, "short_4096": True,
            "short_9000": True}
    for k, v in want.items():
        assert O.store_check(c[k]) == v, k


def mixed_input():
    c = cases()
    order = ["noise", "text", "noise_248", "noise_232", "cycle", "noise_7bit", "noise_hi", "noise_rep1", "noise_rep8", "zeros", "noise"]
    return b"".join(c[k] for k in order) + c["short_9000"]


@pytest.mark.parametrize("kw", [dict(), dict(max_chain=8, lazy=True), dict(max_chain=8, lazy=True, split=True),
                                dict(max_chain=8, lazy=True, dict=True)])
def test_oracle_stream(kw):
    data = mixed_input()
    z, bt = O.compress(data, store_check=True, want_btypes=True, **kw)
    assert zlib.decompress(z) == data
    z0, bt0 = O.compress(data, store_check=False, want_btypes=True, **kw)
    checked = [O.store_check(data[o:o + 32768]) for o in range(0, len(data), 32768)]
    assert any(checked) and not all(checked)
    for k, c in enumerate(checked):
        if c:
            assert bt[k] == 0
    if not kw.get("dict"):   # without history the unchecked blocks are coded the same way
        assert all(bt[k] == bt0[k] for k, c in enumerate(checked) if not c)
    # noise: the checked stream is never much larger than the parsed one
    assert len(z) <= len(z0) * 1.002 + 64


# ---------------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = D.Encoder(0, 8 << 20)
    yield e
    e.close()


@gpu
@pytest.mark.parametrize("k,lazy,split,dct", [(0, False, False, False), (8, True, False, False), (8, True, True, False),
                                               (8, True, False, True), (4, False, True, True)])
def test_gpu_stream_equals_oracle(enc, k, lazy, split, dct):
    data = mixed_input()
    fl = D.DMX_ZLIB | D.DMX_F_STORE_CHECK | (D.DMX_F_LAZY if lazy else 0) | (D.DMX_F_SPLIT if split else 0) | \
        (D.DMX_F_DICT if dct else 0)
    z, _ = enc.compress_bytes(data, max_chain=k, flags=fl)
    assert z == O.compress(data, max_chain=k, lazy=lazy, split=split, dict=dct, store_check=True)
    assert zlib.decompress(z) == data
    assert D.compress(data, max_chain=k, lazy=lazy, split=split, dict=dct, store_check=True) == z


@gpu
@pytest.mark.parametrize("sw", [1024, 4096, 5000, 32767])
def test_gpu_windows_and_edges(enc, sw):
    data = mixed_input()[:200003]
    for n in (0, 1, 4095, 4096, 4097, sw, sw + 1, 3 * sw + 999, len(data)):
        d = data[:n]
        z, _ = enc.compress_bytes(d, sw=sw, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_STORE_CHECK | D.DMX_F_LAZY)
        assert z == O.compress(d, sw=sw, max_chain=8, lazy=True, store_check=True), (sw, n)


@gpu
def test_gpu_state_not_stale(enc):
    """A checked encode (noise stored) followed by an unchecked one on the same context:
    the second must parse every block (no stale stored marks)."""
    data = mixed_input()
    enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_STORE_CHECK)
    z, _ = enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB | D.DMX_F_SPLIT)
    assert z == O.compress(data, max_chain=8, split=True)
    z, _ = enc.compress_bytes(data, max_chain=8, flags=D.DMX_ZLIB)
    assert z == O.compress(data, max_chain=8)


@gpu
def test_gpu_fd_api_and_inflate(tmp_path):
    data = mixed_input() * 3
    fi, fo = tmp_path / "in", tmp_path / "out"
    fi.write_bytes(data)
    env = {"DMX_STORE_CHECK": "1", "DMX_MAX_CHAIN": "8", "DMX_LAZY": "1", "DMX_CHUNK_MB": "4"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with open(fi, "rb") as a, open(fo, "wb") as b:
            assert D.deflate_compress(a.fileno(), b.fileno(), -1, 32768, 0) == 0
    finally:
        for k, v in old.items():
            os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)
    z = fo.read_bytes()
    assert zlib.decompress(z) == data
    assert z == O.compress(data, max_chain=8, lazy=True, store_check=True)


@gpu
def test_gpu_noise_256mib_round_trip():
    """At size: every noise block stored (ratio = 1 + framing), zlib and GPU inflate exact."""
    torch = pytest.importorskip("torch")
    n = 256 << 20
    host = D.gen_random(n, 0x5EED)
    e = D.Encoder(0, n)
    try:
        d_in = torch.from_numpy(host).to("cuda:0")
        o = D.Opts(32768, 8, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK, 0)
        z_t, res = e.compress_tensor(d_in, opts=o)
        nblk = n // 32768
        assert res.out_len == 2 + nblk * (32768 + 5) + 4
        z = z_t[:res.out_len].cpu().numpy().tobytes()
        assert zlib.decompress(z) == host.tobytes()
        ix, nb = e.block_index()
        assert nb == nblk
        out, st = D.inflate_gpu(z_t[:res.out_len], n, index=ix, nblk=nb)
        assert st == 0
        assert torch.equal(out.cpu(), torch.from_numpy(host))
    finally:
        e.close()
