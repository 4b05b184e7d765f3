"""Work lists of DMX_F_STORE_CHECK (dmx_worklist_kernel): K1 / K2 / K4 take only
the blocks they have work for, the prefix of noise blocks at their speculative offsets is
written whole by K0 and skipped by K4.  Every launch shape (DMX_WORKLIST=list: the persistent
K1 and the list-striding K2 / K4; =plain: a workgroup per block with the skip; =0: no work
lists) must write the oracle's stream byte for byte, and the adaptive choice (the previous
encode's hint) too, whatever it picks.

Bar: bit-exact against the oracle (store_check=True), zlib inflates."""
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import deflate_compression_amd as D  # noqa: E402
from deflate_compression_amd import shard as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

B = 32768


def _noise(n, seed):
    return D.gen_random(n, seed).tobytes()


def _cases():
    text = D.gen_text(6 * B, 77).tobytes()
    z = bytes(3 * B)
    return {
        "all_noise": _noise(9 * B, 1),
        "noise_prefix_then_text": _noise(5 * B, 2) + text[:3 * B] + _noise(2 * B + 777, 3),
        "text_in_noise": _noise(3 * B, 4) + text[:B] + _noise(4 * B, 5),
        "noise_zeros_text": _noise(2 * B, 6) + z + text[:2 * B] + _noise(B + 100, 7),
        "text_only": text,
        "noise_short_tail": _noise(4 * B + 5000, 8),
        # a 1- / 2- / 3-byte last block after a stored prefix: its fixed-Huffman bits share a
        # word with the prefix's last bytes (the apply launch and the tail zeroing
        # must keep those bytes)
        "noise_1byte_tail": _noise(3 * B + 1, 16),
        "noise_2byte_tail": _noise(5 * B + 2, 17),
        "noise_3byte_tail": _noise(2 * B + 3, 18),
        "one_block_noise": _noise(B, 9),
        "two_blocks_noise": _noise(2 * B, 10),
    }


@pytest.fixture(scope="module")
def enc():
    e = D.Encoder(0, 16 << 20)
    yield e
    e.close()


def _with_shape(e, val, fn):
    """fn() with the context's launch shapes forced (dmx_ctx_set_hook; None = adaptive)."""
    e.set_hook("worklist", val)
    try:
        return fn()
    finally:
        e.set_hook("worklist", None)


def _with_hook(e, name, val, fn):
    e.set_hook(name, val)
    try:
        return fn()
    finally:
        e.set_hook(name, None if name == "dedupe" else 0)


@pytest.mark.parametrize("shape", ["list", "plain", "0", None])
@pytest.mark.parametrize("name", sorted(_cases()))
def test_worklist_shapes_match_oracle(enc, shape, name):
    data = _cases()[name]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    want = O.compress(data, max_chain=7, lazy=True, store_check=True, deep=True)
    for rep in range(2):   # the second encode on the context follows the first one's hint
        z, r = _with_shape(enc, shape, lambda: enc.compress_bytes(data, max_chain=7, flags=fl))
        assert r.status == 0
        assert z == want, (name, shape, rep, len(z), len(want))
    assert zlib.decompress(z) == data


@pytest.mark.parametrize("shape", ["list", "plain"])
@pytest.mark.parametrize("k", [0, 8])
def test_worklist_exhaustive_and_greedy(enc, shape, k):
    data = _cases()["noise_prefix_then_text"]
    z, _ = _with_shape(enc, shape, lambda: enc.compress_bytes(data, max_chain=k, flags=D.DMX_ZLIB | D.DMX_F_STORE_CHECK))
    assert z == O.compress(data, max_chain=k, store_check=True)


@pytest.mark.parametrize("shape", ["list", "plain"])
@pytest.mark.parametrize("sw", [8192, 20000])
def test_worklist_small_windows(enc, shape, sw):
    data = _noise(6 * sw, 11) + D.gen_text(3 * sw, 12).tobytes() + _noise(2 * sw + 9, 13)
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
    z, _ = _with_shape(enc, shape, lambda: enc.compress_bytes(data, sw=sw, max_chain=6, flags=fl))
    assert z == O.compress(data, sw=sw, max_chain=6, lazy=True, store_check=True)


@pytest.mark.parametrize("shape", ["list", "plain"])
def test_worklist_shard_framing(enc, shape):
    """Shards without the zlib header (speculative offsets from bit 0) and without BFINAL."""
    data = np.frombuffer(_noise(6 * B, 14) + D.gen_text(2 * B, 15).tobytes(), dtype=np.uint8)
    for r in range(3):
        lo, hi = S.shard_range(data.size, r, 3)
        fl = D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | S.shard_flags(r, 3)
        piece = data[lo:hi]
        t = torch.from_numpy(piece.copy()).cuda()
        z, _ = _with_shape(enc, shape, lambda: enc.compress_tensor(t, opts=D.Opts(B, 7, fl, 0)))
        assert z.cpu().numpy().tobytes() == O.compress(piece, max_chain=7, lazy=True, store_check=True,
                                                        flags=S.shard_flags(r, 3)), (shape, r)


def test_worklist_with_dict_and_split(enc):
    data = _cases()["noise_prefix_then_text"]
    for shape in ("list", "plain"):
        z, _ = _with_shape(enc, shape, lambda: enc.compress_bytes(
            data, max_chain=7, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DICT))
        assert z == O.compress(data, max_chain=7, lazy=True, store_check=True, dict=True), shape
        z, _ = _with_shape(enc, shape, lambda: enc.compress_bytes(
            data, max_chain=7, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_SPLIT))
        assert z == O.compress(data, max_chain=7, lazy=True, store_check=True, split=True), shape


def test_worklist_inflate_gpu(enc):
    """The indexed GPU inflate of a stream whose noise prefix K0 wrote whole."""
    data = _cases()["noise_prefix_then_text"]
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    out, r = _with_shape(enc, "list", lambda: enc.compress_tensor(
        t, opts=D.Opts(B, 7, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK, 0)))
    ix, n = enc.block_index()
    dec, st = D.inflate_gpu(out, len(data), ix, n)
    assert st == 0 and dec.cpu().numpy().tobytes() == data


def _uniform_cases():
    runs = b"".join(bytes([v]) * B for v in (0, 0, 7, 0, 255, 7, 7, 0))
    return {
        "zeros": bytes(10 * B),
        "zeros_tail": bytes(6 * B + 12345),
        "runs_of_bytes": runs + bytes([9]) * 500,
        "uniform_in_noise": _noise(2 * B, 21) + bytes(4 * B) + _noise(B, 22) + bytes([65]) * (3 * B) + b"x",
        "uniform_and_text": bytes(3 * B) + D.gen_text(2 * B, 23).tobytes() + bytes(3 * B) + D.gen_text(B, 24).tobytes(),
    }


@pytest.mark.parametrize("shape", ["list", "plain", None])
@pytest.mark.parametrize("name", sorted(_uniform_cases()))
def test_uniform_dedupe_matches_oracle(enc, shape, name):
    """DMX_DEDUPE=1: full blocks of one byte value (block 1 .. nblk - 2) are coded once per byte
    value and copied bit for bit to their offsets (dmx_dup_copy_kernel) -- the stream is the
    oracle's; =0 the same stream without the dedupe."""
    data = _uniform_cases()[name]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    want = O.compress(data, max_chain=7, lazy=True, store_check=True, deep=True)
    for dd in (1, 0):
        z, r = _with_hook(enc, "dedupe", dd,
                          lambda: _with_shape(enc, shape, lambda: enc.compress_bytes(data, max_chain=7, flags=fl)))
        assert r.status == 0
        assert z == want, (name, shape, dd, len(z), len(want))
    assert zlib.decompress(z) == data


def test_uniform_dedupe_inflate_and_split(enc):
    data = _uniform_cases()["uniform_in_noise"]
    enc.set_hook("dedupe", 1)
    try:
        t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
        out, r = enc.compress_tensor(t, opts=D.Opts(B, 7, D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK, 0))
        ix, n = enc.block_index()
        dec, st = D.inflate_gpu(out, len(data), ix, n)
        assert st == 0 and dec.cpu().numpy().tobytes() == data
        z, _ = enc.compress_bytes(data, max_chain=7, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_SPLIT)
        assert z == O.compress(data, max_chain=7, lazy=True, store_check=True, split=True)
    finally:
        enc.set_hook("dedupe", None)


def _multi_tile(sw):
    """Over 3 worklist tiles (WLC x WLT = 4 096 blocks each) of sw-byte blocks: a noise prefix
    that crosses the first tile, uniform runs of byte values that recur in later tiles (their
    representatives in an earlier tile), text blocks, a short tail."""
    rng = np.random.default_rng(31)
    parts, seed = [], 40

    def noise(k):
        nonlocal seed
        seed += 1
        parts.append(_noise(k * sw, seed))

    noise(5000)
    parts.append(bytes(200 * sw))
    noise(100)
    parts.append(D.gen_text(40 * sw, 41).tobytes())
    parts.append(bytes([7]) * (300 * sw))
    noise(3000)
    parts.append(bytes(100 * sw))
    parts.append(bytes([7]) * (100 * sw) + bytes([200]) * (50 * sw))
    parts.append(D.gen_text(20 * sw, 42).tobytes())
    noise(4000)
    parts.append(rng.integers(0, 256, 777, dtype=np.uint8).tobytes())
    return b"".join(parts)


@pytest.mark.parametrize("shape", ["list", None])
def test_worklist_multi_tile(shape):
    """The list builder's workgroups each count the blocks before their tile: lists, the stored
    prefix M, the dups and their representatives across tiles (DMX_DEDUPE 1 and 0) -- the
    oracle's stream byte for byte."""
    sw = 4096
    data = _multi_tile(sw)
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
    want = O.compress(data, sw=sw, max_chain=7, lazy=True, store_check=True)
    e = D.Encoder(0, len(data), sw=sw)
    try:
        e.set_hook("worklist", shape)
        for dd in (1, 0):
            e.set_hook("dedupe", dd)
            for rep in range(2):
                z, r = e.compress_bytes(data, sw=sw, max_chain=7, flags=fl)
                assert r.status == 0
                assert z == want, (shape, dd, rep, len(z), len(want))
    finally:
        e.close()


def test_stage_timing_modes():
    """set_timing: every stage boundary evented, or only one stage's two events (bench.py's
    timed region); the stream is the same either way."""
    data = _cases()["noise_prefix_then_text"]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    e = D.Encoder(0, len(data), max_chain=7, flags=fl)
    try:
        want = O.compress(data, max_chain=7, lazy=True, store_check=True, deep=True)
        e.set_timing(True)
        for _ in range(3):
            z, _ = e.compress_bytes(data, max_chain=7, flags=fl)
            assert z == want
        st, cnt = e.stage_times()
        assert cnt == 3 and all(st[k] > 0 for k in ("pre", "match", "huff", "scan", "pack", "total"))
        for stage in D.Encoder.STAGES:
            e.set_timing(True, stage=stage)
            z, _ = e.compress_bytes(data, max_chain=7, flags=fl)
            assert z == want
            st, cnt = e.stage_times()
            assert cnt == 1 and st[stage] > 0, (stage, st)
            assert all(v == 0 for k, v in st.items() if k != stage), (stage, st)
        e.set_timing(True, stage="match", every=3)   # events on encodes 0, 3, 6 of 7
        for _ in range(7):
            z, _ = e.compress_bytes(data, max_chain=7, flags=fl)
            assert z == want
        st, cnt = e.stage_times()
        assert cnt == 3 and st["match"] > 0
        e.set_timing(False)
    finally:
        e.close()


@pytest.mark.parametrize("shift", [1, 4, 8])
@pytest.mark.parametrize("shape", ["list", None])
def test_worklist_unaligned_input(enc, shape, shift):
    """A device input that is not 16-byte aligned: K0 takes its general path (no register
    copy) and the fill kernel writes the rest of the stored prefix; the stream is the oracle's."""
    data = _cases()["noise_prefix_then_text"]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    want = O.compress(data, max_chain=7, lazy=True, store_check=True, deep=True)
    buf = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
    buf[shift:shift + len(data)] = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    t = buf[shift:shift + len(data)]
    assert t.data_ptr() % 16 == shift % 16
    for rep in range(2):
        z, r = _with_shape(enc, shape, lambda: enc.compress_tensor(t, opts=D.Opts(B, 7, fl, 0)))
        assert r.status == 0
        assert z.cpu().numpy().tobytes() == want, (shape, shift, rep)


@pytest.mark.parametrize("name", ["noise_prefix_then_text", "text_only", "noise_zeros_text"])
def test_scan_paths_agree(enc, name):
    """K3's fused scan + apply launch (up to 1 024 tiles) and the three-launch scan
    (DMX_SCAN3=1, every size above that) write the same stream -- the oracle's."""
    data = _cases()[name]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    want = O.compress(data, max_chain=7, lazy=True, store_check=True, deep=True)
    try:
        for v in (1, 0):
            enc.set_hook("scan3", v)
            for rep in range(2):
                z, r = enc.compress_bytes(data, max_chain=7, flags=fl)
                assert r.status == 0 and z == want, (name, v, rep)
                assert r.nblocks == (len(data) + B - 1) // B and r.adler == zlib.adler32(data)
    finally:
        enc.set_hook("scan3", 0)


def _many_blocks(nblk, sw, seed):
    """nblk blocks of sw bytes, mostly zeros (cheap for the oracle), with text and noise
    runs spread over every scan tile, and a ragged tail."""
    rng = np.random.default_rng(seed)
    a = np.zeros(nblk * sw - sw // 3, dtype=np.uint8)
    text = D.gen_text(64 * sw, seed)
    for s in range(0, nblk - 64, 331):
        k = int(rng.integers(1, 32))
        if rng.integers(0, 2):
            a[s * sw:(s + k) * sw] = text[:k * sw]
        else:
            a[s * sw:(s + k) * sw] = rng.integers(0, 256, k * sw, dtype=np.uint8)
    return a


@pytest.mark.parametrize("sw,ntile", [(4096, 257), (1024, 1025)])
def test_scan_many_tiles(sw, ntile):
    """K3 above 65 536 blocks: the fused launch's threads compose C = 2 tile aggregates each
    (257 tiles), and just past its 1 024-tile limit the three-launch path takes over (1 025
    tiles) -- both the oracle's stream, with DMX_SCAN3 forced and not."""
    import time
    hb = os.environ.get("DMX_TEST_HEARTBEAT")   # progress for a watchdog (each step names itself)

    def beat(msg):
        if hb:
            with open(hb, "a") as h:
                h.write(f"scan_many_tiles sw={sw} ntile={ntile}: {msg} {time.time():.1f}\n")

    nblk = ntile * 256 - 100
    a = _many_blocks(nblk, sw, 5 + ntile)
    assert (a.size + sw - 1) // sw == nblk and (nblk + 255) // 256 == ntile
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK
    beat("input")
    want = O.compress_par(a, sw=sw, max_chain=4, lazy=True, store_check=True, threads=8)
    beat("oracle")
    e = D.Encoder(0, a.size, sw=sw)
    try:
        t = torch.from_numpy(a).cuda()
        for v in (1, 0):
            e.set_hook("scan3", v)
            for rep in range(2):
                z, r = e.compress_tensor(t, opts=D.Opts(sw, 4, fl, 0))
                beat(f"encode scan3={v} rep={rep}")
                assert r.status == 0 and r.nblocks == nblk
                same = z.cpu().numpy().tobytes() == want   # (no assertion diff of 11 MB streams)
                assert same, (sw, ntile, v, rep, int(r.out_len), len(want))
    finally:
        e.close()


def test_debug_stop_env_is_ignored(monkeypatch):
    """the phase knockout is a compile-time variant; with DMX_DEBUG_STOP exported
    the product library still writes the oracle's stream."""
    monkeypatch.setenv("DMX_DEBUG_STOP", "1")
    data = _cases()["noise_prefix_then_text"]
    fl = D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK | D.DMX_F_DEEP
    e = D.Encoder(0, len(data))
    try:
        for k in (7, 0):
            z, r = e.compress_bytes(data, max_chain=k, flags=fl)
            assert r.status == 0
            assert z == O.compress(data, max_chain=k, lazy=True, store_check=True, deep=True), k
    finally:
        e.close()
