"""The reference's compress_stats estimate fields (DMX_STATS=ref, the default of the fd_stats
channel), host side only: libdmx's restatement of the reference's adaptive Huffman trees and
code-length pricing (csrc/dmx_refstats.c; src/aht.c:239-277, src/h_tree.c:75-302,
src/deflate_compress.c:290-298) against the records the reference's own encoder wrote for
every golden block (tests/golden/ref_stats.npz, tools/make_golden.py from oracle/_ref).
No GPU: the tokens are the golden ones."""
import hashlib
import json
import os

import numpy as np
import pytest

import deflate_compression_amd as D

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLD, "manifest.json")))["cases"]


@pytest.fixture(scope="module")
def ref_est():
    z = np.load(os.path.join(GOLD, "ref_stats.npz"))
    return {k: np.cumsum(z[k].astype(np.int64), axis=0) for k in z.files}


def test_every_record_equals_reference(golden_tokens, ref_est):
    for name, toks in golden_tokens.items():
        est = D.ref_estimates(toks)
        assert est.shape == (toks.size, 3)
        bad = np.nonzero((est != ref_est[name]).any(axis=1))[0]
        assert bad.size == 0, (name, int(bad[0]), est[bad[0]], ref_est[name][bad[0]])
        assert list(est[-1]) == MAN[name]["ref_last_record"][1:4], name


def test_full_record_stream_digest(golden_tokens):
    """bytes / ll / d from the tokens plus the estimates: the reference's 24-byte record
    stream, byte for byte (manifest records_sha256)."""
    for name, toks in golden_tokens.items():
        t = toks.astype(np.int64)
        lit = (t >> 9) == 0
        ll = np.where(lit, t & 0xFF, t & 0x1FF)
        d = np.where(lit, 0, t >> 9)
        adv = np.where(lit, 1, ll)
        bytes_ = 1 + np.concatenate([[0], np.cumsum(adv)[:-1]])
        rec = np.column_stack([bytes_, D.ref_estimates(toks), ll, d]).astype("<i4")
        assert hashlib.sha256(rec.tobytes()).hexdigest() == MAN[name]["records_sha256"], name


def test_stream_state_continues_across_calls(golden_tokens):
    """One tree state over the stream: feeding in pieces equals feeding at once (how
    write_stats feeds one sw block at a time)."""
    L = D.lib()
    toks = np.concatenate([golden_tokens["bee0"], golden_tokens["rand4k"], golden_tokens["runs32k"]])
    whole = D.ref_estimates(toks)
    e = L.dmx_refest_create()
    try:
        parts = [D.ref_estimates(p, state=e) for p in np.array_split(toks, 7)]
    finally:
        L.dmx_refest_destroy(e)
    assert np.array_equal(np.vstack(parts), whole)


def test_invalid_token_is_range_error():
    with pytest.raises(D.DeflateError) as ei:
        D.ref_estimates(np.array([65, (40000 << 9) | 5], dtype=np.uint32))   # distance > 32768
    assert ei.value.code == -D.E["E_RANGE"]
    with pytest.raises(D.DeflateError):
        D.ref_estimates(np.array([(1 << 9) | 259], dtype=np.uint32))    # length 259
