"""CPU-side tests: libdmx.so loads and exports every symbol include/dmx.h declares,
the host inflate (deflate_decompress) against zlib and the reference's PNG KATs,
Adler-32 combine, generators, and the fail-loudly contract without a GPU."""
import hashlib
import json
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

import deflate_compression_amd as D
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
MAN = json.load(open(os.path.join(GOLD, "manifest.json")))


def declared_functions():
    src = open(os.path.join(REPO, "include", "dmx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;{]*\)\s*;", src, flags=re.M)
    return sorted(set(names))


def test_all_declared_symbols_exported():
    names = declared_functions()
    assert "deflate_compress" in names and "deflate_decompress" in names and "dmx_encode_async" in names
    out = subprocess.check_output(["nm", "-D", "--defined-only", D.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    L = D.lib()
    for n in names:
        assert getattr(L, n) is not None


def test_library_is_gfx950_code_object():
    blob = open(D.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for k in (b"dmx_match_kernel", b"dmx_huff_kernel", b"dmx_scan_kernel",
              b"dmx_pack_kernel"):
        assert k in blob


@pytest.mark.parametrize("name", ["bee0", "rand32k", "zeros32k", "alldist", "px_sunrise_b", "bee_n3"])
def test_inflate_oracle_streams(golden_cases, name):
    d = golden_cases[name]
    z = O.compress(d)
    assert D.deflate_decompress(z) == d


def test_inflate_zlib_streams():
    rng = np.random.default_rng(0)
    for lvl in (0, 1, 6, 9):
        for n in (0, 1, 100, 70000):
            d = D.gen_text(n, 3).tobytes() if n else b""
            assert D.deflate_decompress(zlib.compress(d, lvl)) == d
    d = rng.integers(0, 4, 200000, dtype=np.uint8).tobytes()
    assert D.deflate_decompress(zlib.compress(d, 9)) == d


def test_inflate_png_kats():
    """Reference fixtures: png/img/*.png (fixed Huffman), util/*.png (dynamic,
    multi-block); pngtest.png decodes to the 52 bytes walked through in
    png/pngtest.png.txt:20-318."""
    for nm, m in MAN["idat"].items():
        z = open(os.path.join(GOLD, "idat", nm + ".zlib"), "rb").read()
        raw = D.deflate_decompress(z)
        assert len(raw) == m["raw_len"]
        assert hashlib.sha256(raw).hexdigest() == m["raw_sha256"]
        if "raw_hex" in m:
            assert raw.hex() == m["raw_hex"]


def test_inflate_nullterm():
    assert D.deflate_decompress(zlib.compress(b"abc"), 1) == b"abc\0"


@pytest.mark.parametrize("bad,code", [
    (b"\x78", "E_ZHEAD"),
    (b"\x79\x9c\x03\x00\x00\x00\x00\x01", "E_ZCMPMT"),
    (b"\x88\x9c\x03\x00\x00\x00\x00\x01", "E_ZSLWIN"),
    (b"\x78\x9d\x03\x00\x00\x00\x00\x01", "E_ZFCHCK"),
    (b"\x78\xbb" + b"\x00" * 8, "E_ZPDICT"),
    (b"\x78\x9c\x03\x00\x00\x00\x00\x02", "E_ZADL32"),
    (b"\x78\x9c\x07\x00", "E_ZBTYPE"),
    (b"\x78\x9c\x01\x05\x00\x00\x00abcde", "E_ZNLEN"),
])
def test_inflate_errors(bad, code):
    with pytest.raises(D.DeflateError) as ei:
        D.deflate_decompress(bad)
    assert ei.value.code == -D.E[code]


def test_inflate_truncated():
    z = zlib.compress(D.gen_text(5000, 1).tobytes())
    with pytest.raises(D.DeflateError):
        D.deflate_decompress(z[:-7])


def test_adler_combine():
    rng = np.random.default_rng(1)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        assert D.adler32_combine(zlib.adler32(a), zlib.adler32(b), len(b)) == zlib.adler32(a + b)


def test_generators_deterministic():
    a, b = D.gen_text(200000, 5), D.gen_text(200000, 5)
    assert np.array_equal(a, b) and not np.array_equal(a, D.gen_text(200000, 6))
    r = zlib.compress(a.tobytes(), 6)
    assert 0.3 < len(r) / a.size < 0.5         # enwik-like compressibility
    x = D.gen_random(1 << 16, 0x5EED)
    assert np.array_equal(x, D.gen_random(1 << 16, 0x5EED))
    assert len(zlib.compress(x.tobytes())) > x.size


def test_max_compressed_bound():
    for n in (0, 1, 32768, 32769, 10 ** 6):
        assert D.max_compressed(n) >= len(O.compress(D.gen_random(n, 1).tobytes())) if n <= 10 ** 6 else True


def test_no_cpu_fallback_without_gpu():
    """On a host without a GPU every encode fails loudly (no silent CPU path)."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(D.DeflateError) as ei:
        D.compress(b"hello world")
    assert ei.value.code == -D.E["E_NEXIST"]
    r, w = os.pipe()
    os.write(w, b"abc")
    os.close(w)
    assert D.deflate_compress(r, -1, -1, 32768, 0) == -D.E["E_NEXIST"]
    os.close(r)


def test_bad_stats_mode_fails_before_encoding(tmp_path, monkeypatch):
    """An unknown DMX_STATS value is rejected with -E_INVAL before anything is read, encoded
    or written (no GPU needed: the check comes first)."""
    monkeypatch.setenv("DMX_STATS", "bogus")
    fi, fo, fs = tmp_path / "in", tmp_path / "out", tmp_path / "st"
    fi.write_bytes(b"hello hello hello")
    a = os.open(fi, os.O_RDONLY)
    b = os.open(fo, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    c = os.open(fs, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        assert D.deflate_compress(a, b, c, 32768, 0) == -D.E["E_INVAL"]
        assert os.lseek(a, 0, os.SEEK_CUR) == 0
    finally:
        for x in (a, b, c):
            os.close(x)
    assert fo.read_bytes() == b"" and fs.read_bytes() == b""


def test_product_does_not_reference_oracle():
    """The shipped package never imports or links the oracle."""
    pkg = os.path.join(REPO, "deflate_compression_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".c", ".h", ".hip", "Makefile")):
                txt = open(os.path.join(root, f)).read()
                assert "oracle" not in txt.lower().replace("oracle_", ""), f
    out = subprocess.check_output(["nm", "-D", D.LIB_PATH], text=True)
    assert "dmx_oracle" not in out


def test_product_library_has_no_debug_knockout():
    """the phase knockout that ends every block after P0 / P1 / P2 (wrong streams)
    exists only in diagnostic variants built with -DDMX_DEBUG_STOP (tools/build_var.sh): the
    product library never reads such a switch from the environment, and an encode reads no
    environment variable at all (test hooks are per-context, dmx_ctx_set_hook)."""
    blob = open(D.LIB_PATH, "rb").read()
    assert b"DMX_DEBUG_STOP" not in blob
    src = open(os.path.join(REPO, "deflate_compression_amd", "csrc", "dmx_kernels.hip")).read()
    body = src[src.index('extern "C" int dmx_encode_async('):]
    body = body[:body.index("\n}\n")]
    assert "getenv" not in body
