"""Deterministic inputs for the golden token fixtures (shared by tools/make_golden.py
and the tests).  Pure data generation: no reference code, no oracle."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bee() -> bytes:
    """test_files/original/bee_movie_script.txt of the reference (57 641 B), kept as a fixture."""
    with open(os.path.join(GOLDEN, "bee_movie_script.txt"), "rb") as f:
        return f.read()


def px_slices() -> dict:
    """32 KiB slices of the reference's raw RGB logs results/sunrise*.px (fixture copy)."""
    z = np.load(os.path.join(GOLDEN, "px_slices.npz"), allow_pickle=False)
    return {k: z[k].tobytes() for k in z.files}


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def _alpha(seed: int, letters: bytes, n: int) -> bytes:
    return _rng(seed).choice(np.frombuffer(letters, np.uint8), n).astype(np.uint8).tobytes()


def _runs(seed: int, n: int) -> bytes:
    r = _rng(seed)
    out = bytearray()
    while len(out) < n:
        out += bytes([int(r.integers(0, 256))]) * int(r.integers(1, 400))
    return bytes(out[:n])


def _all_dists(n: int) -> bytes:
    """Matches at every distance class: a random 32K-ish buffer whose tail repeats
    pieces from geometrically spread distances (exercises all 30 distance codes)."""
    r = _rng(77)
    base = bytearray(r.integers(0, 256, n, dtype=np.uint8).tobytes())
    pos = 20000
    for d in [1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768,
              1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 20000]:
        if pos + 40 > n:
            break
        for k in range(12):
            base[pos + k] = base[pos + k - d]
        pos += 12 + 5
    return bytes(base)


def cases() -> dict:
    b = bee()
    c = {
        "bee0": b[:32768],
        "bee1": b[32768:],
        "zeros32k": bytes(32768),
        "zeros1000": bytes(1000),
        "rand32k": _rng(0x5EED).integers(0, 256, 32768, dtype=np.uint8).tobytes(),
        "rand4k": _rng(5).integers(0, 256, 4096, dtype=np.uint8).tobytes(),
        "ab20000": _alpha(1, b"ab", 20000),
        "abcd32k": _alpha(2, b"abcd", 32768),
        "alpha16_32k": _alpha(3, b"abcdefghijklmnop", 32768),
        "runs32k": _runs(4, 32768),
        "period7": (b"abcdefg" * 5000)[:32768],
        "alldist": _all_dists(32768),
        "bytes256": (bytes(range(256)) * 128),
    }
    for n in (3, 4, 5, 10, 100, 1000, 4095, 4096, 8191, 8192, 16385, 32767):
        c[f"bee_n{n}"] = b[1000:1000 + n]
    c.update(px_slices())
    return c
