"""Seeded small-alphabet inputs for the adaptive chain depth (DMX_F_DEEP),
shared by tests/test_deep.py (CPU) and tests/test_gpu_deep.py (GPU)."""
import binascii

import numpy as np

import deflate_compression_amd as D


def bitdump(n: int, seed: int) -> bytes:
    """Text shaped like a bit-level walkthrough of a stream (the reference's
    png/pngtest.png.txt style): groups of 8 binary digits, tabs, labels, newlines."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < n:
        out += b"\t\t\t\tProgress: \n\t\t\t\t"
        for _ in range(int(rng.integers(6, 40))):
            v = int(rng.integers(0, 256)) if rng.random() < 0.7 else 0xFF
            out += format(v, "08b").encode() + (b"\n\t\t\t\t" if rng.random() < 0.15 else b" ")
        out += b"\n\t\t\t\tCode: " + format(int(rng.integers(0, 512)), "09b").encode() + b"\n"
        out += b"\t\t\t\t\tVal: " + str(int(rng.integers(0, 300))).encode() + b"\n\n"
    return bytes(out[:n])


def inputs() -> dict:
    rng = np.random.default_rng(5)
    text = D.gen_text(200000, 31).tobytes()
    return {
        "bitdump": bitdump(150000, 1),
        "bin01": rng.choice(np.frombuffer(b"01", dtype=np.uint8), 70000).tobytes(),
        "dna": rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 70000).tobytes(),
        "hex": binascii.hexlify(text[:40000]),
        # deep and text blocks side by side, a short deep tail
        "mixed": text[:40000] + bitdump(50000, 2) + text[40000:80000] + bitdump(9000, 3),
        "text": text,
    }
