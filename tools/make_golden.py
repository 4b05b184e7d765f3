#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE encoder (build container only).

1. `make -C oracle -f Makefile.ref` compiles /root/reference's own encoder
   (src/deflate_compress.c + aht.c + h_tree.c) via oracle/ref_driver.c into
   oracle/_ref/ref_tokens (git-ignored).
2. For every case of tests/golden_inputs.cases() the reference's per-token
   compress_stats stream (deflate_ext.h:19-31) is converted to the token encoding
   (t = byte | dist<<9 | len) and stored in ref_tokens.npz; manifest.json keeps
   the token count + SHA-256 and the stats' last-record estimate fields.
   ref_stats.npz keeps every record's estimate fields (tree_bits, ll_bits, d_bits;
   deflate_compress.c:292-298) as int32 first differences, SHA-256 of the whole
   24-byte record stream in the manifest (`records_sha256`).
3. The zlib streams inside the reference's PNG fixtures (png/img/*.png, util/*.png)
   are extracted to idat/*.zlib with the length + SHA-256 of their inflation
   (Python zlib 1.2.11 is the decoder of record; pngtest.png's 52 bytes are also
   the hand-decoded walkthrough png/pngtest.png.txt:20-318).

Re-run after changing golden_inputs.py:  python tools/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import subprocess
import sys
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("DMX_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import oracle as O  # noqa: E402
import golden_inputs  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")


def png_idat(path: str) -> bytes:
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    p, out = 8, b""
    while p < len(b):
        ln = struct.unpack(">I", b[p:p + 4])[0]
        typ = b[p + 4:p + 8]
        if typ == b"IDAT":
            out += b[p + 8:p + 8 + ln]
        p += 12 + ln
    return out


def main() -> None:
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "-f", "Makefile.ref",
                           f"REF={REF}"])
    assert O.ref_available()
    toks, ests, man = {}, {}, {"cases": {}, "idat": {}}
    for name, data in golden_inputs.cases().items():
        st = O.ref_stats(data)
        t = O.ref_tokens(data)
        assert O.replay(t) == data, f"reference replay mismatch on {name}"
        toks[name] = t
        ests[name] = np.diff(st[:, 1:4].astype(np.int64), axis=0, prepend=0).astype(np.int32)
        man["cases"][name] = {
            "n": len(data),
            "ntok": int(t.size),
            "tokens_sha256": hashlib.sha256(t.astype("<u4").tobytes()).hexdigest(),
            "input_sha256": hashlib.sha256(data).hexdigest(),
            "ref_last_record": [int(x) for x in st[-1]],
            "records_sha256": hashlib.sha256(st.astype("<i4").tobytes()).hexdigest(),
        }
        print(f"{name:14s} n={len(data):6d} ntok={t.size}")
    np.savez_compressed(os.path.join(GOLD, "ref_tokens.npz"), **toks)
    np.savez_compressed(os.path.join(GOLD, "ref_stats.npz"), **ests)
    for rel in ["png/img/pngtest.png", "png/img/pngtest2.png", "png/img/pngtest3.png",
                "util/image.png", "util/image1.png", "util/sunset.png"]:
        z = png_idat(os.path.join(REF, rel))
        raw = zlib.decompress(z)
        nm = os.path.basename(rel).replace(".png", "")
        with open(os.path.join(GOLD, "idat", nm + ".zlib"), "wb") as f:
            f.write(z)
        man["idat"][nm] = {"source": rel, "zlib_len": len(z), "raw_len": len(raw),
                           "raw_sha256": hashlib.sha256(raw).hexdigest()}
        if nm == "pngtest":
            man["idat"][nm]["raw_hex"] = raw.hex()
        print(f"idat {nm}: {len(z)} -> {len(raw)}")
    with open(os.path.join(GOLD, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
