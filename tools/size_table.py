"""Size of the bounded lazy parses (K = 6, 7, 8) against S_ref, the reference-semantics
stream (exhaustive greedy, deflate_compress.c:243-288), on real text held by the reference
tree -- read as input bytes only, nothing of it is written under tests/ -- plus the two
inputs the bench line quotes (the seeded C3 generator and the bee corpus tiled).

Build container only (it reads /root/reference); CPU oracle (test infrastructure).
    python tools/size_table.py [--out profiles/r04_size/size_table.md]
"""
from __future__ import annotations

import argparse
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
KS = (6, 7, 8)
COLS = [(k, False) for k in KS] + [(k, True) for k in KS]   # (K, DMX_F_DEEP)


def inputs():
    import deflate_compression_amd as D
    bee = open(os.path.join(REPO, "tests", "golden", "bee_movie_script.txt"), "rb").read()
    yield "C3 generator (seed 0xE5818), 8 MB", D.gen_text(8 << 20, 0xE5818).tobytes()
    yield "bee corpus tiled to 8 MB (`real_text`)", (bee * ((8 << 20) // len(bee) + 1))[:8 << 20]
    pats = ["test_files/original/*.txt", "docs/*.txt", "README.md", "png/*.txt", "results/*.txt",
            "src/*.c", "src/include/*.h", "src/png/*.c", "src/png/include/*.h", "tests/*.c", "util/src/*.c",
            "util/README.md"]
    for p in pats:
        for f in sorted(glob.glob(os.path.join(REF, p))):
            b = open(f, "rb").read()
            if len(b) >= 64:
                yield os.path.relpath(f, REF), b


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r04_size", "size_table.md"))
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--deep-chain", type=int, default=0, help="DMX_F_DEEP depth (dmx_opts.deep_chain; 0 = 64)")
    a = ap.parse_args()
    O.set_deep_chain(a.deep_chain)
    rows = []
    tot = {c: 0 for c in ["ref"] + COLS}
    for name, b in inputs():
        ref = len(O.compress_par(b, max_chain=0, lazy=False, threads=a.threads))
        s = {c: len(O.compress_par(b, max_chain=c[0], lazy=True, store_check=True, deep=c[1], threads=a.threads))
             for c in COLS}
        if not name.startswith(("C3", "bee")):
            tot["ref"] += ref
            for c in COLS:
                tot[c] += s[c]
        rows.append((name, len(b), ref, s))
        print(name, len(b), ref, {c: f"{100.0 * (s[c] - ref) / ref:+.2f}" for c in COLS}, flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write("# Bounded lazy parse vs S_ref on reference-held text (oracle, `tools/size_table.py`)\n\n")
        f.write("S_ref = the reference-semantics stream (exhaustive greedy, 32 KiB blocks). Columns: "
                "stream size of the K-candidate lazy parse (store check on) relative to S_ref; \"deep\" = "
                "with DMX_F_DEEP (small-alphabet blocks search DMX_DEEP_CHAIN deep, 32 since round 5; the bench default is K=7 lazy deep). "
                "The reference's files are read as input bytes only.\n\n")
        hd = [f"K={k} lazy" + (" deep" if d else "") for k, d in COLS]
        f.write("| Input | Bytes | S_ref bytes | " + " | ".join(hd) + " |\n")
        f.write("|---|---|---|" + "---|" * len(COLS) + "\n")
        for name, n, ref, s in rows:
            f.write(f"| {name} | {n} | {ref} | " + " | ".join(f"{100.0 * (s[c] - ref) / ref:+.2f} %" for c in COLS)
                    + " |\n")
        f.write(f"| all reference files together | | {tot['ref']} | "
                + " | ".join(f"{100.0 * (tot[c] - tot['ref']) / tot['ref']:+.2f} %" for c in COLS) + " |\n")
        worst = {c: max(100.0 * (s[c] - ref) / ref for _, _, ref, s in rows) for c in COLS}
        f.write("| worst row | | | " + " | ".join(f"{worst[c]:+.2f} %" for c in COLS) + " |\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
