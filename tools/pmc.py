"""HBM traffic per launch from rocprofv3 counter CSVs (bench.py roofline.traffic).

Counters are collected in their own passes, one per counter (FETCH_SIZE and WRITE_SIZE
do not fit one pass of the 4 TCC slots on gfx950):

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- python3 bench.py ...

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled.
WRITE_SIZE is taken as is.  Returns bytes per launch of the named kernel, averaged
over its dispatches, or None when the kernel is not in the files.
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

FETCH_SCALE = 2.0 * 1024.0
WRITE_SCALE = 1024.0


def _files(spec: str):
    out = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if os.path.isdir(part):
            out += glob.glob(os.path.join(part, "**", "*counter_collection.csv"), recursive=True)
        else:
            out.append(part)
    return out


def per_kernel(spec: str):
    """{kernel_name: {counter: mean value per dispatch}} over all CSVs in spec."""
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in _files(spec):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                c = row.get("Counter_Name", "")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(disp[k][c]))
                acc[k][c] += v
                disp[k][c].add((f, did))
    return {k: {c: acc[k][c] / max(1, len(disp[k][c])) for c in acc[k]} for k in acc}


def traffic_per_launch(spec: str, kernel: str):
    """HBM bytes per launch (corrected FETCH + WRITE) for the kernel whose name contains `kernel`."""
    tab = per_kernel(spec)
    hit = [v for k, v in tab.items() if kernel in k]
    if not hit:
        return None
    m = hit[0]
    fetch = m.get("FETCH_SIZE")
    write = m.get("WRITE_SIZE")
    if fetch is None and write is None:
        return None
    return {
        "bytes": round((fetch or 0.0) * FETCH_SCALE + (write or 0.0) * WRITE_SCALE),
        "fetch_bytes": None if fetch is None else round(fetch * FETCH_SCALE),
        "write_bytes": None if write is None else round(write * WRITE_SCALE),
        "correction": "FETCH_SIZE KiB x2 (gfx950 half-count), WRITE_SIZE KiB x1",
    }


def counters_json(pmc_spec: str, sq_spec: str, nblk: int, parsed: int, source: str, parse: str, workload: str,
                  kernel: str = "dmx_match_kernel") -> dict:
    """tools/roofline_counters.json for bench.py: per-block FETCH / WRITE bytes (corrected)
    and SQ instruction counts of `kernel`, from a profile of the bench configuration itself
    (nblk blocks per launch, `parsed` of them through the kernel)."""
    out = {"source": source, "parse": parse, "workload": workload, "blocks_per_launch": nblk, "kernels": {}}
    t = traffic_per_launch(pmc_spec, kernel) if pmc_spec else None
    sq = {k: v for k, v in per_kernel(sq_spec).items() if kernel in k} if sq_spec else {}
    k = {}
    if t:
        k["fetch_bytes_per_block"] = t["fetch_bytes"] / nblk
        k["write_bytes_per_block"] = t["write_bytes"] / nblk
    if sq:
        m = next(iter(sq.values()))
        for c, name in (("SQ_INSTS_VALU", "valu_per_block"), ("SQ_INSTS_SALU", "salu_per_block"),
                        ("SQ_INSTS_LDS", "lds_per_block"), ("SQ_LDS_BANK_CONFLICT", "lds_conflict_cycles_per_block"),
                        ("SQ_LDS_IDX_ACTIVE", "lds_active_cycles_per_block")):
            if c in m:
                k[name] = m[c] / parsed
    out["kernels"][kernel] = k
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--counters-json":
        # --counters-json PMC_DIRS SQ_DIRS NBLK PARSED SOURCE PARSE WORKLOAD > tools/roofline_counters.json
        import json
        a = sys.argv[2:]
        print(json.dumps(counters_json(a[0], a[1], int(a[2]), int(a[3]), a[4], a[5], a[6]), indent=1))
        sys.exit(0)
    spec = sys.argv[1]
    for k, v in sorted(per_kernel(spec).items()):
        short = k.split("(")[0]
        print(f"{short:40s} " + " ".join(f"{c}={x:.1f}" for c, x in sorted(v.items())))
