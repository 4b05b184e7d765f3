#!/usr/bin/env python3
"""bench.py -- DEFLATE encode throughput on MI355X (BASELINE.json metric).

One "step" = one full encode of the rank's resident input (HBM -> HBM zlib stream),
i.e. every kernel of the hot path.  N = 1 workload: config C3 (enwik8-sized enwik-style
text, 100 000 000 B, 3 052 blocks of 32 KiB).  N > 1 (one process per GPU): weak
scaling, every rank encodes its own 100 MB shard (per-rank seed) framed as a shard of one
stream, and the compressed chunks are gathered to rank 0 over RCCL (point-to-point over
xGMI) inside the timed region.

`python bench.py --gpus N` with WORLD_SIZE unset starts the N rank processes itself
(torch.distributed.run, before anything touches the GPU) and exits with their status;
a rank whose world differs from --gpus exits non-zero.  Before timing, rank 0 inflates the
stitched N-rank stream (header + chunks + combined Adler-32) and compares it with every
rank's input: a wrong stream makes the run fail.

Prints ONE JSON line on rank 0 (see DESIGN.md §5 for the roofline accounting).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time
import zlib

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
TIMING_EVERY = 4  # the timed region events the dominant stage on every 4th step (from its first)
# VALU issue ceiling: 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 32-bit integer
# instruction (tools/valu_peak.hip measured 3.7-4.2 cycles, 526-630 G/s; profiles/r02_a)
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 4.0
COUNTERS = os.path.join(REPO, "tools", "roofline_counters.json")

WORKLOADS = {
    # name: (bytes per rank, generator, seed, description)
    "text": (100_000_000, "text", 0xE5818, "C3: enwik8-sized enwik-style wiki text (seeded generator)"),
    "zeros": (1 << 30, "zeros", 0, "1 GiB of 0x00 (zero-entropy run, C2 scaled up)"),
    "random": (1 << 30, "random", 0x5EED, "C4: 1 GiB splitmix64 bytes (stored-block path)"),
    "enwik9": (1_000_000_000, "text", 0xE5819, "C5: 1 GB enwik9-style text split across the ranks (strong)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="text", choices=sorted(WORKLOADS))
    ap.add_argument("--bytes", type=int, default=0, help="override bytes per rank")
    ap.add_argument("--max-chain", type=int, default=int(os.environ.get("DMX_MAX_CHAIN", "7")),
                    help="0 = exhaustive (reference parse); K = K newest chain entries (default 7: the "
                         "fastest K inside the <= 2 %% size budget vs S_ref on every reference-held text "
                         "with --deep, profiles/r04_size/size_table.md)")
    ap.add_argument("--deep", type=int, default=int(os.environ.get("DMX_DEEP", "1")),
                    help="1 = adaptive chain depth: small-alphabet blocks search 32 deep (DMX_F_DEEP, DMX_DEEP_CHAIN)")
    ap.add_argument("--lazy", type=int, default=int(os.environ.get("DMX_LAZY", "1")),
                    help="1 = lazy evaluation parse (DMX_F_LAZY, SURVEY §8 f2)")
    ap.add_argument("--split", type=int, default=int(os.environ.get("DMX_SPLIT", "0")),
                    help="1 = adaptive block splitting (DMX_F_SPLIT, SURVEY §8 f3)")
    ap.add_argument("--store-check", type=int, default=int(os.environ.get("DMX_STORE_CHECK", "1")),
                    help="1 = noise blocks stored without a parse (DMX_F_STORE_CHECK, DESIGN.md §4.7)")
    ap.add_argument("--dict", type=int, default=int(os.environ.get("DMX_DICT", "0")),
                    help="1 = cross-block dictionary (DMX_F_DICT, SURVEY §8 f1); N > 1: halo exchange of "
                         "the block before each shard inside the step")
    ap.add_argument("--tradeoff", default="4,6,8,16",
                    help="N = 1: also time these max_chain values (same flags) for the speed/size curve "
                         "(reported under 'tradeoff'; '' = skip)")
    ap.add_argument("--exhaustive-steps", type=int, default=3,
                    help="also time this many exhaustive-parse steps (reported under 'exhaustive')")
    ap.add_argument("--gather", default="root", choices=["root", "root-sync", "all", "none"],
                    help="N > 1: root = chunks to rank 0 point-to-point, pipelined (the gather of step i-1 "
                         "overlaps the encode of step i, double-buffered); root-sync = the same, step by step; "
                         "all = max-padded all_gather; none = encode only")
    ap.add_argument("--pipeline-test", type=int, default=0,
                    help="run the pipelined gather loop at N = 1 too (single-rank process group; tests the path)")
    ap.add_argument("--cpu-budget", type=float, default=8.0,
                    help="seconds per CPU baseline leg (0 = skip the CPU legs)")
    ap.add_argument("--real-text", type=int, default=1,
                    help="N = 1, text workload: also encode the reference's corpus tiled to 100 MB "
                         "(reported under 'real_text'; 0 = skip)")
    ap.add_argument("--long-run", type=float, default=1.0,
                    help="N = 1: after the timed steps, time further steps for about this many seconds "
                         "(reported under 'long_run'; 0 = skip)")
    ap.add_argument("--traffic-csv", default="",
                    help="comma-separated rocprofv3 counter CSVs / dirs (FETCH_SIZE and WRITE_SIZE passes); "
                         "default: the committed tools/roofline_counters.json")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: start the ranks and check the world over gloo, no GPU work")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv) -> int:
    """--gpus N > 1 without a launcher: start N ranks with torch.distributed.run (nothing in
    this process has touched a GPU) and return their exit status.  Rank 0 prints the line."""
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    log("bench: starting", args.gpus, "ranks:", " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launch_check(args, json_fd: int) -> int:
    """--launch-check: the launcher and the world size, over gloo, without a GPU."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    ok = int(t.item()) == world * (world + 1) // 2
    dist.barrier()
    if rank == 0:
        os.write(json_fd, (json.dumps({"launch_check": True, "n_gpus": world, "ranks_ok": ok}) + "\n").encode())
    dist.destroy_process_group()
    return 0 if ok else 1


def make_input(kind: str, n: int, seed: int):
    import numpy as np
    import deflate_compression_amd as D
    if kind == "text":
        return D.gen_text(n, seed)
    if kind == "random":
        return D.gen_random(n, seed)
    return np.zeros(n, dtype=np.uint8)


def parse_str(args) -> str:
    return (("exhaustive" if args.max_chain == 0 else f"max_chain={args.max_chain}")
            + (", lazy" if args.lazy else ", greedy") + (", split" if args.split else "")
            + (", dict" if args.dict else "") + (", store-check" if args.store_check else "")
            + (", deep" if args.deep and 0 < args.max_chain < 64 else ""))


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
    quota = None   # the cgroup's CPU quota in cores (cgroup v2 cpu.max), when one is set
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    # the CPU legs run on every core of the process's affinity (SURVEY §8d ii: all cores) and
    # on the box's nominal share (OMP_NUM_THREADS); the line reports the faster as the baseline
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": aff, "threads": aff, "share_threads": share,
            "cgroup_cpu_quota": quota}


def cpu_baselines(data, args, budget_s: float):
    """CPU legs on rank 0 (SURVEY §8d ii), on the GPU box's host cores, in the same run:
      same_parse  -- oracle/dmx_oracle.c (C port of the reference parse + our Huffman/emitter)
                     with the GPU line's parse flags, blocks in parallel on every core of the
                     process's affinity (OpenMP), over the whole workload when the budget allows
                     (else a bounded sample); its stream over the whole input is kept as the
                     full-size parity witness of the GPU stream;
      share       -- the same leg on the box's nominal CPU share (OMP_NUM_THREADS), a sample;
      exhaustive  -- the same port with the reference's own exhaustive parse, all cores: its
                     stream over the whole input is S_ref, the size the GPU stream is compared
                     with, and the parity witness of the GPU's exhaustive stream;
      reference   -- the reference encoder itself (oracle/_ref, built from /root/reference's own
                     sources), one process per 32 KiB block, 1 core, with its per-token estimator
                     (only where it was built).
    """
    from oracle import oracle as O
    info = cpu_info()
    out = {}
    n = int(data.size)
    sw = 32768

    def leg(max_chain, lazy, split, dct, store, deep, budget, name, thr, want_full):
        kw = dict(lazy=lazy, split=split, dict=dct, store_check=store, threads=thr, deep=deep)
        piece = min(n, sw * max(4 * thr, 32))
        t0 = time.perf_counter()
        O.compress_par(data[:piece], sw, max_chain, flags=5, **kw)   # probe: the first piece
        tp = time.perf_counter() - t0
        z = None
        if piece and tp / piece * n <= 2 * budget:
            # the whole workload in one call: one stream, its exact size
            t0 = time.perf_counter()
            z = O.compress_par(data, sw, max_chain, flags=7, **kw)
            dt = time.perf_counter() - t0
            done, how = n, "all"
        else:   # a bounded sample: pieces until the budget is spent (first piece included)
            done, dt = piece, tp
            while done < n and dt < budget:
                hi = min(n, done + piece)
                q0 = time.perf_counter()
                O.compress_par(data[done:hi], sw, max_chain, flags=4, **kw)
                dt += time.perf_counter() - q0
                done = hi
            how = "first"
            if want_full and tp / piece * n <= 8 * budget:   # the parity witness, untimed
                z = O.compress_par(data, sw, max_chain, flags=7, **kw)
        return {"value": round(done / dt / 1e9, 6), "unit": "GB/s", "cores": thr, "kind": "port",
                "sample": f"{how} {done} B of the workload, oracle/dmx_oracle.c {name}, blocks in parallel on "
                          f"{thr} OpenMP threads (dmx_oracle_compress_par)",
                "cpu_model": info["cpu_model"], "nproc": info["nproc"]}, done, z

    parse = parse_str(args)
    same = (args.max_chain, bool(args.lazy), bool(args.split), bool(args.dict), bool(args.store_check),
            bool(args.deep))
    # the box's CPU share (OMP_NUM_THREADS = the cgroup quota): more threads than that only
    # oversubscribe the quota
    best_thr = info["share_threads"]
    r, _, z = leg(*same, budget_s, f"compress ({parse}: the GPU line's parse)", best_thr, True)
    r["parse"] = parse
    out["same_parse_stream"] = z
    out["same_parse"] = r
    # the port at the GPU line's parse on ONE core, a bounded sample
    r1, _, _ = leg(*same, min(budget_s, 10.0), f"compress ({parse}: the GPU line's parse), one core", 1, False)
    r1["parse"] = parse
    out["same_parse_1core"] = r1
    r, done, z = leg(0, False, False, False, False, False, budget_s,
                     "compress (the reference's exhaustive greedy parse + Huffman/emitter)", best_thr, True)
    r["parse"] = "exhaustive, greedy (reference semantics)"
    out["exhaustive"] = r
    out["s_ref_stream"] = z   # the reference parse's stream over the whole input (None: too slow here)
    if O.ref_available():
        t0 = time.perf_counter()
        done = 0
        while done < n and time.perf_counter() - t0 < budget_s:
            O.ref_stats(data[done:done + sw].tobytes())
            done += min(sw, n - done)
        dt = time.perf_counter() - t0
        out["reference"] = {"value": round(done / dt / 1e9, 9), "unit": "GB/s", "cores": 1, "kind": "reference",
                            "sample": f"first {done} B of the workload in 32 KiB blocks through the reference "
                                      "encoder (src/deflate_compress.c + aht.c + h_tree.c, oracle/_ref), "
                                      "1 process at a time, incl. its per-token estimator",
                            "cpu_model": info["cpu_model"]}
    return out, info


def real_text_leg(enc_flags, args, dev, local, stream):
    """Representativeness check: real text instead of the seeded generator -- the
    reference's own corpus (tests/golden/bee_movie_script.txt, 57 641 B of CRLF text) tiled to
    100 MB and cut into independent 32 KiB blocks (every block starts at a different offset of
    the corpus), encoded with the bench's parse; GB/s over 5 steps, size vs its own S_ref (the
    port's exhaustive stream, all cores) and byte parity with the port at the same parse."""
    import numpy as np
    import torch
    import deflate_compression_amd as D
    from oracle import oracle as O
    bee = np.frombuffer(open(os.path.join(REPO, "tests", "golden", "bee_movie_script.txt"), "rb").read(),
                        dtype=np.uint8)
    n = 100_000_000
    host = np.resize(bee, n)
    thr = cpu_info()["share_threads"]
    e = D.Encoder(local, n, 32768, args.max_chain, enc_flags)
    try:
        d_in = torch.from_numpy(host).to(dev)
        cap = D.max_compressed(n)
        d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
        e.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
        r = e.result(stream)
        z = d_out[:int(r.out_len)].cpu().numpy().tobytes()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            e.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / 5
    finally:
        e.close()
    port = O.compress_par(host, 32768, args.max_chain, lazy=bool(args.lazy), split=bool(args.split),
                          dict=bool(args.dict), store_check=bool(args.store_check), threads=thr,
                          deep=bool(args.deep))
    sref = O.compress_par(host, 32768, 0, threads=thr)
    return {"value": round(n / dt / 1e9, 3), "unit": "GB/s", "ms_per_step": round(dt * 1e3, 4), "steps": 5,
            "input": "tests/golden/bee_movie_script.txt (the reference's corpus) tiled to 100 000 000 B, "
                     "independent 32 KiB blocks", "parse": parse_str(args),
            "ratio": round(len(z) / n, 5), "s_ref_bytes": len(sref),
            "size_vs_ref_pct": round((len(z) / len(sref) - 1) * 100, 3),
            "parity_vs_port": z == port, "inflates": zlib.decompress(z) == host.tobytes(),
            "nsortfallback_total": int(r.nsortfallback_total)}


def end_to_end(host, args):
    """The drop-in fd API end to end (file-in/file-out): read(fd_in), H2D, encode,
    D2H, write(fd_out), with the bench's parse settings; best of 3 (the first call also
    creates the cached device context).  PCIe-inclusive, so never the headline value."""
    import tempfile
    import deflate_compression_amd as D
    env = {"DMX_MAX_CHAIN": str(args.max_chain), "DMX_LAZY": str(args.lazy), "DMX_SPLIT": str(args.split),
           "DMX_DICT": str(args.dict), "DMX_STORE_CHECK": str(args.store_check), "DMX_DEEP": str(args.deep)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    td = tempfile.mkdtemp(dir="/tmp")
    fi, fo = os.path.join(td, "in"), os.path.join(td, "out")
    try:
        host.tofile(fi)
        best, rc, st_best = None, 0, None
        for _ in range(3):
            a = os.open(fi, os.O_RDONLY)
            b = os.open(fo, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            t0 = time.perf_counter()
            rc = D.deflate_compress(a, b, -1, 32768, 0)
            t1 = time.perf_counter()
            os.close(a)
            os.close(b)
            if best is None or t1 - t0 < best:
                best, st_best = t1 - t0, D.fd_last_stats()
        with open(fo, "rb") as f:
            z = f.read()
        ok = rc == 0 and zlib.decompress(z) == host.tobytes()
        # the same call with fd_out = /dev/null: the path without the box's file-write ceiling
        # (DESIGN.md §6b), i.e. read + H2D + encode + D2H + the writer thread's write calls
        bn, rcn, stn = None, 0, None
        for _ in range(3):
            a = os.open(fi, os.O_RDONLY)
            b = os.open(os.devnull, os.O_WRONLY)
            t0 = time.perf_counter()
            rcn = D.deflate_compress(a, b, -1, 32768, 0)
            t1 = time.perf_counter()
            os.close(a)
            os.close(b)
            if bn is None or t1 - t0 < bn:
                bn, stn = t1 - t0, D.fd_last_stats()
        return {"value": round(host.size / best / 1e9, 3), "unit": "GB/s", "ms": round(best * 1e3, 2), "rc": rc,
                "compressed_bytes": len(z), "inflates": ok,
                "path": "deflate_compress(fd_in, fd_out): read + H2D + encode + D2H + write, best of 3",
                "stage_busy_ms": st_best,
                "sink_devnull": {"value": round(host.size / bn / 1e9, 3), "unit": "GB/s", "ms": round(bn * 1e3, 2),
                                 "rc": rcn, "path": "the same with fd_out = /dev/null (no file-write ceiling)",
                                 "stage_busy_ms": stn},
                "stage_note": "stage_busy_ms (dmx_fd_last_stats): reader/writer thread time in read/write, "
                              "H2D/encode/D2H device time summed over chunks; the stages overlap, so the "
                              "largest bounds the call"}
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for x in (fi, fo):
            if os.path.exists(x):
                os.remove(x)
        os.rmdir(td)


def verify_stitched(chunks, adlers, lens, expected_pieces) -> bool:
    """Rank 0: the N shard chunks + the combined Adler-32 trailer must inflate (zlib) to the
    concatenation of every rank's input (expected_pieces: callables returning rank r's bytes)."""
    from deflate_compression_amd import shard as S
    adler = S.combine_adler(adlers, lens)
    d = zlib.decompressobj()
    pend = b""
    r = 0
    want = expected_pieces[0]() if expected_pieces else b""
    try:
        for part in list(chunks) + [S.trailer(adler)]:
            pend += d.decompress(part)
            while r < len(expected_pieces) and len(pend) >= len(want):
                if pend[:len(want)] != want:
                    return False
                pend = pend[len(want):]
                r += 1
                want = expected_pieces[r]() if r < len(expected_pieces) else b""
        pend += d.flush()
    except zlib.error:   # corrupt stream or Adler-32 mismatch
        return False
    return d.eof and r == len(expected_pieces) and pend == b"" and not d.unused_data


def roofline_counters(kname: str, parse: str, workload: str):
    """Per-block SQ / PMC figures of `kname` from the committed profile (tools/roofline_counters.json,
    written by tools/pmc.py from profiles/<tag>), if it was taken on this configuration."""
    try:
        with open(COUNTERS) as f:
            c = json.load(f)
    except (OSError, ValueError):
        return None, "tools/roofline_counters.json missing"
    if c.get("parse") != parse or c.get("workload") != workload:
        return None, f"counters were taken on {c.get('workload')!r} / {c.get('parse')!r}"
    k = c.get("kernels", {}).get(kname)
    if not k:
        return None, f"no counters for {kname}"
    return {**k, "source": c.get("source")}, None


def main() -> int:
    # The contract is ONE JSON line on stdout.  Libraries print there too (RCCL's version
    # banner at communicator creation), so fd 1 points at stderr for the whole run and the
    # JSON line is written to the saved original.
    argv = sys.argv[1:]
    args = parse_args(argv)
    # OpenMP threads (the oracle's CPU legs) that spin after a parallel region eat the cgroup's
    # CPU quota and starve the host threads of the GPU legs: passive waiting, before libgomp loads
    os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
    if args.gpus < 1:
        log("bench: --gpus must be >= 1")
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, argv)   # before any GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")
        return 2
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.launch_check:
        return launch_check(args, json_fd)

    import numpy as np
    import torch
    import torch.distributed as dist
    import deflate_compression_amd as D
    from deflate_compression_amd import shard as S

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_pg = world > 1 or bool(args.pipeline_test)
    if use_pg:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    per_rank, gen, seed, desc = WORKLOADS[args.workload]
    strong = args.workload == "enwik9"
    if args.bytes:
        per_rank = args.bytes
    full = None
    if strong:
        total = per_rank
        full = make_input(gen, total, seed)
        lo, hi = S.shard_range(total, rank, world)
        host = np.ascontiguousarray(full[lo:hi])
        if rank != 0:
            full = None
    else:
        host = make_input(gen, per_rank, seed + rank)
    n = int(host.size)
    flags = D.DMX_ZLIB if world == 1 else S.shard_flags(rank, world)
    if args.lazy:
        flags |= D.DMX_F_LAZY
    if args.split:
        flags |= D.DMX_F_SPLIT
    if args.dict:
        flags |= D.DMX_F_DICT
    if args.store_check:
        flags |= D.DMX_F_STORE_CHECK
    if args.deep:
        flags |= D.DMX_F_DEEP
    enc = D.Encoder(local, n, 32768, args.max_chain, flags)
    d_in = torch.from_numpy(host).to(dev)
    cap = D.max_compressed(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    lens = S.shard_lengths(n, dev) if (world > 1 and args.dict) else None
    halo = [None]

    def halo_exchange():
        if lens is not None:   # f1 across shards: the block before this shard, from the previous rank
            halo[0] = S.exchange_history(d_in, n, lens=lens, out=halo[0])
            enc.opts.dict, enc.opts.dict_len = (halo[0].data_ptr(), halo[0].numel()) if halo[0] is not None \
                else (None, 0)

    def step():
        halo_exchange()
        enc.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
        if world > 1 and args.gather != "none":
            r = enc.result(stream)   # chunk length (device -> host) before the exchange
            S.gather_chunks(d_out, int(r.out_len), root=None if args.gather == "all" else 0)

    # Pipelined gather (N > 1, --gather root): step i encodes into buffer i % 2 on the compute
    # stream while the chunk of step i - 1 goes to rank 0 on a comm stream.  The chunk length
    # comes back through an asynchronous 64 B copy into pinned memory; the compute stream
    # waits for the gather that last used a buffer before encoding into it again.
    pipelined = use_pg and args.gather == "root"
    last_buf = [d_out]
    if pipelined:
        d_outs = [d_out, torch.empty_like(d_out)]
        res_h = [torch.zeros(64, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        enc_done = [torch.cuda.Event(), torch.cuda.Event()]
        gat_done = [None, None]
        comm = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)

        def p_encode(i):
            k = i % 2
            if gat_done[k] is not None:
                cur.wait_event(gat_done[k])
            halo_exchange()
            enc.encode_async(d_in.data_ptr(), n, d_outs[k].data_ptr(), cap, stream)
            enc.result_async(res_h[k].data_ptr(), stream)
            enc_done[k].record(cur)
            last_buf[0] = d_outs[k]

        def p_gather(i):
            k = i % 2
            enc_done[k].synchronize()
            ln = int(np.frombuffer(res_h[k].numpy()[:8].tobytes(), dtype=np.uint64)[0])
            with torch.cuda.stream(comm):
                comm.wait_event(enc_done[k])
                S.gather_chunks(d_outs[k], ln, root=0)
                ev = torch.cuda.Event()
                ev.record(comm)
                gat_done[k] = ev

        def run(steps):
            for i in range(steps):
                p_encode(i)
                if i >= 1:
                    p_gather(i - 1)
            if steps:
                p_gather(steps - 1)
    else:
        def run(steps):
            for _ in range(steps):
                step()

    # correctness of the measured configuration (outside the timed region)
    run(1)
    torch.cuda.synchronize(dev)
    res = enc.result(stream)
    out_len = int(res.out_len)
    ok = True
    stitched = None
    z = None
    if world == 1:
        z = d_out[:out_len].cpu().numpy().tobytes()
        ok = zlib.decompress(z) == host.tobytes()
        if not ok:
            log("ERROR: stream does not inflate to the input")
    else:
        # rank 0 stitches every rank's chunk (header on rank 0's, sync flushes between, BFINAL
        # on the last) with the combined Adler-32 and inflates it against every rank's input
        comm_s = torch.cuda.current_stream(dev)
        torch.cuda.synchronize(dev)
        outs, glens = S.gather_chunks(last_buf[0], out_len, root=0)
        meta = torch.tensor([n, int(res.adler)], dtype=torch.int64, device=dev)
        metas = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(metas, meta)
        comm_s.synchronize()
        flag = torch.zeros(1, dtype=torch.int64, device=dev)
        if rank == 0:
            ns = [int(m[0].item()) for m in metas]
            ads = [int(m[1].item()) for m in metas]
            chunks = [o.cpu().numpy().tobytes() for o in outs]
            if strong:
                bounds = [S.shard_range(per_rank, r, world) for r in range(world)]
                pieces = [(lambda lo=lo, hi=hi: full[lo:hi].tobytes()) for lo, hi in bounds]
            else:
                pieces = [(lambda r=r: make_input(gen, per_rank, seed + r).tobytes()) for r in range(world)]
            t0 = time.perf_counter()
            ok = verify_stitched(chunks, ads, ns, pieces)
            stitched = {"inflates": ok, "bytes": sum(len(c) for c in chunks) + 4, "input_bytes": sum(ns),
                        "check_s": round(time.perf_counter() - t0, 2),
                        "how": "rank 0: chunks gathered over RCCL + combined Adler-32 trailer, zlib inflate, "
                               "compared with every rank's input"}
            if not ok:
                log("ERROR: the stitched multi-rank stream does not inflate to the ranks' inputs")
            flag[0] = 1 if ok else 0
        dist.broadcast(flag, 0)
        ok = bool(flag.item())
        del full
    # GPU inflate of the same stream: every block decoded in parallel from the
    # encoder's block index, compared bit for bit with the input; timed with events.  Dict
    # streams reference the previous block: the chained decode (cells + pointer jumping,
    # dmx_inflate_chained_async), also every block in parallel.
    ix, nblk = enc.block_index()
    dec = torch.empty(n, dtype=torch.uint8, device=dev)
    ist = torch.zeros(16, dtype=torch.uint8, device=dev)
    Lib = D.lib()
    inf_src = last_buf[0]
    chained = bool(args.dict)
    work = None
    if chained:
        wb = int(Lib.dmx_inflate_chained_work(n, nblk))
        work = torch.empty(wb + 256, dtype=torch.uint8, device=dev)
        wptr = (work.data_ptr() + 255) & ~255

    def inflate():
        if chained:
            rc = Lib.dmx_inflate_chained_async(inf_src.data_ptr(), out_len, ix.data_ptr(), nblk, dec.data_ptr(), n,
                                               wptr, wb, ist.data_ptr(), stream)
        else:
            rc = Lib.dmx_inflate_async(inf_src.data_ptr(), out_len, ix.data_ptr(), nblk, dec.data_ptr(), n,
                                       ist.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"GPU inflate launch: {rc}")

    if world == 1 or not chained:
        inflate()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    inf_reps = 3 if (world == 1 or not chained) else 0
    for _ in range(inf_reps):
        inflate()
    ev1.record()
    torch.cuda.synchronize(dev)
    gpu_inflate = None
    if inf_reps:
        inf_ms = ev0.elapsed_time(ev1) / inf_reps
        h = ist.cpu().numpy()
        inf_status = int(np.frombuffer(h[:4].tobytes(), np.int32)[0])
        inf_len = int(np.frombuffer(h[8:16].tobytes(), np.uint64)[0])
        inf_ok = inf_status == 0 and inf_len == n and bool(torch.equal(dec, d_in))
        if not inf_ok:
            log(f"ERROR: GPU inflate status {inf_status}, {inf_len} of {n} bytes, or a byte mismatch")
            ok = False
        gpu_inflate = {"GBps_out": round(n / inf_ms / 1e6, 3), "ms": round(inf_ms, 4), "bit_exact": inf_ok,
                       "mode": "chained: every block in parallel into 16-bit cells (references to the bytes "
                               "before the block), references resolved by pointer jumping" if chained else
                               "indexed: one single-wave workgroup per block",
                       "kernel": "dmx_inflate_index_kernel<true> + dmx_cells_*" if chained else
                                 "dmx_inflate_index_kernel"}
        if chained:   # how fast the chains resolve: reference-list lengths after prep and each jump launch
            lists = (ctypes.c_uint32 * 41)()
            if Lib.dmx_inflate_chained_lists(wptr, lists, 41, stream) == 0:
                ls = list(lists)
                while len(ls) > 1 and ls[-1] == 0 and ls[-2] == 0:
                    ls.pop()
                gpu_inflate["reference_lists"] = ls
    del work
    del dec
    run(args.warmup)
    torch.cuda.synchronize(dev)
    # every stage's HIP-event time from an untimed pass (an event at every stage boundary costs
    # a few us of idle per boundary: on C4 that was 0.48 -> 0.59 ms per step); the timed region
    # then records only the dominant stage's two events, for the roofline's launch time, on
    # every TIMING_EVERY-th step (a sample of the timed steps, at a quarter of the idle)
    enc.set_timing(True)
    run(max(args.steps, 1))
    torch.cuda.synchronize(dev)
    stage_ms, nstage = enc.stage_times()
    dom = max((k for k in stage_ms if k != "total"), key=stage_ms.get)
    enc.set_timing(True, stage=dom, every=TIMING_EVERY)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    dom_ms_timed, dom_n_timed = enc.stage_times()
    dom_ms_timed = dom_ms_timed[dom]
    enc.set_timing(False)
    dt = t1 - t0
    fb_total = int(enc.result(stream).nsortfallback_total)   # every encode of this context so far
    # a longer run of the same step (outside the timed region): the timed region above is what
    # the driver asked for; this shows the rate holds over about a second of back-to-back steps
    long_run = None
    if world == 1 and args.long_run > 0 and not pipelined:
        reps = max(args.steps, int(args.long_run / max(dt / max(args.steps, 1), 1e-4)))
        torch.cuda.synchronize(dev)
        q0 = time.perf_counter()
        run(reps)
        torch.cuda.synchronize(dev)
        q1 = time.perf_counter()
        long_run = {"steps": reps, "s": round(q1 - q0, 3), "value": round(n * reps / (q1 - q0) / 1e9, 3),
                    "ms_per_step": round((q1 - q0) / reps * 1e3, 4)}
    # the speed / size curve over max_chain, same input and flags (outside the timed region)
    tradeoff = []
    if world == 1 and args.tradeoff and not pipelined:
        for kc in [int(x) for x in args.tradeoff.split(",") if x.strip()]:
            if kc == args.max_chain:
                continue
            te = D.Encoder(local, n, 32768, kc, flags)
            te.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
            t_len = int(te.result(stream).out_len)
            torch.cuda.synchronize(dev)
            q0 = time.perf_counter()
            for _ in range(5):
                te.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
            torch.cuda.synchronize(dev)
            q1 = time.perf_counter()
            te.close()
            tradeoff.append({"max_chain": kc, "value": round(n * 5 / (q1 - q0) / 1e9, 3), "unit": "GB/s",
                             "ratio": round(t_len / n, 5), "compressed_bytes": t_len, "steps": 5})
    exh = None
    exh_stream = None
    if world == 1 and args.max_chain != 0 and args.exhaustive_steps > 0:
        # the reference's own parse (every earlier position of the bucket), same input
        ex = D.Encoder(local, n, 32768, 0, flags & ~(D.DMX_F_LAZY | D.DMX_F_DICT | D.DMX_F_SPLIT | D.DMX_F_STORE_CHECK
                                                    | D.DMX_F_DEEP))
        ex.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
        ex_len = int(ex.result(stream).out_len)
        torch.cuda.synchronize(dev)
        e0 = time.perf_counter()
        for _ in range(args.exhaustive_steps):
            ex.encode_async(d_in.data_ptr(), n, d_out.data_ptr(), cap, stream)
        torch.cuda.synchronize(dev)
        e1 = time.perf_counter()
        ex_res = ex.result(stream)
        exh_stream = d_out[:ex_len].cpu().numpy().tobytes()
        ex.close()
        exh = {"value": round(n * args.exhaustive_steps / (e1 - e0) / 1e9, 3), "unit": "GB/s",
               "ratio": round(ex_len / n, 5), "compressed_bytes": ex_len, "steps": args.exhaustive_steps,
               "nsortfallback_total": int(ex_res.nsortfallback_total)}
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        nn = torch.tensor([n, out_len], dtype=torch.int64, device=dev)
        dist.all_reduce(nn)
        tot_in, tot_out = int(nn[0].item()), int(nn[1].item())
    else:
        tot_in, tot_out = n, out_len

    if rank == 0:
        ms_step = dt / args.steps * 1e3
        value = tot_in * args.steps / dt / 1e9
        kname = {"pre": "dmx_hist_kernel_t" if args.dict else "dmx_store_check_kernel",
                 "huff": "dmx_split_plan_kernel" if args.split else "dmx_huff_kernel"}.get(dom, f"dmx_{dom}_kernel")
        dom_ms = dom_ms_timed   # HIP events around the dominant stage inside the timed region
        algo_bytes = n + out_len   # per launch on this rank: input read + stream written
        achieved = algo_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        parse = parse_str(args)
        traffic, valu, why = None, None, None
        if args.traffic_csv:
            try:
                import importlib.util
                spec = importlib.util.spec_from_file_location("pmc", os.path.join(REPO, "tools", "pmc.py"))
                pmc = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(pmc)
                traffic = pmc.traffic_per_launch(args.traffic_csv, kname)
                if traffic:
                    traffic["source"] = "this run's --traffic-csv"
            except Exception as e:  # pragma: no cover
                log("traffic csv unreadable:", e)
        ctr, why = roofline_counters(kname, parse, args.workload)
        nblk_all = int(res.nblocks)
        if ctr:
            parsed_blocks = nblk_all - int(res.nstored)   # K0-stored blocks skip the match kernel
            if traffic is None and ctr.get("fetch_bytes_per_block") is not None:
                traffic = {"bytes": round((ctr["fetch_bytes_per_block"] + ctr["write_bytes_per_block"]) * nblk_all),
                           "fetch_bytes": round(ctr["fetch_bytes_per_block"] * nblk_all),
                           "write_bytes": round(ctr["write_bytes_per_block"] * nblk_all),
                           "correction": "FETCH_SIZE KiB x2 (gfx950 half-count), WRITE_SIZE KiB x1",
                           "source": f"profile-run counters, {ctr['source']} (per block x this launch's blocks)"}
            if ctr.get("valu_per_block") and dom_ms > 0:
                vpl = ctr["valu_per_block"] * parsed_blocks
                va = vpl / (dom_ms * 1e-3) / 1e9
                valu = {"achieved": round(va, 1), "peak": round(VALU_PEAK_GIPS, 1), "unit": "G VALU wave-instr/s",
                        "frac": round(va / VALU_PEAK_GIPS, 4), "instr_per_launch": round(vpl),
                        "instr_per_block": round(ctr["valu_per_block"]),
                        "peak_basis": "256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 integer VALU instruction "
                                      "(tools/valu_peak.hip: 526-630 G/s measured)",
                        "source": f"SQ_INSTS_VALU per block from {ctr['source']} x this launch's parsed blocks, "
                                  "divided by this run's HIP-event launch time"}
        cpu, info = ({}, cpu_info())
        e2e = zl6 = real = None
        if world == 1 and args.cpu_budget > 0:
            # the GPU-side legs first: the CPU legs' threads must not share the host with them
            try:
                e2e = end_to_end(host, args)
            except Exception as e:  # pragma: no cover
                log("end-to-end fd API leg failed:", e)
            if args.real_text and args.workload == "text":
                real = real_text_leg(flags, args, dev, local, stream)
                if not (real["parity_vs_port"] and real["inflates"]):
                    log("ERROR: real-text stream differs from the port's or does not inflate")
                    ok = False
            cpu, info = cpu_baselines(host, args, args.cpu_budget)
            zl6 = len(zlib.compress(host.tobytes(), 6))   # context: zlib -6 on the same input
        base = cpu.get("same_parse")
        size_pct = s_ref_bytes = None
        # full-size parity witness: the port's stream at the GPU line's exact parse,
        # over the whole input, must equal the GPU stream byte for byte; a mismatch fails the run
        parity = parity_exh = None
        if cpu.get("same_parse_stream") is not None and z is not None:
            parity = cpu["same_parse_stream"] == z
            if not parity:
                log("ERROR: GPU stream differs from the CPU port's stream at the same parse")
                ok = False
        sref = cpu.get("s_ref_stream")
        if sref is not None:
            s_ref_bytes = len(sref)
            size_pct = round((out_len / s_ref_bytes - 1) * 100, 3)
            for t in tradeoff:
                t["size_vs_ref_pct"] = round((t["compressed_bytes"] / s_ref_bytes - 1) * 100, 3)
            if exh_stream is not None:
                parity_exh = exh_stream == sref
                exh["parity_vs_port"] = parity_exh
                if not parity_exh:
                    log("ERROR: GPU exhaustive stream differs from the CPU port's (the reference parse)")
                    ok = False
        line = {
            "metric": "encode GB/s (uncompressed in) + compression ratio vs CPU ref, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": desc,
                "name": args.workload,
                "bytes_per_rank": n,
                "block": 32768,
                "parse": parse,
                "parallelism": f"blocks sharded over {world} GPU(s)" + (f", gather={args.gather}" if world > 1 else "")
                               + (", pipelined" if pipelined else ""),
            },
            "ratio": round(out_len / n, 5),
            "parity_vs_port": parity,
            "nsortfallback": fb_total,
            "size_vs_ref_pct": size_pct,
            "s_ref_bytes": s_ref_bytes,
            "exhaustive": exh,
            "tradeoff": tradeoff or None,
            "long_run": long_run,
            "compressed_bytes_rank0": out_len,
            "compressed_bytes_all": tot_out,
            "inflate_ok": ok,
            "stitched": stitched,
            "gpu_inflate": gpu_inflate,
            "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
            "stage_ms_source": "HIP events at every stage boundary, an untimed pass of the same steps before the "
                               "timed region (the timed region records only the dominant stage's two events)",
            "roofline": {
                "bound": "hbm" if kname == "dmx_store_check_kernel" else "valu",
                "kernel": kname,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "frac_basis": "HBM: algorithmic bytes (input + stream) per launch / launch time / 8 TB/s" +
                              ("" if kname == "dmx_store_check_kernel" else
                               "; the binding roofline is roofline.valu (integer VALU issue)"),
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_detail": traffic,
                "algorithmic_bytes_per_launch": algo_bytes,
                "launch_ms": round(dom_ms, 4),
                "launch_ms_source": f"HIP events around stage '{dom}' on the encode stream on every "
                                    f"{TIMING_EVERY}th step of the timed region ({dom_n_timed} of {args.steps})",
                "launches_timed": dom_n_timed,
                "valu": valu,
                "counters_note": why,
            },
            "end_to_end_fd_api": e2e,
            "zlib6": None if zl6 is None else {"ratio": round(zl6 / n, 5), "compressed_bytes": zl6,
                                                 "ours_vs_zlib6_pct": round((out_len / zl6 - 1) * 100, 3)},
            "cpu_baseline": base,
            "cpu_baseline_exhaustive": cpu.get("exhaustive"),
            "cpu_baseline_1core": cpu.get("same_parse_1core"),
            "real_text": real,
            "cpu_baseline_reference": cpu.get("reference"),
            "host": info,
        }
        if base and base["value"]:
            line["gpu_over_cpu"] = round(value / base["value"], 1)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    enc.close()
    if use_pg:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
