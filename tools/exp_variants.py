"""Diagnostic: build copies of the match kernel with one part knocked out (output is wrong
by construction) to see what a phase's time is made of.  Usage (build, CPU):
  python tools/exp_variants.py build      -> build/exp/libdmx_<name>.so
and on the GPU box:
  python tools/exp_variants.py run        -> P0 / search / walk cycles per variant
"""
import os, subprocess, sys, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "deflate_compression_amd", "csrc")
OUT = os.path.join(R, "build", os.environ.get("DMX_EXP_DIR", "exp"))

VARIANTS = {
    "base": [],
    # P0 knockouts (round 2): what each LDS operation of the two sort passes costs
    "nocnt1": [("        count_add<RUNCHK>(C + (wave << 7), h & 127u, x < nvl, false);\n", "")],
    "nocnt2": [("        count_add<RUNCHK>(C2, ((dst >> 11) << 6) | (h >> 7), valid, false);   // pass 2: (wave, digit)\n", "")],
    "nosc1": [("            L.sorted[dst] = (uint16_t)x;\n            D2[dst] = (uint8_t)(h >> 7);\n", "")],
    "nosc2": [("            if (valid) L.sorted[dst] = (uint16_t)p;\n", "            if (valid && dst == 0xFFFFu) L.sorted[0] = (uint16_t)p;\n")],
    "norank": [("    if (!RUNCHK) return valid ? atomicAdd(&T[v], 1u) : 0u;", "    if (!RUNCHK) return valid ? ((T[v] + (threadIdx.x & 63)) & 32767u) : 0u;")],
    # walk: the distance permute's random reads (winner entries) and scatter stores
    "noperm_rd": [("                    else if (jj) dist = ((pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu) - (uint32_t)L.sorted[kk - jj];",
                   "                    else if (jj) dist = jj;")],
    "noperm_st": [("                    L.sorted[(pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu] = (uint16_t)(dw[e >> 1] >> (16 * (e & 1)));",
                   "                    L.sorted[kk] = (uint16_t)(dw[e >> 1] >> (16 * (e & 1)));")],
    # P0 rank by a wave-level multisplit: same-digit lane masks from 7 ballots,
    # the rank by popcount, one LDS add per (wave, distinct digit), the base by ds_bpermute
    "ms_rank": [("    if (!RUNCHK) return valid ? atomicAdd(&T[v], 1u) : 0u;",
                 """    if (!RUNCHK) {
        uint64_t eq = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 7; b++) {
            const uint64_t bb = __ballot(valid && ((v >> b) & 1u));
            eq &= ((v >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t lead = eq ? (uint32_t)__builtin_ctzll(eq) : 0u;
        uint32_t base = 0;
        if (valid && (eq & lt) == 0) base = atomicAdd(&T[v], (uint32_t)__popcll(eq));
        base = (uint32_t)__shfl((int)base, (int)lead);
        return valid ? base + (uint32_t)__popcll(eq & lt) : 0u;
    }""")],
    # K0 (C4 noise): the 4-gram bitmap's LDS atomics, knocked out and compacted
    "k0_nobm": [("                atomicOr(&bm[x >> 20], 1u << ((x >> 15) & 31));\n", "")],
    "k0_compact": [("""#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t lo = w[j >> 2], hi = w[(j >> 2) + 1];
            const uint32_t g4 = (j & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(j & 3)) : lo;
            if (((uint32_t)j & smask) == 0 && p + j < bn) atomicAdd(&hist[(lo >> (8 * (j & 3))) & 0xFFu], 1u);
            const uint32_t x = g4 * 0x9E3779B1u;
            if (p + j + 4 <= bn && !(x & (7u << 11))) {   // sampled by content
                qn++;
                atomicOr(&bm[x >> 20], 1u << ((x >> 15) & 31));
            }
        }
""", """        uint32_t sm = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t lo = w[j >> 2], hi = w[(j >> 2) + 1];
            const uint32_t g4 = (j & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(j & 3)) : lo;
            if (((uint32_t)j & smask) == 0 && p + j < bn) atomicAdd(&hist[(lo >> (8 * (j & 3))) & 0xFFu], 1u);
            const uint32_t x = g4 * 0x9E3779B1u;
            if (p + j + 4 <= bn && !(x & (7u << 11))) sm |= 1u << j;
        }
        qn += (uint32_t)__builtin_popcount(sm);
        while (sm) {
            const uint32_t j = (uint32_t)__builtin_ctz(sm), q = j >> 2;
            sm &= sm - 1;
            const uint32_t lo = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
            const uint32_t hi = q == 0 ? w[1] : q == 1 ? w[2] : q == 2 ? w[3] : w[4];
            const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, j & 3) * 0x9E3779B1u;
            atomicOr(&bm[x >> 20], 1u << ((x >> 15) & 31));
        }
""")],
    # exhaustive later windows: filter steps with their LDS reads in flight together
    "xu1": [("#define XU 4 ", "#define XU 1 ")],
    "xu2": [("#define XU 4 ", "#define XU 2 ")],
    "xu8": [("#define XU 4 ", "#define XU 8 ")],
    "w0h4_4": [("#define DMX_W0H4 8 ", "#define DMX_W0H4 4 ")],
    "w0h4_12": [("#define DMX_W0H4 8 ", "#define DMX_W0H4 12 ")],
    "w0h4_16": [("#define DMX_W0H4 8 ", "#define DMX_W0H4 16 ")],
    # P1 (K <= 8) knockouts: the sort check, the result stores, the queued extension
    "p1_nochk": [("                    if (__ballot(act && ei >= 1 && pk > sk)) L.sortbad = 1;", "")],
    "p1_nostore": [("                store_short<DICT>(L, k, i, m >= 3 ? m : 0u, m >= 3 ? 8u - (jkey & 7u) : 0u, hbk);", "                if (m == 0x1234u) L.len8[i] = 1;")],
    "p1_noq": [("                ext_queue<DICT, RUNS>(L, bn, K, Qw, qn, lane, hbk);", "")],
    # Huffman plans without the 8-waves-per-SIMD request (7 per SIMD, no SGPR spills)
    "huff7": [("__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void dmx_huff_kernel(",
               "__global__ __launch_bounds__(64) void dmx_huff_kernel("),
              ("__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void dmx_split_plan_kernel(",
               "__global__ __launch_bounds__(64) void dmx_split_plan_kernel(")],
    "noseed": [("        if (H4 && act) bestkey = seed;   // the best", "        if (H4 && act) bestkey = 0 * seed;   // the best")],
    "now1": [("            if (jmax == 0) break;\n            iters += jmax;", "            if (jmax == 0 || jb) break;\n            iters += jmax;")],
    "nold": [("for (uint32_t u = 0; u < XU; u++) v[u] = ld4(L.data, xs[u]);", "for (uint32_t u = 0; u < XU; u++) v[u] = xs[u];")],
    "k0_nohist": [("            if (((uint32_t)j & smask) == 0 && p + j < bn) atomicAdd(&hist[(lo >> (8 * (j & 3))) & 0xFFu], 1u);\n", "")],
}

def build():
    os.makedirs(OUT, exist_ok=True)
    base = open(os.path.join(SRC, "dmx_kernels.hip")).read()
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(VARIANTS)
    for name in names:
        reps = VARIANTS[name]
        s = base
        if any(a not in s for a, _ in reps):
            print("skip", name, "(pattern no longer in the source)")
            continue
        for a, b in reps:
            s = s.replace(a, b)
        src = os.path.join(OUT, f"k_{name}.hip")
        open(src, "w").write(s)
        obj = os.path.join(OUT, f"k_{name}.o")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "--offload-arch=gfx950", "-std=c++17",
                               "-I", SRC, "-I", os.path.join(R, "include"), "-c", "-o", obj, src])
        objs = [os.path.join(R, "build", "dmx", f) for f in ("dmx_host.o", "dmx_inflate.o", "dmx_gen.o", "dmx_inflate_dev.o", "dmx_refstats.o")]
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                               os.path.join(OUT, f"libdmx_{name}.so"), obj] + objs + ["-lm", "-lpthread"])
        print("built", name)

def run():
    for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else VARIANTS):
        r = subprocess.run([sys.executable, __file__, "one", name], capture_output=True, text=True, timeout=300)
        print(name, r.stdout.strip() or r.stderr[-300:])

def one_k0(name):
    """C4: 1 GiB of noise with the store check; K0's HIP-event time ('pre') and the stream's hash."""
    sys.path.insert(0, R)
    import hashlib, numpy as np, torch
    import deflate_compression_amd as D
    D.LIB_PATH = os.path.join(OUT, f"libdmx_{name}.so")
    n = 1 << 30
    t = torch.from_numpy(D.gen_random(n)).cuda()
    e = D.Encoder(0, n, max_chain=6, flags=D.DMX_ZLIB | D.DMX_F_LAZY | D.DMX_F_STORE_CHECK)
    out, r = e.compress_tensor(t)
    e.set_timing(True)
    for _ in range(10):
        out, r = e.compress_tensor(t)
    st = e.stage_times()
    h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    e.close()
    print(json.dumps({"stage_ms": st, "bytes": int(out.numel()), "sha": h}))

def one_split(name):
    """C3 text, K=6 lazy: the Huffman stage ('huff', HIP events) unsplit and with DMX_F_SPLIT."""
    sys.path.insert(0, R)
    import hashlib, numpy as np, torch
    import deflate_compression_amd as D
    D.LIB_PATH = os.path.join(OUT, f"libdmx_{name}.so")
    n = 100_000_000
    t = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    res = {}
    for tag, fl in (("plain", 0), ("split", D.DMX_F_SPLIT)):
        e = D.Encoder(0, n, max_chain=6, flags=D.DMX_ZLIB | D.DMX_F_LAZY | fl)
        out, r = e.compress_tensor(t)
        e.set_timing(True)
        for _ in range(10):
            out, r = e.compress_tensor(t)
        st, cnt = e.stage_times()
        res[tag] = {"huff_ms": round(st["huff"] / max(cnt, 1), 4), "sha": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}
        e.close()
    print(json.dumps(res))

def run_split():
    for name in sys.argv[2].split(","):
        r = subprocess.run([sys.executable, __file__, "one_split", name], capture_output=True, text=True, timeout=300)
        print(name, r.stdout.strip() or r.stderr[-300:], flush=True)

def run_k0():
    for name in sys.argv[2].split(","):
        r = subprocess.run([sys.executable, __file__, "one_k0", name], capture_output=True, text=True, timeout=300)
        print(name, r.stdout.strip() or r.stderr[-300:], flush=True)

def one(name):
    os.environ["DMX_STAMPS"] = "1"
    sys.path.insert(0, R)
    import numpy as np, torch
    import deflate_compression_amd as D
    D.LIB_PATH = os.path.join(OUT, f"libdmx_{name}.so")
    n = 20_000_000
    t = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    lazy = D.DMX_F_LAZY if os.environ.get("EXP_LAZY", "1") == "1" else 0
    e = D.Encoder(0, n, max_chain=int(os.environ.get("EXP_K", "6")), flags=D.DMX_ZLIB | lazy)
    for _ in range(2):
        out, r = e.compress_tensor(t)
    st = e.stamps(r.nblocks).astype(np.float64)
    e.close()
    import hashlib
    sha = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"sha": sha, "w1": round(st[:, 5].mean() / 1e3, 1), "walk": round(st[:, 2].mean() / 1e3, 1), "p0": round(st[:, 0].mean() / 1e3, 1), "pass1_end": round(st[:, 9].mean() / 1e3, 1),
                      "pass2_end": round(st[:, 10].mean() / 1e3, 1), "search": round(st[:, 1].mean() / 1e3, 1),
                      "deferred": round(st[:, 3].mean() / 1e3, 1), "iters": round(st[:, 4].mean() / 16, 1),
                      "h4_sort_end": round((st[:, 15] % 2**48).mean() / 1e3, 1), "total": round(st[:, 7].mean() / 1e3, 1)}))

if __name__ == "__main__":
    if sys.argv[1] == "one_k0":
        one_k0(sys.argv[2])
    elif sys.argv[1] == "one_split":
        one_split(sys.argv[2])
    else:
        {"build": build, "run": run, "run_k0": run_k0, "run_split": run_split}.get(sys.argv[1], lambda: one(sys.argv[2]))()
