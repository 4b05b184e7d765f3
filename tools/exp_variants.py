"""Diagnostic: build copies of the match kernel with one part knocked out (output is wrong
by construction) to see what a phase's time is made of.  Usage (build, CPU):
  python tools/exp_variants.py build      -> build/exp/libdmx_<name>.so
and on the GPU box:
  python tools/exp_variants.py run        -> P0 / search / walk cycles per variant
"""
import os, subprocess, sys, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "deflate_compression_amd", "csrc")
OUT = os.path.join(R, "build", "exp")

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
        objs = [os.path.join(R, "build", "dmx", f) for f in ("dmx_host.o", "dmx_inflate.o", "dmx_gen.o", "dmx_inflate_dev.o")]
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                               os.path.join(OUT, f"libdmx_{name}.so"), obj] + objs + ["-lm", "-lpthread"])
        print("built", name)

def run():
    for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else VARIANTS):
        r = subprocess.run([sys.executable, __file__, "one", name], capture_output=True, text=True, timeout=300)
        print(name, r.stdout.strip() or r.stderr[-300:])

def one(name):
    os.environ["DMX_STAMPS"] = "1"
    sys.path.insert(0, R)
    import numpy as np, torch
    import deflate_compression_amd as D
    D.LIB_PATH = os.path.join(OUT, f"libdmx_{name}.so")
    n = 20_000_000
    t = torch.from_numpy(D.gen_text(n, 0xE5818)).cuda()
    e = D.Encoder(0, n, max_chain=int(os.environ.get("EXP_K", "6")), flags=D.DMX_ZLIB | D.DMX_F_LAZY)
    for _ in range(2):
        out, r = e.compress_tensor(t)
    st = e.stamps(r.nblocks).astype(np.float64)
    e.close()
    print(json.dumps({"w1": round(st[:, 5].mean() / 1e3, 1), "walk": round(st[:, 2].mean() / 1e3, 1), "p0": round(st[:, 0].mean() / 1e3, 1), "pass1_end": round(st[:, 9].mean() / 1e3, 1),
                      "pass2_end": round(st[:, 10].mean() / 1e3, 1), "search": round(st[:, 1].mean() / 1e3, 1),
                      "total": round(st[:, 7].mean() / 1e3, 1)}))

if __name__ == "__main__":
    {"build": build, "run": run}.get(sys.argv[1], lambda: one(sys.argv[2]))()
