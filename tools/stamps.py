"""Diagnostic: per-phase cycle stamps of the match kernel (run with DMX_STAMPS=1)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DMX_STAMPS"] = "1"
import numpy as np, torch
import deflate_compression_amd as D
if os.environ.get("DMX_LIBV"): D.LIB_PATH = os.environ["DMX_LIBV"]

def run(kind, n, mc, flags=D.DMX_ZLIB | D.DMX_F_LAZY):
    if kind == "bitdump":   # the small-alphabet input of tests/deep_inputs.py
        from tests.deep_inputs import bitdump
        a = np.frombuffer(bitdump(n, 1), dtype=np.uint8).copy()
    else:
        a = D.gen_text(n, 0xE5818) if kind == "text" else (D.gen_random(n, 1) if kind == "random" else np.zeros(n, np.uint8))
    t = torch.from_numpy(a).cuda()
    e = D.Encoder(0, n, max_chain=mc, flags=flags)
    for _ in range(2):
        out, r = e.compress_tensor(t)
    st = e.stamps(r.nblocks).astype(np.float64)
    e.close()
    print(json.dumps({"kind": kind, "mc": mc, "p0_kcyc": round(st[:, 0].mean() / 1e3, 1),
                      "search_kcyc": round(st[:, 1].mean() / 1e3, 1), "walk_kcyc": round(st[:, 2].mean() / 1e3, 1),
                      "deferred_kcyc": round(st[:, 3].mean() / 1e3, 1), "iters_per_wave": round(st[:, 4].mean() / 16, 1),
                      "w1_kcyc": round(st[:, 5].mean() / 1e3, 1), "w1w3_kcyc": round(st[:, 6].mean() / 1e3, 1),
                      "total_kcyc": round(st[:, 7].mean() / 1e3, 1),
                      "p0_staged_kcyc": round(st[:, 8].mean() / 1e3, 1), "p0_pass1_end_kcyc": round(st[:, 9].mean() / 1e3, 1),
                      "p0_pass2_end_kcyc": round(st[:, 10].mean() / 1e3, 1),
                      "walk_rounds": round(st[:, 11].mean(), 2),
                      **({} if flags & D.DMX_F_DICT else {"p3_list_kcyc": round(st[:, 12].mean() / 1e3, 1), "p3_done_kcyc": round(st[:, 13].mean() / 1e3, 1)}), "walk_fallback_frac": round(float((st[:, 11] >= 8).mean()), 3),
                      **({"h4_trigram_pass_end_kcyc": round((st[:, 14] % 2**48).mean() / 1e3, 1), "h4_passes": round((st[:, 14] // 2**48).mean(), 3), "h4_sort_end_kcyc": round((st[:, 15] % 2**48).mean() / 1e3, 1), "h4_deferred_walks": round((st[:, 15] // 2**48).mean(), 1)}
                         if mc == 0 and not flags & D.DMX_F_DICT else {}),
                      **({"p1b_end_kcyc": round(st[:, 14].mean() / 1e3, 1), "w1_walk_end_kcyc": round(st[:, 15].mean() / 1e3, 1)}
                         if mc != 0 and not flags & D.DMX_F_DICT else {}),
                      **({"hist_staged_kcyc": round(st[1:, 12].mean() / 1e3, 1), "hist_total_kcyc": round(st[1:, 13].mean() / 1e3, 1)}
                         if flags & D.DMX_F_DICT else {})}))

# args: kind:max_chain[:opts]  (opts: d = with the cross-block dictionary, DMX_F_DICT; g = greedy, no lazy;
# e = DMX_F_DEEP; kind text | random | zeros | bitdump)
cfgs = [("text", 1, ""), ("text", 16, ""), ("text", 0, ""), ("random", 0, ""), ("zeros", 0, "")]
if len(sys.argv) > 1:
    cfgs = [(a.split(":") + [""])[:3] for a in sys.argv[1:]]
for kind, mc, opt in cfgs:
    fl = D.DMX_ZLIB | (0 if "g" in opt else D.DMX_F_LAZY) | (D.DMX_F_DICT if "d" in opt else 0) | \
        (D.DMX_F_DEEP if "e" in opt else 0)
    run(kind, 20_000_000 if kind == "text" else (4 << 20 if kind == "bitdump" else 64 << 20), int(mc), fl)
