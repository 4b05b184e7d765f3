#!/bin/bash
# One GPU-box pass for a round's evidence: GPU parity tests, kernel-trace stats,
# the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes, no other tracing), one SQ
# pass, all on the bench configuration itself, then tools/roofline_counters.json (the
# per-block counters bench.py's roofline reads) and the bench line.
# usage (on the box):  bash tools/profile_round.sh r02_v1 [extra bench args]
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BA="--cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 $*"
echo "[1/6] pytest -m gpu"; timeout -k 10 900 python3 -u -m pytest "$R/tests" -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
echo "[2/6] kernel trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 $BA > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo "[3/6] pmc FETCH_SIZE"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f" -o f -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > "$OUT/bench_pmc_f.json" 2> "$OUT/pmc_f.err"
echo "[4/6] pmc WRITE_SIZE"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w" -o w -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_w.err"
echo "[5/6] pmc SQ"; timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_sq" -o sq -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_sq.err"
python3 "$R/tools/pmc.py" "$OUT/pmc_f,$OUT/pmc_w" > "$OUT/pmc_summary.txt"
python3 "$R/tools/pmc.py" "$OUT/pmc_sq" > "$OUT/sq_summary.txt"
python3 - "$OUT" "$R" "$TAG" <<'PY'
import json, subprocess, sys
out, r, tag = sys.argv[1:4]
b = json.load(open(f"{out}/bench_pmc_f.json"))
nblk = -(-b["config"]["bytes_per_rank"] // 32768)
wl = b["config"]["name"]
parse = b["config"]["parse"]
stored = 0   # the text / zeros configurations store no block through K0
cj = subprocess.check_output([sys.executable, f"{r}/tools/pmc.py", "--counters-json", f"{out}/pmc_f,{out}/pmc_w",
                              f"{out}/pmc_sq", str(nblk), str(nblk - stored), f"profiles/{tag}", parse, wl])
open(f"{out}/roofline_counters.json", "wb").write(cj)
print(cj.decode())
PY
echo "[6/6] bench"; timeout -k 10 400 python3 "$R/bench.py" --traffic-csv "$OUT/pmc_f,$OUT/pmc_w" $* > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
