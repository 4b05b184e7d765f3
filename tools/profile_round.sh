#!/bin/bash
# One GPU-box pass for a round's evidence: GPU parity tests, kernel-trace stats,
# the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes, no other tracing),
# then the bench line with roofline.traffic from those counters.
# usage (on the box):  bash tools/profile_round.sh r01_v1 [extra bench args]
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BA="--cpu-budget 0 --exhaustive-steps 0 --tradeoff= $*"
echo "[1/5] pytest -m gpu"; timeout -k 10 900 python3 -u -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
echo "[2/5] kernel trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 $BA > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo "[3/5] pmc FETCH_SIZE"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f" -o f -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_f.err"
echo "[4/5] pmc WRITE_SIZE"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w" -o w -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_w.err"
echo "[5/5] bench"; timeout -k 10 400 python3 "$R/bench.py" --traffic-csv "$OUT/pmc_f,$OUT/pmc_w" $* > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
python3 "$R/tools/pmc.py" "$OUT/pmc_f,$OUT/pmc_w" > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
