#!/bin/bash
# C4 (1 GiB random, the stored-block path) evidence: kernel trace, the two PMC passes
# (separate runs, no other tracing) and the bench line with this run's traffic.
# usage (on the box):  bash tools/profile_c4.sh TAG
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BA="--workload random --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0"
echo "[1/4] kernel trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 $BA > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
echo "[2/4] pmc FETCH_SIZE"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f" -o f -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_f.err"
echo "[3/4] pmc WRITE_SIZE"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w" -o w -- python3 "$R/bench.py" --steps 2 --warmup 0 $BA > /dev/null 2> "$OUT/pmc_w.err"
python3 "$R/tools/pmc.py" "$OUT/pmc_f,$OUT/pmc_w" > "$OUT/pmc_summary.txt"
echo "[4/4] bench"; timeout -k 10 400 python3 "$R/bench.py" --workload random --traffic-csv "$OUT/pmc_f,$OUT/pmc_w" --cpu-budget 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
