#!/bin/bash
# Round-end confirmation on one MI355X: the whole GPU suite, smoke(), the default bench line
# (the driver's command) and a kernel-trace summary of the bench configuration.
# usage (on the box): bash tools/final_check.sh TAG
set -uo pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python3 "$R/bench.py" > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit 1
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['ms_per_step'], d['stage_ms'], d.get('exhaustive', {}).get('value'), d.get('gpu_inflate', {}).get('value'))"
