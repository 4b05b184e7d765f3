#!/bin/bash
# Kernel-trace summaries of the dict bench (chained inflate included) and the C4 noise bench,
# after the store-check / dict GPU tests.  usage (on the box): bash tools/gpu_prof_dict.sh TAG
set -uo pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest "$R/tests/test_store_check.py" "$R/tests/test_gpu_dict.py" -m gpu -x -v -p no:cacheprovider \
    --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
Q="--cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0 --steps 5 --warmup 1"
cd /tmp
for c in dict random; do
    A=$([ $c = dict ] && echo "--dict 1" || echo "--workload random")
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$c" -o run -- \
        python3 "$R/bench.py" $A $Q > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -5 "$OUT/bench_$c.err"; exit 1; }
    find "$OUT/tr_$c" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$c.csv" \;
    python3 -c "
import csv,json
d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['stage_ms'], d.get('gpu_inflate'))
for r in csv.DictReader(open('$OUT/kernel_stats_$c.csv')):
    print('  ', r['Name'][:60], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"
done
if [ -x "$R/tools/copy_bw" ]; then
    timeout -k 10 120 "$R/tools/copy_bw" > "$OUT/copy_bw.txt" 2>&1 && cat "$OUT/copy_bw.txt"
fi
