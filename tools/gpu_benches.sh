#!/bin/bash
# Secondary bench lines on one MI355X (no CPU legs): C4 noise, the dictionary mode, zeros,
# split, C5 on one GPU, then a kernel-trace summary of the default configuration.
# usage (on the box): bash tools/gpu_benches.sh TAG [CONFIG...]   CONFIG in random dict zeros split enwik9 trace
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CFGS=${*:-random dict zeros split enwik9 trace}
Q="--cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0"
for c in $CFGS; do
    case $c in
        random) A="--workload random $Q" ;;
        zeros)  A="--workload zeros $Q" ;;
        dict)   A="--dict 1 $Q" ;;
        split)  A="--split 1 $Q" ;;
        enwik9) A="--workload enwik9 $Q" ;;
        trace)  A="" ;;
        *) echo "unknown config $c"; exit 2 ;;
    esac
    if [ "$c" = trace ]; then
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
            python3 "$R/bench.py" --steps 5 --warmup 1 $Q > "$OUT/bench_trace.json" 2> "$OUT/trace.err") || exit 1
        find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
        continue
    fi
    timeout -k 10 300 python3 "$R/bench.py" $A > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "bench $c status $rc: stopping"; tail -5 "$OUT/bench_$c.err"; exit $rc; fi
    python3 -c "
import json; d=json.load(open('$OUT/bench_$c.json'))
print('$c', d['value'], d['ms_per_step'], d['stage_ms'], d.get('ratio'), d.get('gpu_inflate'))
" || true
done
