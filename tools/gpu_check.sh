#!/bin/bash
# One GPU-box pass: the -m gpu suite (optionally a -k filter), then the default bench line.
# A failing test (pytest rc 1) still lets the bench run; a timeout, abort, crash or fault
# (any other status) ends the script there, so nothing else touches the GPU after it.
# usage (on the box): bash tools/gpu_check.sh TAG [PYTEST_K] [BENCH_ARGS...]
set -uo pipefail
TAG=$1
K=${2:-}
shift 2 2>/dev/null || shift $#
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export DMX_TEST_HEARTBEAT=$OUT/heartbeat.txt   # long tests append progress here (the silence watchdog)
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python3 -u -m pytest "$R/tests" -m gpu -x -v -p no:cacheprovider --timeout 240 \
    --timeout-method thread "${KARG[@]}" > "$OUT/pytest.log" 2>&1
rc=$?
tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "pytest status $rc: stopping"; exit $rc; fi
timeout -k 10 600 python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?
tail -3 "$OUT/bench.err"
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], 'parity', d.get('parity_vs_port'), 'fb', d.get('nsortfallback'), 'stage', d['stage_ms'])
print('exh', d.get('exhaustive'))
print('real', d.get('real_text'))
print('cpu', d.get('cpu_baseline', {}).get('value'), d.get('cpu_baseline', {}).get('cores'), d.get('cpu_baseline_share'))
" || true
exit $(( rc == 0 ? brc : rc ))
