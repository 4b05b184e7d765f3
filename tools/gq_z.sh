# tests + split bench (gpu_check) + the default bench line, quiet legs
set -uo pipefail
T=${1:-r03_z}
bash tools/gpu_check.sh $T "" --split 1 --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0 || exit $?
timeout -k 10 300 python3 bench.py --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0 > gpurun_out/$T/bench_default.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_default.json')); print('default', d['value'], d['stage_ms'])"
