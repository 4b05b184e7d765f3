# dict / exhaustive parity tests, the dict bench line (quiet legs), exhaustive stamps
set -uo pipefail
T=${1:-r03_d2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dict.py tests/test_gpu_exhaustive.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --dict 1 --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --long-run 0 --real-text 0 > gpurun_out/$T/bench_dict.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_dict.json')); print('dict', d['value'], d['stage_ms'], d['ratio'])"
EXP_K=0 EXP_LAZY=0 DMX_EXP_DIR=exp3 timeout -k 10 300 python3 tools/exp_variants.py run base > gpurun_out/$T/exh.txt 2>&1; cat gpurun_out/$T/exh.txt
