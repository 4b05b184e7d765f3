set -uo pipefail
T=${1:-r03_eq}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dict.py tests/test_gpu_split.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || exit $rc
EXP_K=6 EXP_LAZY=1 DMX_EXP_DIR=exp3 timeout -k 10 300 python3 tools/exp_variants.py run base,eq_old,base,eq_old > gpurun_out/$T/eq.txt 2>&1; cat gpurun_out/$T/eq.txt
