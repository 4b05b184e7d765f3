set -uo pipefail
mkdir -p gpurun_out/r03_w
EXP_K=0 EXP_LAZY=0 DMX_EXP_DIR=exp3 timeout -k 10 300 python3 tools/exp_variants.py run ${1:-base} > gpurun_out/r03_w/w0.txt 2>&1; cat gpurun_out/r03_w/w0.txt
grep -q '"sha"' gpurun_out/r03_w/w0.txt || exit 3
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_exhaustive.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r03_w/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03_w/pytest.log
exit $rc
