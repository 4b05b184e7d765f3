set -uo pipefail
T=${1:-r03_h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dict.py tests/test_gpu_inflate.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || exit $rc
IB_ARGS="--chained 1" bash tools/inflate_variants.sh run h2 h3 h4 h3i4 > gpurun_out/$T/hops.txt 2>&1; cat gpurun_out/$T/hops.txt
