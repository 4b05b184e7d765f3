# Huffman parity tests, the huff-stage variants, then the secondary bench lines
set -uo pipefail
T=${1:-r03_q}
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_dict.py tests/test_gpu_boundary.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || exit $rc
DMX_EXP_DIR=exp3 timeout -k 10 400 python3 tools/exp_variants.py run_split base,huff7,base,huff7 > gpurun_out/$T/huff.txt 2>&1; cat gpurun_out/$T/huff.txt
bash tools/gpu_benches.sh $T random dict zeros split enwik9
