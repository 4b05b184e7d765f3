set -uo pipefail
T=${1:-r03_q}
mkdir -p gpurun_out/$T
DMX_EXP_DIR=exp3 timeout -k 10 400 python3 tools/exp_variants.py run_split base,huff7,base,huff7 > gpurun_out/$T/huff.txt 2>&1; cat gpurun_out/$T/huff.txt
