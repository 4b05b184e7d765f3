set -uo pipefail
mkdir -p gpurun_out/r03_p1
EXP_K=6 EXP_LAZY=1 DMX_EXP_DIR=exp3 timeout -k 10 300 python3 tools/exp_variants.py run ${1:-base} > gpurun_out/r03_p1/p1.txt 2>&1; cat gpurun_out/r03_p1/p1.txt
