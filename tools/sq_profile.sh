#!/bin/bash
# SQ counter passes for the kernels of one bench configuration (diagnostic).
# usage (on the box): bash tools/sq_profile.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BA="--steps 1 --warmup 0 --cpu-budget 0 --exhaustive-steps 0 --tradeoff= --bytes 20000000 $*"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
B="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
i=0
for set in "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/sq$i" -o sq -- python3 "$R/bench.py" $BA > /dev/null 2> "$OUT/sq$i.err"
done
python3 "$R/tools/pmc.py" "$OUT/sq1,$OUT/sq2" | tee "$OUT/sq_summary.txt"
