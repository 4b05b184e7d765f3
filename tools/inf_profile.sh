#!/bin/bash
# SQ counters + kernel trace for the GPU inflate kernels (diagnostic).
# usage (on the box): bash tools/inf_profile.sh TAG [inflate_bench args]
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BA="--steps 2 --stream-mb 1 $*"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_ANY"
B="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 "$R/tools/inflate_bench.py" $BA > "$OUT/bench.json" 2> "$OUT/kt.err"
i=0
for set in "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d "$OUT/sq$i" -o sq -- python3 "$R/tools/inflate_bench.py" $BA > /dev/null 2> "$OUT/sq$i.err"
done
python3 "$R/tools/pmc.py" "$OUT/sq1,$OUT/sq2" | tee "$OUT/sq_summary.txt"
cat "$OUT/bench.json"
