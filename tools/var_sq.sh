#!/bin/bash
# SQ counters and phase stamps of the match kernel for library variants (diagnostic, on the box):
#   bash tools/var_sq.sh TAG "v1 v2 ..."   ("" = libdmx.so; build/var/libdmx_NAME.so otherwise)
# C3 text, 20 MB, K = 7 lazy (tools/phase_run.py); stamps at K = 7 and K = 0 (tools/stamps.py)
set -uo pipefail
TAG=$1; VARS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for v in $VARS; do
  [ "$v" = base ] && lib="" || lib=$R/build/var/libdmx_$v.so
  ( cd /tmp && DMX_LIBV=$lib timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_$v" -o sq \
      -- python3 "$R/tools/phase_run.py" 20 7 1 > "$OUT/sq_$v.log" 2>&1 ) || exit $?
  echo "== $v" >> "$OUT/var_sq.txt"
  python3 "$R/tools/pmc.py" "$OUT/sq_$v" | grep -E "match_(pf_)?kernel" >> "$OUT/var_sq.txt"
  DMX_LIBV=$lib timeout -k 10 120 python3 "$R/tools/stamps.py" text:7 text:0:g >> "$OUT/var_sq.txt" 2>&1 || exit $?
done
cat "$OUT/var_sq.txt"
