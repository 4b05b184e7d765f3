#!/bin/bash
# SQ counters of the match kernel truncated after each phase (diagnostic library variants
# built with -DDMX_DEBUG_STOP=1|2|3, never the product library): the per-phase VALU / SALU /
# LDS instruction counts by difference.
# build first (here):  for s in 1 2 3; do bash tools/build_var.sh stop$s -DDMX_DEBUG_STOP=$s; done
# usage (on the box): bash tools/phase_profile.sh TAG [MB K lazy]
set -euo pipefail
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
for st in 1 2 3 0; do
  if [ "$st" = 0 ]; then unset DMX_LIBV; else export DMX_LIBV=$R/build/var/libdmx_stop$st.so; fi
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/ph$st" -o ph -- python3 "$R/tools/phase_run.py" "$@" > "$OUT/ph$st.log" 2>&1
  echo "== stop $st" >> "$OUT/phase_summary.txt"
  python3 "$R/tools/pmc.py" "$OUT/ph$st" | grep match_kernel >> "$OUT/phase_summary.txt"
done
cat "$OUT/phase_summary.txt"
