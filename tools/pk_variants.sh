#!/bin/bash
# Diagnostic (on the box): stage times and stream hash of the default library and of pack
# variants built by tools/build_var.sh (e.g. `bash tools/build_var.sh t4 -DTPT=4 -DPK_RING=2048`).
# usage: [ST_ARGS="MB K FLAGS"] bash tools/pk_variants.sh TAG VARIANT...   (stage_time.py arguments)
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in "" "$@"; do
  if [ -n "$v" ]; then export DMX_LIBV=build/var/libdmx_$v.so; else unset DMX_LIBV; fi
  echo "variant ${v:-default}" >> gpurun_out/$TAG/st.txt
  timeout -k 10 120 python3 tools/stage_time.py ${ST_ARGS:-100 7 lce} >> gpurun_out/$TAG/st.txt 2>&1 || exit 3
done
cat gpurun_out/$TAG/st.txt
