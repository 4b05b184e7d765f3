#!/bin/bash
# One GPU-box session of round 6 (on the box): the -m gpu suite, then A/B timing of library
# variants (tools/pipe_time.py, C3 100 MB), variant test runs, diagnostics.  Every GPU step
# has its own time limit; a timeout / crash / fault status ends the script there.
# usage: bash tools/r06_session.sh TAG "VARIANTS" [PYTEST_DESELECT...]
set -uo pipefail
TAG=$1
VARS=${2:-}
shift 2 2>/dev/null || shift $#
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export DMX_TEST_HEARTBEAT=$OUT/heartbeat.txt
stop() { echo "step status $1: stopping"; exit "$1"; }
DES=()
for d in "$@"; do DES+=(--deselect "$d"); done
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest "$R/tests" -m gpu -x -v -p no:cacheprovider --timeout 240 \
      --timeout-method thread "${DES[@]}" > "$OUT/pytest.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest.log"
  [ $rc -le 1 ] || stop $rc
fi
for rep in 1 2; do
  for v in "" $VARS; do
    ( if [ -n "$v" ]; then export DMX_LIBV=$R/build/var/libdmx_$v.so; fi
      timeout -k 10 120 python3 "$R/tools/pipe_time.py" 100 7 lce text 20 ) >> "$OUT/pipe.txt" 2>&1 || stop $?
    ( if [ -n "$v" ]; then export DMX_LIBV=$R/build/var/libdmx_$v.so; fi
      timeout -k 10 120 python3 "$R/tools/pipe_time.py" 100 0 "" text 4 ) >> "$OUT/pipe.txt" 2>&1 || stop $?
  done
done
grep -h "GBps" "$OUT/pipe.txt"
if [ -n "${EXTRA:-}" ]; then bash -c "$EXTRA" || stop $?; fi
exit 0
