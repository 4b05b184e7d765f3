#!/bin/bash
# Round 6 (on the box): K2 variants -- phase stamps (tools/k2_stamps.py) of the stamp builds,
# stage times (tools/stage_time.py, C3 100 MB, the bench's parse) of base vs the variants in
# $VARS, then the parity suites that exercise K2 (plain, split, dict).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_q}
STAMPS=${STAMPS-k2s k2old}
VARS=${VARS-lenloop}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $STAMPS; do
  echo "== $v" >> "$OUT/k2.txt"
  DMX_LIBV=$R/build/var/libdmx_$v.so timeout -k 10 120 python3 "$R/tools/k2_stamps.py" 20 >> "$OUT/k2.txt" 2>&1 || exit $?
done
for rep in 1 2; do
  for v in base $VARS; do
    [ "$v" = base ] && lib="" || lib=$R/build/var/libdmx_$v.so
    echo "== $v" >> "$OUT/stage.txt"
    DMX_LIBV=$lib timeout -k 10 120 python3 "$R/tools/stage_time.py" 100 7 lce text >> "$OUT/stage.txt" 2>&1 || exit $?
  done
done
timeout -k 10 500 python3 -u -m pytest "$R/tests/test_gpu_parity.py" "$R/tests/test_gpu_split.py" "$R/tests/test_gpu_dict.py" \
    -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
grep -hv amdgpu "$OUT/k2.txt"; grep -h "==\|stage_ms" "$OUT/stage.txt" | sed 's/.config.*stage_ms/stage_ms/' 
exit $rc
