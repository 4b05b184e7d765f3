#!/bin/bash
# Round 6 (on the box): K2 / K4 variants -- stage times (tools/stage_time.py, C3 100 MB, the
# bench's parse) per library, K2 phase stamps of the windowed and the LDS merge, and the
# K2 / pack parity suites with the default library.  Every GPU step has its own time limit.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_p}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base mergelds pt512 pt512t2 pt128t8; do
    [ "$v" = base ] && lib="" || lib=$R/build/var/libdmx_$v.so
    echo "== $v" >> "$OUT/stage.txt"
    DMX_LIBV=$lib timeout -k 10 120 python3 "$R/tools/stage_time.py" 100 7 lce text >> "$OUT/stage.txt" 2>&1 || exit $?
  done
done
for v in k2s k2sl; do
  echo "== $v" >> "$OUT/k2.txt"
  DMX_LIBV=$R/build/var/libdmx_$v.so timeout -k 10 120 python3 "$R/tools/k2_stamps.py" 20 >> "$OUT/k2.txt" 2>&1 || exit $?
done
for rep in 1 2 3; do
  for v in base fdnohead; do
    [ "$v" = base ] && lib="" || lib=$R/build/var/libdmx_$v.so
    DMX_LIBV=$lib timeout -k 10 100 python3 "$R/tools/fd_chunk.py" 100 16 >> "$OUT/fd.txt" 2>&1 || exit $?
  done
done
timeout -k 10 500 python3 -u -m pytest "$R/tests/test_gpu_parity.py" "$R/tests/test_gpu_split.py" "$R/tests/test_gpu_dict.py" "$R/tests/test_gpu_boundary.py" \
    -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
grep -v amdgpu "$OUT/stage.txt" "$OUT/k2.txt"; grep -h GBps "$OUT/fd.txt" | cut -c1-120
exit $rc
