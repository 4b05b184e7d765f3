#!/bin/bash
# round-6 session hi: the split extension queue (qf) and the exhaustive survivor queue (sq):
# correctness, counters + stamps
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_j
export TMPDIR=/tmp
PY="python3 -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread"
DMX_LIBV=$R/build/var/libdmx_ring.so timeout -k 10 500 $PY tests/test_gpu_parity.py tests/test_gpu_exhaustive.py \
    tests/test_gpu_deep.py tests/test_gpu_dict.py tests/test_gpu_split.py tests/test_gpu_worklist.py > "$OUT/ring.log" 2>&1
rc=$?; tail -2 "$OUT/ring.log"; [ $rc -le 1 ] || exit $rc
bash tools/var_sq.sh r06_j "base ring" || exit $?
