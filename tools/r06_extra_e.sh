#!/bin/bash
# round-6 session e extras: P3 batch correctness, counters + stamps
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_e
export TMPDIR=/tmp
PY="python3 -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread"
DMX_LIBV=$R/build/var/libdmx_wr.so timeout -k 10 500 $PY tests/test_gpu_parity.py tests/test_gpu_exhaustive.py \
    tests/test_gpu_deep.py tests/test_gpu_dict.py tests/test_gpu_split.py > "$OUT/wr.log" 2>&1
rc=$?; tail -2 "$OUT/wr.log"; [ $rc -le 1 ] || exit $rc
bash tools/var_sq.sh r06_e "p3s p3b wr nbx5" || exit $?
