#!/bin/bash
# round-6 session c extras: counters + stamps of variants, qg correctness, hint switch
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_c
export TMPDIR=/tmp
PY="python3 -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread"
DMX_LIBV=$R/build/var/libdmx_qg.so timeout -k 10 500 $PY tests/test_gpu_parity.py tests/test_gpu_exhaustive.py \
    tests/test_gpu_deep.py tests/test_gpu_dict.py tests/test_gpu_split.py tests/test_gpu_shards.py > "$OUT/qg.log" 2>&1
rc=$?; tail -2 "$OUT/qg.log"; [ $rc -le 1 ] || exit $rc
bash tools/var_sq.sh r06_c "base quads qg" || exit $?
timeout -k 10 300 python3 tools/hint_switch.py > "$OUT/hint.json" 2>&1 || exit $?
cat "$OUT/hint.json"
