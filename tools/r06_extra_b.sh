#!/bin/bash
# round-6 session extras (on the box): variant correctness, claim guard, hint switch, scan probes
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06_b}
export TMPDIR=/tmp
PY="python3 -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread"
DMX_LIBV=$R/build/var/libdmx_all.so timeout -k 10 500 $PY tests/test_gpu_parity.py tests/test_gpu_exhaustive.py \
    tests/test_gpu_deep.py tests/test_gpu_dict.py tests/test_gpu_split.py tests/test_gpu_shards.py > "$OUT/all.log" 2>&1
rc=$?; tail -2 "$OUT/all.log"; [ $rc -le 1 ] || exit $rc
DMX_LIBV=$R/build/var/libdmx_claim.so timeout -k 10 400 $PY tests/test_gpu_exhaustive.py tests/test_gpu_worklist.py \
    --deselect tests/test_gpu_worklist.py::test_scan_many_tiles > "$OUT/claim.log" 2>&1
rc=$?; tail -2 "$OUT/claim.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/hint_switch.py > "$OUT/hint.json" 2>&1 || exit $?
cat "$OUT/hint.json"
timeout -k 10 100 python3 tools/scan_probe.py 4096 257 > "$OUT/probe1.txt" 2>&1
rc=$?; cat "$OUT/probe1.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python3 tools/scan_probe.py 1024 1025 > "$OUT/probe2.txt" 2>&1
rc=$?; cat "$OUT/probe2.txt"; exit $rc
