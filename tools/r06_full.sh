#!/bin/bash
# round-6 evidence pass (on the box): profile_round (GPU suite, trace, PMC, SQ, bench with
# traffic), then the secondary lines (C4, dict, zeros, split, C5) and the small-alphabet depths
set -uo pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/profile_round.sh" "$TAG" || exit $?
bash "$R/tools/gpu_benches.sh" "${TAG}_sec" random dict zeros split enwik9 || exit $?
timeout -k 10 300 python3 "$R/tools/deep_bench.py" 32 > "$R/gpurun_out/${TAG}_sec/deep.txt" 2>&1 || exit $?
grep -v amdgpu "$R/gpurun_out/${TAG}_sec/deep.txt"
