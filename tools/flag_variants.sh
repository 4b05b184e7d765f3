# Diagnostic: libdmx.so built with alternative LLVM scheduler strategies, benched side by side.
#   bash tools/flag_variants.sh build     (CPU)  -> build/flagexp/libdmx_<name>.so
#   bash tools/flag_variants.sh run       (GPU)  -> one bench line per variant
R=$(cd "$(dirname "$0")/.." && pwd)
V="base: ilp:-mllvm%-amdgpu-sched-strategy=max-ilp mem:-mllvm%-amdgpu-sched-strategy=max-memory-clause iter:-mllvm%-amdgpu-sched-strategy=iterative-ilp"
if [ "$1" = build ]; then
  for v in $V; do
    n=${v%%:*}; f=$(echo "${v#*:}" | tr '%' ' ')
    make -s -C "$R/deflate_compression_amd/csrc" BUILD="$R/build/flagexp/$n" OUT="$R/build/flagexp/libdmx_$n.so" \
      HIPFLAGS="-O3 -fPIC --offload-arch=gfx950 -std=c++17 -Wall -Wno-unused-function $f" &
  done
  wait
else
  for v in $V; do
    n=${v%%:*}
    timeout -k 10 120 python -c "
import sys, runpy; sys.path.insert(0, '$R')
import deflate_compression_amd as D; D.LIB_PATH = '$R/build/flagexp/libdmx_$n.so'
sys.argv = ['bench.py', '--steps', '10', '--warmup', '3', '--cpu-budget', '0', '--tradeoff=', '--exhaustive-steps', '0']
runpy.run_path('$R/bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ratio'], d['stage_ms'])" || exit 1
  done
fi
