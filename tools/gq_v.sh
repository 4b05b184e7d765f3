# dict validation + inflate variant timings (ring sizes; chained-decode link hops)
set -uo pipefail
T=${1:-r03_d3}
bash tools/gq_d.sh $T || exit $?
bash tools/inflate_variants.sh run iwx4k iwx8k iwx16k > gpurun_out/$T/iwx.txt 2>&1; cat gpurun_out/$T/iwx.txt
IB_ARGS="--chained 1" bash tools/inflate_variants.sh run hop1 hop2 hop2i2 > gpurun_out/$T/hops.txt 2>&1; cat gpurun_out/$T/hops.txt
