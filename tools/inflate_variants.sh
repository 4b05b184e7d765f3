#!/bin/bash
# Build libdmx variants with other inflate compile-time settings (CPU side):
#   bash tools/inflate_variants.sh build NAME "-DDMX_IWX=16384" ...
# and time them on the GPU box: bash tools/inflate_variants.sh run NAME...
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/build/exp3
if [ "$1" = build ]; then
    shift
    while [ $# -ge 2 ]; do
        mkdir -p "$O"
        /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -std=c++17 $2 -I "$R/deflate_compression_amd/csrc" -I "$R/include" \
            -c -o "$O/inf_$1.o" "$R/deflate_compression_amd/csrc/dmx_inflate_dev.hip"
        /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$O/libdmx_$1.so" "$O/inf_$1.o" \
            "$R/build/dmx/dmx_kernels.o" "$R/build/dmx/dmx_host.o" "$R/build/dmx/dmx_inflate.o" "$R/build/dmx/dmx_gen.o" \
            "$R/build/dmx/dmx_refstats.o" -lm -lpthread
        rm -f "$O/inf_$1.o"
        echo "built $1"
        shift 2
    done
else
    shift
    for v in "$@"; do
        echo -n "$v "
        DMX_LIB=$O/libdmx_$v.so timeout -k 10 200 python3 "$R/tools/inflate_bench.py" --steps 10 ${IB_ARGS:-}
    done
fi
