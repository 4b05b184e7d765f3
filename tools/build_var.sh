#!/bin/bash
# Diagnostic library variants: build/var/libdmx_NAME.so from the same sources with extra
# defines (timing knockouts, stamps).  Load one with DMX_LIBV=build/var/libdmx_NAME.so.
#   bash tools/build_var.sh NAME -DMACRO[=V] ...
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
make -s -C "$R/deflate_compression_amd/csrc" OUT="$R/build/var/libdmx_$NAME.so" BUILD="$R/build/var/$NAME" \
    DEFS="$*"
echo "built build/var/libdmx_$NAME.so"
