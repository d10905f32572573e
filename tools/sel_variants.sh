#!/bin/bash
# Build select-kernel variants (macro settings) as whole libraries for in-process A/B runs:
#   tools/sel_variants.sh NAME "MACROS" [NAME "MACROS" ...]  ->  build/selab/lib<NAME>.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/selab; mkdir -p "$OUT"
others=$(ls "$ROOT"/build/obj/*.o | grep -v dd_select.o)
while [ $# -ge 2 ]; do
  name=$1; macros=$2; shift 2
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wall $macros -c \
    -o "$OUT/sel_$name.o" "$ROOT/data_diet_distributed_amd/csrc/dd_select.hip"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/lib$name.so" $others "$OUT/sel_$name.o" &
done
wait
ls -la "$OUT"/*.so
