#!/bin/bash
# Build two variants of libdd.so for an in-process A/B (tools/ab_conv.py):
#   A = the sources at git revision $1 (default HEAD), B = the working tree.
set -euo pipefail
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/${AB_DIR:-build/abx}
rm -rf "$OUT/A"
mkdir -p "$OUT/A/data_diet_distributed_amd/csrc" "$OUT/A/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" data_diet_distributed_amd/csrc/) \
         include/dd_capi.h; do
  git -C "$ROOT" show "$REV:$f" > "$OUT/A/$f"
done
FLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Wall"
/opt/rocm/bin/hipcc $FLAGS -o "$OUT/libA.so" "$OUT"/A/data_diet_distributed_amd/csrc/*.hip &
/opt/rocm/bin/hipcc $FLAGS -o "$OUT/libB.so" "$ROOT"/data_diet_distributed_amd/csrc/*.hip &
wait
ls -la "$OUT"/*.so
