#!/bin/bash
# whole-job sweep of the launch lanes and chunk sizes on the current tree (bench.py, alternated
# twice): lanes 2 / 3 / 4 at 1024-row chunks, lanes 3 at 2048-row chunks.  gpurun_out/<tag>/
set -uo pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-lanes}
mkdir -p "$OUT"
for r in 1 2; do
  for cfg in "3 1024" "2 1024" "4 1024" "3 2048"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --lanes $1 \
        --el2n-chunk $2 --grand-batch $2 --json-out "$OUT/bench_l$1_c$2_$r.json" \
        > "$OUT/bench_l$1_c$2_$r.log" 2>&1 || exit 1
    echo "lanes=$1 chunk=$2 r=$r $(grep -o '"value": [0-9.]*' "$OUT/bench_l$1_c$2_$r.log" | head -1)"
  done
done
