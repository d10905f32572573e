#!/bin/bash
# whole-job A/B of DD_CONV_XCD (bench.py defaults, alternated three times) under gpurun_out/<tag>/
set -uo pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-xcdjob}
mkdir -p "$OUT"
for r in 1 2 3; do
  for x in 1 0; do
    DD_CONV_XCD=$x timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
        --json-out "$OUT/bench_x${x}_$r.json" > "$OUT/bench_x${x}_$r.log" 2>&1 || exit 1
    echo "x=$x r=$r $(grep -o '"value": [0-9.]*' "$OUT/bench_x${x}_$r.log" | head -1)"
  done
done
