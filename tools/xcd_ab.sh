#!/bin/bash
# A/B of the XCD-contiguous persistent tile order of the conv3x3 kernels (DD_CONV_XCD): per-shape
# time (tools/conv_micro.py, alternated twice), per-shape PMC traffic (tools/pmc_conv_traffic.sh)
# and the whole job (bench.py, alternated twice).  Output under gpurun_out/<tag>/.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-xcd}
mkdir -p "$OUT"
for r in 1 2; do
  for x in 0 1; do
    DD_CONV_XCD=$x timeout -k 10 200 python -u tools/conv_micro.py --only conv --batch 1024 \
        --iters 20 > "$OUT/micro_x${x}_$r.log" 2>&1 || exit 1
  done
done
for x in 0 1; do
  DD_CONV_XCD=$x timeout -k 10 400 bash tools/pmc_conv_traffic.sh "$OUT/pmc_x$x" > "$OUT/pmc_x$x.log" 2>&1 || exit 1
done
for r in 1 2; do
  for x in 0 1; do
    DD_CONV_XCD=$x timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --json-out "$OUT/bench_x${x}_$r.json" > "$OUT/bench_x${x}_$r.log" 2>&1 || exit 1
  done
done
grep -h "conv3x3" "$OUT"/micro_x*.log
cat "$OUT/pmc_x0/table.txt" "$OUT/pmc_x1/table.txt"
for f in "$OUT"/bench_x*.log; do echo "$f $(grep -o '"value": [0-9.]*' "$f" | head -1)"; done
