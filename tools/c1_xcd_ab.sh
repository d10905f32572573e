#!/bin/bash
# A/B of the XCD-contiguous tile order of conv1x1_kernel (DD_C1_XCD): the ResNet-50 1x1 shapes
# (tools/conv_micro.py --only c1x1, alternated twice) and config 4 at N = 10 240 (alternated
# twice).  Output under gpurun_out/<tag>/.
set -uo pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-c1xcd}
mkdir -p "$OUT"
for r in 1 2; do
  for x in 0 1; do
    DD_C1_XCD=$x timeout -k 10 200 python -u tools/conv_micro.py --only c1x1 --batch 1024 \
        --iters 10 > "$OUT/micro_x${x}_$r.log" 2>&1 || exit 1
  done
done
for r in 1 2; do
  for x in 0 1; do
    DD_C1_XCD=$x timeout -k 10 400 python -u bench.py --arch resnet50 --classes 100 --n 10240 \
        --steps 2 --warmup 1 --no-cpu-baseline --json-out "$OUT/c4_x${x}_$r.json" \
        > "$OUT/c4_x${x}_$r.log" 2>&1 || exit 1
    echo "x=$x r=$r $(grep -o '"value": [0-9.]*' "$OUT/c4_x${x}_$r.log" | head -1)"
  done
done
paste <(grep -h conv1x1 "$OUT/micro_x0_1.log" | cut -c1-45) <(grep -h conv1x1 "$OUT/micro_x0_2.log" | awk '{print $5}') <(grep -h conv1x1 "$OUT/micro_x1_1.log" | awk '{print $5}') <(grep -h conv1x1 "$OUT/micro_x1_2.log" | awk '{print $5}')
