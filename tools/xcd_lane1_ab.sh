#!/bin/bash
# same-box A/B of DD_CONV_XCD inside the job: single-lane bench steps (the bench's own sampled
# per-launch timing of conv3x3, as its roofline), alternated three times.  gpurun_out/<tag>/
set -uo pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-xcdl1}
mkdir -p "$OUT"
for r in 1 2 3; do
  for x in 0 1; do
    DD_CONV_XCD=$x timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --lanes 1 --json-out "$OUT/b_x${x}_$r.json" > "$OUT/b_x${x}_$r.log" 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('$OUT/b_x${x}_$r.json')); r=d['roofline']
print('x=$x r=$r value', round(d['value'],1), 'conv3x3 us', round(r['avg_launch_us'],1), 'frac', round(r['frac'],4))"
  done
done
