#!/bin/bash
# A/B of the XCD-contiguous order for the persistent down_fwd grid (DD_DOWN_XCD=2 vs the
# default 1): the three head shapes (tools/conv_micro.py --only down, alternated twice) and the
# bench's PMC traffic per kernel kind (tools/pmc_bench.sh).  Output under gpurun_out/<tag>/.
set -uo pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${1:-downxcd}
mkdir -p "$OUT"
for r in 1 2; do
  for x in 1 2; do
    DD_DOWN_XCD=$x timeout -k 10 200 python -u tools/conv_micro.py --only down --batch 1024 \
        --iters 20 > "$OUT/micro_x${x}_$r.log" 2>&1 || exit 1
  done
done
for x in 1 2; do
  DD_DOWN_XCD=$x timeout -k 10 400 bash tools/pmc_bench.sh "$OUT/pmc_x$x" > "$OUT/pmc_x$x.log" 2>&1 || exit 1
done
grep -h down_fwd "$OUT"/micro_x*.log
for x in 1 2; do python3 -c "
import json,sys; d=json.load(open('$OUT/pmc_x$x/pmc_traffic.json'))
print('x=$x', {k: round(v['hbm_bytes_per_launch']/1e6,1) for k,v in d.items()})"; done
