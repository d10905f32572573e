#!/bin/bash
# the fused unit-input 1x1 launches under the tile-family and XCD-order knobs, both networks
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r06knobu}
mkdir -p "$OUT"
for set in in c4; do
  flag=""; [ $set = c4 ] && flag="--cifar"
  for cfg in "base" "DD_C1_FAMILY=3" "DD_C1_XCD=1" "DD_C1_FAMILY=3 DD_C1_XCD=1" "DD_C1_FAMILY=1" "base2"; do
    if [ "${cfg:0:4}" = "base" ]; then envs=(); else envs=($cfg); fi
    tag=$(echo "$cfg" | tr ' =' '_-')
    env "${envs[@]}" timeout -k 10 300 python -u tools/c1_micro.py --batch 512 --iters 10 $flag \
        --epi unit > "$OUT/${set}_$tag.log" 2>&1 || { echo "failed $set $cfg"; tail -5 "$OUT/${set}_$tag.log"; exit 1; }
  done
done
echo "session done"
