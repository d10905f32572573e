#!/bin/bash
# 1x1 GraNd launches (forward epilogues fp16, backward-data bf16) under the tile-family and
# XCD-order knobs, on config 4's shapes (A/B, one box)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r06knobg}
mkdir -p "$OUT"
for epi in grandf grandb; do
  for cfg in "base" "DD_C1_FAMILY=3" "DD_C1_XCD=1" "DD_C1_FAMILY=3 DD_C1_XCD=1" "base2"; do
    if [ "${cfg:0:4}" = "base" ]; then envs=(); else envs=($cfg); fi
    tag=$(echo "$cfg" | tr ' =' '_-')
    env "${envs[@]}" timeout -k 10 300 python -u tools/c1_micro.py --batch 512 --iters 10 \
        --cifar --epi $epi > "$OUT/${epi}_$tag.log" 2>&1 || { echo "failed $epi $cfg"; tail -5 "$OUT/${epi}_$tag.log"; exit 1; }
  done
done
echo "session done"
