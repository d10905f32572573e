#!/bin/bash
# config 4's GraNd backward-data 1x1 GEMMs under the tile-family and XCD-order knobs
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r06knobb}
mkdir -p "$OUT"
for cfg in "base" "DD_C1_FAMILY=3" "DD_C1_XCD=1" "DD_C1_FAMILY=3 DD_C1_XCD=1" "DD_C1_FAMILY=1" "base2"; do
  if [ "${cfg:0:4}" = "base" ]; then envs=(); else envs=($cfg); fi
  tag=$(echo "$cfg" | tr ' =' '_-')
  env "${envs[@]}" timeout -k 10 300 python -u tools/c1_micro.py --batch 512 --iters 10 \
      --epi bwd > "$OUT/bwd_$tag.log" 2>&1 || { echo "failed $cfg"; tail -5 "$OUT/bwd_$tag.log"; exit 1; }
done
echo "session done"
