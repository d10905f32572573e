#!/bin/bash
# Interleaved A/B of one environment knob on tools/conv_micro.py (same build, one process per
# run, rounds alternate so box drift cancels):
#   tools/ab_env.sh <out> <rounds> <only> <VAR> <value> [<value> ...]
# e.g. tools/ab_env.sh gpurun_out/stag 2 conv DD_CONV_STAGGER 0 4000 8000
set -uo pipefail
OUT=$1; ROUNDS=$2; ONLY=$3; VAR=$4; shift 4
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 200 python -u tools/conv_micro.py --only "$ONLY" --batch 1024 \
        --iters 10 > "$OUT/${VAR}_${v}_r$r.txt" 2>&1 || exit 1
  done
done
for v in "$@"; do echo "== $VAR=$v"; cat "$OUT"/${VAR}_${v}_r*.txt | grep -v Warning; done
