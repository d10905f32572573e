#!/bin/bash
# whole-job A/B of run-time knobs on the headline config (one box, alternated)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r06kj}
mkdir -p "$OUT"
i=0
for cfg in "base" "DD_CONV_STAGGER=2000" "DD_DOWN_WA=2" "DD_CONV_TILE=narrow" "base" "DD_CONV_STAGGER=2000"; do
  i=$((i+1))
  if [ "$cfg" = "base" ]; then envs=(); else envs=($cfg); fi
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      --json-out "$OUT/run$i.json" > "$OUT/run$i.log" 2>&1 || { echo "failed $cfg"; tail -5 "$OUT/run$i.log"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/run$i.json'));print('$cfg', round(d['value'],1))" | tee -a "$OUT/summary.txt"
done
echo "session done"
