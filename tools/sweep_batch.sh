#!/bin/bash
# Bench sweep over the GraNd batch and EL2N chunk sizes (results under gpurun_out/sweep/).
set -uo pipefail
OUT=gpurun_out/sweep
mkdir -p "$OUT"
for gb in 1024 2048; do
  for ec in 1024 2048; do
    timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --grand-batch $gb --el2n-chunk $ec --json-out "$OUT/gb${gb}_ec${ec}.json" \
        > "$OUT/gb${gb}_ec${ec}.log" 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('$OUT/gb${gb}_ec${ec}.json'));print($gb,$ec,round(d['value'],1))"
  done
done
