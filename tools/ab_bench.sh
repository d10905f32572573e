#!/bin/bash
# Whole-job A/B of two libdd.so builds: bench.py lines alternated A, B, A, B on one box
#   tools/ab_bench.sh <out dir> <lib A> <lib B> [extra bench.py args...]
# (ENV_A / ENV_B: extra VAR=value settings for one arm, e.g. an A/B of one library's knob)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$1; LA=$2; LB=$3; shift 3
mkdir -p "$OUT"
for r in 1 2; do
  for v in A B; do
    L=$LA; E=${ENV_A:-}; [ $v = B ] && { L=$LB; E=${ENV_B:-}; }
    env $E DD_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" \
        --json-out "$OUT/bench_${v}_$r.json" > "$OUT/bench_${v}_$r.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${v}_$r.log"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, round(d['value'],1), round(d['roofline']['frac'],4))"
  done
done
