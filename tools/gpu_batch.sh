#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03prio; mkdir -p $O
DD_HBM_ONLY=select timeout -k 10 300 tools/hbm_roofline.sh $O/hbm_select > $O/hbm.log 2>&1 || { tail -20 $O/hbm.log; exit 1; }
grep -A1 "16777216, k=8388608  " $O/hbm_select/hbm_roofline.txt
tools/ab_env.sh $O 2 conv DD_CONV_PRIO 0 1 2 || exit 1
for r in 1 2; do
  for v in 0 1 2; do
    DD_CONV_PRIO=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/bench_p${v}_r$r.json > $O/bench_p${v}_r$r.log 2>&1 || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_p${v}_r$r.json'));print('PRIO=$v r$r', round(d['value'],1), round(d['roofline']['frac'],4), [(t['kind'], round(t['rate'],1)) for t in d['top_launch_shapes'][:4]])"
  done
done
