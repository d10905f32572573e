#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03selab; mkdir -p $O
for r in 1 2; do
for v in r16b512p1 r8b1024p1 r16b512p0 r8b1024p0; do
  DD_LIB=build/selab/lib$v.so DD_HBM_ONLY=select timeout -k 10 120 python -u tools/bench_hbm_kernels.py $O/$v.$r.json > $O/$v.$r.log 2>&1 || { tail -5 $O/$v.$r.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.$r.json'));print('$v r$r', [(x['n'], x.get('dist',''), round(x['us'],1)) for x in d])"
done
done
