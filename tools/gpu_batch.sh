#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03dpp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_down.py tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_DIR=build/abx tools/ab_round.sh r03dpp/abd down "none" || exit 1
AB_DIR=build/abx tools/ab_round.sh r03dpp/abb bwd "none" || exit 1
AB_DIR=build/abx tools/ab_round.sh r03dpp/abp pegrad "none" || exit 1
for r in 1 2; do
  for v in A B; do
    DD_LIB=build/abx/lib$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/bench_${v}_r$r.json > $O/bench_${v}_r$r.log 2>&1 || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_${v}_r$r.json'));r=d['rooflines_other'];print('$v r$r', round(d['value'],1), round(d['roofline']['frac'],4), {k: round(r[k]['avg_launch_us'],1) for k in ('down_fwd','down_bwd','pgram','direct3x3')})"
  done
done
