#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03clamp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_el2n_fast.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_DIR=build/abx tools/ab_round.sh r03clamp/ab conv "none fwd" || exit 1
timeout -k 10 600 bash tools/pmc_bench.sh $O/pmc "conv3x3_kernel|conv3x3_r2_kernel" > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
head -8 $O/pmc/pmc_traffic.json
for r in 1 2; do
  for v in A B; do
    DD_LIB=build/abx/lib$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/bench_${v}_r$r.json > $O/bench_${v}_r$r.log 2>&1 || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_${v}_r$r.json'));print('$v r$r', round(d['value'],1), round(d['roofline']['frac'],4))"
  done
done
