#!/bin/bash
# GraNd direct3x3 (32x32): two-step register prefetch (B) and a load ablation (C, wrong
# results: the same rows every step) against the current build (A); parity tests on B
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/d3pf2}
LA=build/abA/libA.so; LB=build/abB/libB.so; LC=build/abC/libC.so
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_conv.py --kernel pegrad --batch 1024 --rounds 7 --iters 10 \
  --lib-a $LA --lib-b $LB > $OUT/ab_pf2.log 2>&1
rc=$?; echo "== A/B pf2 rc=$rc"; cat $OUT/ab_pf2.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${ABL:-}" ]; then
  timeout -k 10 300 python -u tools/ab_conv.py --kernel pegrad --batch 1024 --rounds 5 --iters 10 \
    --lib-a $LA --lib-b $LC > $OUT/ab_ablate_loads.log 2>&1
  rc=$?; echo "== A/C load ablation rc=$rc"; cat $OUT/ab_ablate_loads.log; [ $rc -eq 0 ] || exit $rc
fi
DD_LIB=$LB timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "pegrad or grand or direct" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
