#!/bin/bash
# two-chunk-deep staging prefetch of the 32x32 conv: kernel A/B, parity tests on B, whole job
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/r05q}
LA=${2:-build/abA/libA.so}; LB=${3:-build/abB/libB.so}
mkdir -p $OUT
for e in stats fwd bwd; do
  timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi $e --batch 1024 --rounds 5 --iters 10 \
    --operands f16x3 --lib-a $LA --lib-b $LB > $OUT/ab_conv_$e.log 2>&1
  rc=$?; echo "== conv $e rc=$rc"; grep "32x32\|16x16" $OUT/ab_conv_$e.log
  [ $rc -eq 0 ] || exit $rc
done
DD_LIB=$LB timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_el2n_fast.py tests/test_gpu_f16_operands.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
DD_LIB=$LB DD_PARITY_OUT=$OUT/keepset_swaps.json timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py -k "golden or rank_invariant or lanes or short_tail or grand_at_bench or chunk_and_world" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_pipe.log 2>&1
rc=$?; tail -3 $OUT/pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh $OUT/c2 $LA $LB
