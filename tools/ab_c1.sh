#!/bin/bash
# conv1x1 epilogue specialisation A/B (build/abA/libA.so = before, libdd.so = after)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/r05n}
mkdir -p $OUT
for spec in "stats f16x3" "fwd f16x3" "bwd bf16x3" "none bf16x3"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_conv.py --kernel c1x1 --epi $1 --batch 1024 --rounds 5 --iters 10 \
    --operands $2 --lib-a build/abA/libA.so --lib-b data_diet_distributed_amd/libdd.so > $OUT/ab_c1x1_$1_$2.log 2>&1
  rc=$?; echo "== c1x1 $1 $2 rc=$rc"; grep -v "^$\|amdgpu.ids" $OUT/ab_c1x1_$1_$2.log | tail -8
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_f16_operands.py tests/test_gpu_pipeline.py -k "conv1x1 or c1x1 or gemm or resnet50 or bottleneck or imagenet" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh $OUT/c4 build/abA/libA.so data_diet_distributed_amd/libdd.so --arch resnet50 --classes 100 --n 10240
