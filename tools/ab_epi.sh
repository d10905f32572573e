set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r05m
mkdir -p $OUT
for spec in "conv stats" "conv fwd" "conv bwd" "down stats" "down bias" "c1x1 stats"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_conv.py --kernel $1 --epi $2 --batch 1024 --rounds 5 --iters 10 \
    --operands f16x3 --lib-a build/abA/libA.so --lib-b data_diet_distributed_amd/libdd.so > $OUT/ab_$1_$2.log 2>&1
  rc=$?; echo "== $1 $2 rc=$rc"; grep -v "^$\|amdgpu.ids" $OUT/ab_$1_$2.log | tail -9
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_f16_operands.py tests/test_gpu_el2n_fast.py tests/test_gpu_down.py tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh $OUT/c2 build/abA/libA.so data_diet_distributed_amd/libdd.so
