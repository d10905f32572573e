set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r05o
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_conv.py --kernel c1x1 --epi fwd --batch 1024 --rounds 5 --iters 10 \
    --operands f16x3 --lib-a build/abA/libA.so --lib-b data_diet_distributed_amd/libdd.so > $OUT/ab_c1x1_fwd.log 2>&1
rc=$?; grep -v "^$\|amdgpu.ids" $OUT/ab_c1x1_fwd.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh $OUT/c4 build/abA/libA.so data_diet_distributed_amd/libdd.so --arch resnet50 --classes 100 --n 10240
