set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r05j
mkdir -p $OUT
for spec in "c1x1 none" "c1x1 stats" "c1x1 fwd" "c1x1 bwd" "conv stats" "conv fwd" "conv bwd" "down stats" "down bias"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_conv.py --kernel $1 --epi $2 --batch 1024 --rounds 5 --iters 10 \
    --operands f16x3 --lib-a data_diet_distributed_amd/libdd.so --lib-b build/nt/libB.so > $OUT/ab_nt_$1_$2.log 2>&1
  rc=$?; echo "== $1 $2 rc=$rc"; cat $OUT/ab_nt_$1_$2.log | grep -v "^$" | tail -9
  [ $rc -eq 0 ] || exit $rc
done
