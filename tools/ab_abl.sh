#!/bin/bash
# ablation A/B of the narrow 32x32 conv: the full kernel vs no staging loads / no staging
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/r05p}
mkdir -p $OUT
for v in noload nostage; do
  for e in stats fwd bwd; do
    timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi $e --batch 1024 --rounds 3 --iters 10 \
      --operands f16x3 --lib-a data_diet_distributed_amd/libdd.so --lib-b build/ablx/lib$v.so > $OUT/abl_${v}_$e.log 2>&1
    rc=$?; echo "== $v $e rc=$rc"; grep "32x32" $OUT/abl_${v}_$e.log | sed 's/max rel.*//'
    [ $rc -eq 0 ] || exit $rc
  done
done
