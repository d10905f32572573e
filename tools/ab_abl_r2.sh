#!/bin/bash
# ablation A/B of the r2 conv tiles (16x16 and below): full kernel vs no staging loads /
# no weight loads / no epilogue (libraries from build/ablx, outputs differ by construction)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/r05s}
mkdir -p $OUT
for v in r2noload r2nowload r2noepi; do
  for e in stats fwd bwd; do
    timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi $e --batch 1024 --rounds 3 --iters 10 \
      --operands f16x3 --lib-a data_diet_distributed_amd/libdd.so --lib-b build/ablx/lib$v.so > $OUT/abl_${v}_$e.log 2>&1
    rc=$?; echo "== $v $e rc=$rc"; grep "16x16\|8x8\|4x4" $OUT/abl_${v}_$e.log | sed 's/max rel.*//'
    [ $rc -eq 0 ] || exit $rc
  done
done
