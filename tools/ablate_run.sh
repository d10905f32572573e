#!/bin/bash
# time each ablated conv variant (tools/ablate_conv.py) against the full kernel, per tile family
set -uo pipefail
OUT=gpurun_out/abl
mkdir -p $OUT
for fam in narrow wide; do
  for v in noload nostage nowload noepi; do
    DD_CONV_TILE=$fam timeout -k 10 120 python -u tools/ab_conv.py --epi fwd --rounds 3 --iters 10 \
        --lib-a build/abl/libfull.so --lib-b build/abl/lib$v.so > $OUT/${fam}_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/${fam}_$v.log; exit $rc; }
    echo "== $fam $v"; grep conv3x3 $OUT/${fam}_$v.log | sed 's/max rel.*//'
  done
done
