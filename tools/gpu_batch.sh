#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03selab2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_select.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in h0 h1 h2; do
  DD_LIB=build/selab/lib$v.so DD_HBM_ONLY=select timeout -k 10 300 tools/hbm_roofline.sh $O/hbm$v > $O/hbm$v.log 2>&1 || { tail -20 $O/hbm$v.log; exit 1; }
  echo "== $v"; grep -A1 "16777216, k=8388608  " $O/hbm$v/hbm_roofline.txt
done
