#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03prio2; mkdir -p $O
tools/ab_env.sh $O 2 conv DD_CONV_PRIO 0 1 2 || exit 1
