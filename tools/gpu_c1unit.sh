#!/bin/bash
# the 1x1 residual-unit input: parity tests, then a config-4 / config-5 whole-job A/B
# (DD_FUSE_UNIT_INPUT=0 in arm A: every unit tail a dd_bn_apply pass)
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/r05t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_el2n_fast.py tests/test_gpu_conv1x1.py tests/test_capi_symbols.py tests/test_gpu_pipeline.py -k "unit_input or conv1x1 or resnet50 or imagenet or bottleneck or capi" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ENV_A=DD_FUSE_UNIT_INPUT=0 bash tools/ab_bench.sh $OUT/c4 data_diet_distributed_amd/libdd.so data_diet_distributed_amd/libdd.so --arch resnet50 --classes 100 --n 10240 || exit 1
ENV_A=DD_FUSE_UNIT_INPUT=0 bash tools/ab_bench.sh $OUT/c5 data_diet_distributed_amd/libdd.so data_diet_distributed_amd/libdd.so --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 65536
