#!/bin/bash
# config 4 (ResNet-50 CIFAR-100, EL2N + GraNd): its kernels' tests, then the bench line
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06c4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
DD_PARITY_OUT=$OUT/keepset_swaps.json timeout -k 10 900 python -u -m pytest \
    tests/test_gpu_conv1x1.py tests/test_gpu_f16_operands.py tests/test_gpu_el2n_fast.py \
    tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "conv1x1 or f16 or resnet50 or grand" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/c1_micro.py --batch 512 --iters 10 --cifar --epi grandf > "$OUT/c1_grandf.log" 2>&1 || exit 1
bash tools/gpu_round.sh "$TAG" c4 || exit 1
echo "session done"
