#!/bin/bash
# the 4-element BN apply: its tests, the config-5 network tests, then the config-5 bench line
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06bq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
DD_PARITY_OUT=$OUT/keepset_swaps.json timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_el2n_fast.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "bn_apply or stem7 or imagenet or resnet50" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/gpu_round.sh "$TAG" c5 || exit 1
echo "session done"
