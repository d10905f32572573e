#!/bin/bash
# the ImageNet stem kernel: its tests, the config-5 network tests, a timing against the implicit
# GEMM, then the config-5 bench line
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06s7}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
DD_PARITY_OUT=$OUT/keepset_swaps.json timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_el2n_fast.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "stem7 or imagenet" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/stem7_micro.py > "$OUT/stem7_micro.log" 2>&1 || { tail -20 "$OUT/stem7_micro.log"; exit 1; }
cat "$OUT/stem7_micro.log" | grep -v amdgpu
bash tools/gpu_round.sh "$TAG" c5 || exit 1
echo "session done"
