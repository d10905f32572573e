#!/bin/bash
# ResNet-50 1x1 launch rules: their tests, the per-shape micro-benchmarks of both networks,
# then the config-5 and config-4 bench lines; the first failure ends the session
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06c45}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -2 "$log"
  [ $rc -eq 0 ] || { echo "step failed rc=$rc ($log)"; exit $rc; }
}
DD_PARITY_OUT=$OUT/keepset_swaps.json run 900 "$OUT/pytest.log" python -u -m pytest \
    tests/test_gpu_conv1x1.py tests/test_gpu_f16_operands.py tests/test_gpu_el2n_fast.py \
    tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "conv1x1 or f16 or imagenet or resnet50 or el2n_fast or conv3x3 or bn_apply or channel"
run 300 "$OUT/c1_in.log" python -u tools/c1_micro.py --batch 512 --iters 10
run 300 "$OUT/c1_c4.log" python -u tools/c1_micro.py --batch 512 --iters 10 --cifar
bash tools/gpu_round.sh "$TAG" c5 c4 || exit 1
echo "session done"
