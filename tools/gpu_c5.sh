#!/bin/bash
# config-5 kernels: 1x1 / padded-width tests, the per-shape micro-benchmarks, then the config-5
# bench line; the first failure ends the session
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06c5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run <seconds> <log> cmd...
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  [ $rc -eq 0 ] || { echo "step failed rc=$rc ($log)"; exit $rc; }
}
DD_PARITY_OUT=$OUT/keepset_swaps.json run 600 "$OUT/pytest.log" python -u -m pytest \
    tests/test_gpu_conv1x1.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "conv1x1 or imagenet"
run 300 "$OUT/c1_micro.log" python -u tools/c1_micro.py --batch 512 --iters 10
run 300 "$OUT/gemm_micro.log" python -u tools/gemm_micro.py --batch 512 --iters 10
bash tools/gpu_round.sh "$TAG" c5 || exit 1
echo "session done"
