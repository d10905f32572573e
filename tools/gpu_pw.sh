#!/bin/bash
# padded-width conv3x3 tiles: their tests first, then the per-shape micro-benchmark against
# the implicit GEMM, then the config-5 EL2N tests; the first failure ends the session
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r06pw}
mkdir -p "$OUT"
run() {  # run <seconds> <log> cmd...
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  [ $rc -eq 0 ] || { echo "step failed rc=$rc ($log)"; exit $rc; }
}
run 300 "$OUT/pytest_pw.log" python -u -m pytest tests/test_gpu_el2n_fast.py tests/test_gpu_down.py -m gpu -x -v \
    --timeout 120 --timeout-method thread -k "padded_width or input_affine or down_forward or unsupported"
run 300 "$OUT/gemm_micro.log" python -u tools/gemm_micro.py --batch 512 --iters 10
DD_PARITY_OUT=$OUT/keepset_swaps.json run 600 "$OUT/pytest_c5.log" python -u -m pytest \
    tests/test_gpu_pipeline.py tests/test_gpu_el2n_fast.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "imagenet"
echo "session done"
