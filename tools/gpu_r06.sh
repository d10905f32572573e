#!/bin/bash
# Round-6 GPU session steps (run from the repo root on the box): new-kernel tests first, then
# their micro-benchmarks (A/B against the kernels they replace), then the whole -m gpu suite
# and smoke.  Every GPU step has its own time limit; the first failure ends the session.
#   tools/gpu_r06.sh <tag> [step ...]   steps: new micro tests smoke bench prof
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r06}
shift || true
STEPS=${*:-new micro tests smoke}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run <seconds> <log> cmd...
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  [ $rc -eq 0 ] || { echo "step failed rc=$rc ($log)"; exit $rc; }
}
for s in $STEPS; do
  case $s in
    new)
      run 600 "$OUT/pytest_new.log" python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_el2n_fast.py \
          tests/test_gpu_conv1x1.py -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "pgram_q or row_quads or auto_method or bad_labels or conv_gemm or overflow or out_of_range or unit_input" ;;
    micro)
      run 300 "$OUT/pegrad_pgq.log" python -u tools/bench_pegrad.py --batch 1024 --iters 10
      DD_PGQ=0 run 300 "$OUT/pegrad_direct.log" python -u tools/bench_pegrad.py --batch 1024 \
          --iters 10 --auto-only
      DD_C1_ROWQ=0 run 300 "$OUT/gemm_rowq0.log" python -u tools/gemm_micro.py --batch 512
      run 300 "$OUT/gemm_rowq1.log" python -u tools/gemm_micro.py --batch 512 ;;
    tests)
      DD_PARITY_OUT="$OUT/keepset_swaps.json" run 1100 "$OUT/pytest_gpu.log" \
          python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke)
      run 300 "$OUT/smoke.log" python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' ;;
    bench)
      run 900 "$OUT/bench.log" python -u bench.py --json-out "$OUT/bench.json" ;;
    dbench)
      run 900 "$OUT/bench_driver.log" python -u bench.py --gpus 1 --steps 20 --warmup 5 \
          --json-out "$OUT/bench_driver.json" ;;
    final)  # the round's closing measurement set (tools/gpu_round.sh steps)
      bash tools/gpu_round.sh "$TAG" dbench prof pmc busy || exit 1
      DD_PGQ=1 run 300 "$OUT/busy_pgq.log" bash tools/pmc_pegrad_busy.sh "$OUT/busy_pgq" ;;
    c45)
      bash tools/gpu_round.sh "$TAG" c4 c5 || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $TAG done"
