#!/bin/bash
# One GPU-box session: GPU parity tests, the default bench line, and a rocprofv3 kernel-stats
# profile of a short bench (run from the repo root on the box; results under gpurun_out/).
#   tools/gpu_round.sh <tag> [tests|bench|prof ...]   (default: all three)
set -uo pipefail
export TMPDIR=/tmp
TAG=${1:-run}
shift || true
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
          --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' \
          > "$OUT/smoke.log" 2>&1
      rc=$?; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 900 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
      rc=$?; tail -2 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof" \
          -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
          --json-out "$OUT/bench_under_rocprof.json" > "$OUT/prof.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit $rc; }
      TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
      if [ -n "$TRACE" ]; then
        python3 tools/trace_summary.py "$TRACE" 1 > "$OUT/trace_summary.txt"  # 1 warmup step
        rm -f "$TRACE"
        head -25 "$OUT/trace_summary.txt"
      fi ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
