#!/bin/bash
# rocprofv3 kernel trace + stats of a bench command (run on the GPU box from the repo root).
# Keeps the per-kernel stats; the per-dispatch trace is summarised and deleted (it is
# hundreds of MB for a full job).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
mkdir -p "$OUT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT" -o run -- \
    python3 bench.py "$@"
TRACE=$(find "$OUT" -name '*kernel_trace.csv' | head -1)
if [ -n "$TRACE" ]; then
  python3 tools/trace_summary.py "$TRACE" "${WARMUP:-1}" > "$OUT/trace_summary.txt"
  rm -f "$TRACE"
fi
