#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command (run on the GPU box from the repo root)
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
mkdir -p "$OUT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 bench.py "$@"
