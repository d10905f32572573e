#!/bin/bash
# HBM roofline evidence for the byte-bound kernels (dd_el2n, dd_normalize_u8, dd_select_topk):
# the size sweep of tools/bench_hbm_kernels.py under rocprofv3 --kernel-trace --stats, then
# per-configuration trace times (tools/hbm_trace_table.py).  Run from the repo root on the box.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/hbm}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o hbm \
    -- python3 tools/bench_hbm_kernels.py "$OUT/sweep_events.json" > "$OUT/sweep.log" 2>&1
TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
STATS=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 tools/hbm_trace_table.py "$TRACE" "$OUT/sweep_events.json" "$OUT/hbm_roofline.json" \
    > "$OUT/hbm_roofline.txt"
cp "$STATS" "$OUT/kernel_stats.csv"
rm -f "$TRACE"
cat "$OUT/hbm_roofline.txt"
