#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration (config 4/5 baselines).
#   tools/prof_cfg.sh <tag> <bench args...>
set -uo pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --no-cpu-baseline --json-out "$OUT/bench.json" "$@" > "$OUT/prof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 "$OUT/prof.log"; exit $rc; }
TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_summary.py "$TRACE" "${WARMUP:-1}" > "$OUT/trace_summary.txt"
rm -f "$TRACE"
head -32 "$OUT/trace_summary.txt" | cut -c1-150
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['config']['workload'], d['value'], d['ms_per_step'])"
