#!/bin/bash
# PMC passes (one counter group per run, as the MI355X guide prescribes) over the GraNd
# per-layer norm kernels of a small bench config; parsed by tools/pmc_parse.py.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
ARGS="--n 2560 --ckpts 1 --steps 1 --warmup 0 --no-cpu-baseline"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'pegrad|el2n_rows' -T \
      --output-format csv -d "$OUT/$C" -o run -- python3 bench.py $ARGS > "$OUT/$C.log" 2>&1
done
python3 tools/pmc_parse.py "$OUT" > "$OUT/pmc_summary.json"
cat "$OUT/pmc_summary.json"
