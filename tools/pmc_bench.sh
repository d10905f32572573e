#!/bin/bash
# HBM traffic of the dominant kernel from rocprofv3 PMC counters, one counter per pass (the
# MI355X guide: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2; never combined with tracing).
# Full kernel names (no -T): the conv3x3 staging mode (template argument XF) splits the fused
# unit-input launches into their own kind.  A short bench (1 checkpoint, 10240 examples, chunk sizes as in the full bench) under each
# pass; tools/pmc_traffic.py averages per dispatch and applies the gfx950 FETCH_SIZE x2
# correction for wide streaming reads.
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_bench}
REGEX=${2:-conv3x3_kernel|conv3x3_r2_kernel|pegrad_direct3x3|down_fwd|down_bwd|apply_kernel|pgram}
mkdir -p "$OUT"
ARGS="--n 10240 --ckpts 1 --steps 1 --warmup 0 --no-cpu-baseline --lanes 1"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$REGEX" \
      --output-format csv -d "$OUT/$C" -o run -- python3 bench.py $ARGS > "$OUT/$C.log" 2>&1
  rc=$?
  echo "pass $C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_traffic.py "$OUT" > "$OUT/pmc_traffic.json"
cat "$OUT/pmc_traffic.json"
