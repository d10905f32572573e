#!/bin/bash
# PMC passes over the backbone conv microbench (tools/conv_micro.py), one counter group per
# run (MI355X guide: rocprofv3 does not split counters over passes).  Results: one CSV per pass
# under $OUT/<pass>/, summarised by tools/pmc_table.py.
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_conv}
ONLY=${2:-conv}
SHAPES=${3:-}   # optional conv3x3 shapes for tools/conv_micro.py --shapes
EXTRA=(); [ -n "$SHAPES" ] && EXTRA=(--shapes "$SHAPES")
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P -T --output-format csv -d "$OUT/p$i" -o run -- \
      python3 tools/conv_micro.py --iters 5 --only "$ONLY" "${EXTRA[@]}" > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$? ($P)"
done
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt" 2>&1
cat "$OUT/table.txt"
