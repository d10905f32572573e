#!/bin/bash
# PMC counters of the conv microbench for two libdd builds (tools/ab_build.sh: build/ab/libA.so,
# build/ab/libB.so), one counter group per rocprofv3 run.  Tables: $OUT/{A,B}/table.txt.
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmcab}
ONLY=${2:-conv}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
for v in A B; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    D=$OUT/$v
    mkdir -p $D
    DD_LIB=$PWD/build/ab/lib$v.so timeout -s KILL 90 rocprofv3 --pmc $P -T --output-format csv \
        -d "$D/p$i" -o run -- python3 tools/conv_micro.py --iters 5 --only $ONLY > "$D/p$i.log" 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_table.py $D > $D/table.txt 2>&1
done
