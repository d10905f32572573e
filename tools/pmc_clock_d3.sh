#!/bin/bash
# clock and MFMA busy of the 32x32 GraNd direct3x3 kernel: the final build (A) and the
# load ablation (C: every step re-reads the same rows), each in its own processes -- one
# PMC pass (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES) and one trace pass
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/clk}
mkdir -p $OUT
for v in A C; do
  L=build/abA/libA.so; [ $v = C ] && L=build/abC/libC.so
  DD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d $OUT/pmc_$v -o run -- python3 tools/pegrad_one.py 64 32 64 1 30 > $OUT/pmc_$v.log 2>&1
  rc=$?; echo "== pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$v -o run \
    -- python3 tools/pegrad_one.py 64 32 64 1 30 > $OUT/tr_$v.log 2>&1
  rc=$?; echo "== trace $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find $OUT -name "*.csv" | sort
