set -uo pipefail
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
for fam in wide narrow; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    OUT=gpurun_out/pmcw/$fam
    mkdir -p $OUT
    DD_CONV_TILE=$fam timeout -s KILL 90 rocprofv3 --pmc $P -T --output-format csv -d "$OUT/p$i" -o run -- python3 tools/conv_micro.py --iters 5 --only conv > "$OUT/p$i.log" 2>&1
    rc=$?; echo "$fam pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_table.py gpurun_out/pmcw/$fam > gpurun_out/pmcw/$fam/table.txt 2>&1
done
