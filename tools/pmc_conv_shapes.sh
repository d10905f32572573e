#!/bin/bash
# SQ counters of conv3x3 per layer shape, each shape in its own process (so a kernel's grid row
# is one shape): MFMA busy, waits, LDS bank conflicts and instruction mix per dispatch
#   tools/pmc_conv_shapes.sh <out dir> <shape ...>   (shape = cin:cout:H)
set -uo pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU"
)
for SH in "$@"; do
  i=0
  for P in "${PASSES[@]}"; do
    i=$((i + 1))
    D="$OUT/${SH//:/_}/p$i"
    mkdir -p "$D"
    timeout -s KILL 90 rocprofv3 --pmc $P -T --output-format csv -d "$D" -o run -- \
        python3 tools/conv_micro.py --iters 5 --only conv --batch 1024 --shapes "$SH" > "$D/run.log" 2>&1
    rc=$?
    echo "$SH pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*_*_*"))):
    vals = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "conv3x3" not in row["Kernel_Name"] or "pack" in row["Kernel_Name"]:
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    v = {k: sum(x) / len(x) for k, x in vals.items()}
    busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / max(v.get("GRBM_GUI_ACTIVE", 1) / 8, 1)
    wc = max(v.get("SQ_WAVE_CYCLES", 1), 1)
    mf = max(v.get("SQ_INSTS_MFMA", 1), 1)
    print(f"{os.path.basename(d):12s} mfma_busy {busy:.3f} wait_inst {v.get('SQ_WAIT_INST_ANY',0)/wc:.3f} "
          f"wait_any {v.get('SQ_WAIT_ANY',0)/wc:.3f} wait_lds {v.get('SQ_WAIT_INST_LDS',0)/wc:.3f} "
          f"lds_conflict/idx_active {v.get('SQ_LDS_BANK_CONFLICT',0)/max(v.get('SQ_LDS_IDX_ACTIVE',1),1):.3f} "
          f"per MFMA: valu {v.get('SQ_INSTS_VALU',0)/mf:.2f} lds {v.get('SQ_INSTS_LDS',0)/mf:.2f} "
          f"vmem {v.get('SQ_INSTS_VMEM_RD',0)/mf:.3f} salu {v.get('SQ_INSTS_SALU',0)/mf:.2f}")
PY
