#!/bin/bash
# MFMA busy of the GraNd norm kernels and the backbone conv kernels on the ResNet-18 shapes
# (tools/conv_micro.py --only pegrad,conv): one SQ/GRBM counter pass (7 SQ + 1 GRBM counters,
# within one pass's slots), tabulated by tools/pmc_table.py;
#   mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_busy}
mkdir -p "$OUT/p1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T \
    --output-format csv -d "$OUT/p1" -o run -- \
    python3 tools/conv_micro.py --only pegrad,conv --batch 1024 --iters 5 > "$OUT/p1.log" 2>&1
rc=$?
echo "pass rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt" 2>&1
python3 - "$OUT/table.txt" <<'PY' > "$OUT/mfma_busy.txt"
import re, sys
cur = None
rows = {}
for line in open(sys.argv[1]):
    if not line.startswith(" "):
        cur = line.strip()
        rows[cur] = {}
    else:
        k, v = line.split()[:2]
        rows[cur][k] = float(v)
print(f"{'kernel':70s} {'mfma_busy':>9s} {'wait_inst':>9s} {'wait_any':>9s} {'active':>7s}")
for k, d in rows.items():
    if "GRBM_GUI_ACTIVE" not in d or "SQ_VALU_MFMA_BUSY_CYCLES" not in d:
        continue
    busy = d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["GRBM_GUI_ACTIVE"] / 8)
    wc = max(d.get("SQ_WAVE_CYCLES", 1.0), 1.0)
    print(f"{k[:70]:70s} {busy:9.3f} {d.get('SQ_WAIT_INST_ANY', 0) / wc:9.3f} "
          f"{d.get('SQ_WAIT_ANY', 0) / wc:9.3f} {d.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.3f}")
PY
cat "$OUT/mfma_busy.txt"
