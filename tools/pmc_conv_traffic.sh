#!/bin/bash
# Where conv3x3's PMC traffic goes, per ResNet-18 layer shape: one FETCH_SIZE and one WRITE_SIZE
# pass (rocprofv3 does not split counters over passes) per shape of tools/conv_micro.py, each
# shape in its own process so every dispatch of a run is that shape; tabulated by
# tools/conv_traffic_table.py against the algorithmic bytes and the tile geometry's halo rows.
#   tools/pmc_conv_traffic.sh <out dir> [batch] [epi]
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_conv_traffic}
B=${2:-1024}
mkdir -p "$OUT"
for SH in 64:64:32 128:128:16 256:256:8 512:512:4 3:64:32; do
  for C in FETCH_SIZE WRITE_SIZE; do
    D="$OUT/${SH//:/_}/$C"
    mkdir -p "$D"
    timeout -s KILL 90 rocprofv3 --pmc $C -T --output-format csv -d "$D" -o run -- \
        python3 tools/conv_micro.py --iters 5 --only conv --batch "$B" --shapes "$SH" \
        > "$D/run.log" 2>&1
    rc=$?
    echo "$SH $C rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/conv_traffic_table.py "$OUT" "$B" > "$OUT/table.txt" 2>&1
cat "$OUT/table.txt"
