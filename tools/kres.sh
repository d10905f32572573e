#!/bin/bash
# Per-kernel resource usage (VGPR/AGPR/spills/occupancy/LDS) of one HIP source file.
#   tools/kres.sh <file.hip> [kernel-name-filter]
f=$1; filt=${2:-.}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I"$(dirname "$0")/../include" \
  -I"$(dirname "$f")" -c --cuda-device-only -Rpass-analysis=kernel-resource-usage "$f" \
  -o /dev/null 2>&1 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | awk '
  /Function Name/ {if (n) print line; n=$3; line=n; next}
  /VGPRs:|AGPRs:|Spill:|Occupancy|LDS Size/ {gsub(/ +/," "); line=line " |" $0}
  END {print line}' | grep -E "$filt"
