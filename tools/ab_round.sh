#!/bin/bash
# One GPU-box A/B session: tools/ab_conv.py over the given epilogues (A = build/ab/libA.so,
# B = build/ab/libB.so), then the named GPU test files against the in-tree libdd.so.
#   tools/ab_round.sh <tag> <kernel> "<epis>" [test files ...]
set -uo pipefail
export TMPDIR=/tmp
TAG=$1; KERNEL=$2; EPIS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for e in $EPIS; do
  echo "== $KERNEL epi $e"
  timeout -k 10 240 python -u tools/ab_conv.py --kernel "$KERNEL" --epi "$e" --rounds 5 \
      --iters 10 --batch 1024 --lib-a "${AB_DIR:-build/abx}/libA.so" \
      --lib-b "${AB_DIR:-build/abx}/libB.so" 2>&1 | grep -v amdgpu.ids || exit 1
done | tee "$OUT/ab.txt"
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1
  rc=$?; tail -4 "$OUT/pytest.log"; exit $rc
fi
