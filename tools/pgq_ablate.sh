#!/bin/bash
# pgram_q ablation (GPU box, repo root): the 16x16 GraNd norm with one piece of work removed
# at a time (DD_PGQ_ABL bits: 1 gather, 2 MFMAs, 4 P write-out, 8 staging loads; 15 all), and
# direct3x3 beside it.  Output: gpurun_out/<tag>/pgq_abl.txt
set -uo pipefail
OUT=gpurun_out/${1:-pgq}
mkdir -p "$OUT"
for abl in 0 1 2 4 8 15; do
  echo "== DD_PGQ_ABL=$abl" >> "$OUT/pgq_abl.txt"
  DD_PGQ=1 DD_PGQ_ABL=$abl timeout -k 10 200 python -u tools/bench_pegrad.py --batch 1024 \
      --iters 10 --auto-only 2>&1 | grep -E "^l2 " >> "$OUT/pgq_abl.txt" || exit 1
done
echo "== direct3x3 (DD_PGQ=0)" >> "$OUT/pgq_abl.txt"
DD_PGQ=0 timeout -k 10 200 python -u tools/bench_pegrad.py --batch 1024 --iters 10 --auto-only \
    2>&1 | grep -E "^l2 " >> "$OUT/pgq_abl.txt"
cat "$OUT/pgq_abl.txt"
