#!/bin/bash
# dd_select_topk: current build (A) against the working tree (B), the select sizes of the HBM
# sweep in alternated processes; then the select and pegrad GPU tests on the in-tree library
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${1:-gpurun_out/absel}
LA=build/abA/libA.so; LB=build/abB/libB.so
mkdir -p $OUT
for i in 1 2; do
  for v in A B; do
    L=$LA; [ $v = B ] && L=$LB
    DD_LIB=$L DD_HBM_ONLY=select timeout -k 10 180 python -u tools/bench_hbm_kernels.py $OUT/sel_${v}_$i.json > $OUT/sel_${v}_$i.log 2>&1
    rc=$?; echo "== $v $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python - $OUT <<'PY'
import json, sys, glob, statistics
out = sys.argv[1]
res = {}
for v in "AB":
    for f in sorted(glob.glob(f"{out}/sel_{v}_*.log")):
        for line in open(f):
            if line.startswith("{"):
                r = json.loads(line)
                key = (r.get("n"), r.get("k"), r.get("dist", ""))
                res.setdefault(key, {}).setdefault(v, []).append(r["us"])
for key, d in res.items():
    a, b = statistics.median(d["A"]), statistics.median(d["B"])
    print(f"select n={key[0]} k={key[1]} {key[2]:8s} A {a:8.1f} us  B {b:8.1f} us  B/A speed {a / b:5.3f}")
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_select.py -k "select or pegrad" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
