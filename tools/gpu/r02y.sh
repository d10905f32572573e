set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=$GRAFT_REPO_ROOT/gpurun_out/r02y
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u tools/conv_micro.py --only conv,down --batch 1024 > $O/base_$r.txt 2>&1 || exit 1
  DD_DOWN_NA=2 timeout -k 10 200 python -u tools/conv_micro.py --only down --batch 1024 > $O/downna2_$r.txt 2>&1 || exit 1
  DD_CONV_TILE=wide timeout -k 10 200 python -u tools/conv_micro.py --only conv --batch 1024 > $O/wide_$r.txt 2>&1 || exit 1
done
