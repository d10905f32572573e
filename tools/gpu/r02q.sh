set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
for f in 1 2 3; do
DD_C1_FAMILY=$f timeout -k 10 200 python -u tools/conv_micro.py --only c1x1 > $O/c1x1_f${f}_$r.txt 2>&1 || exit 1
done
done
