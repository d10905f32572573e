set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=$GRAFT_REPO_ROOT/gpurun_out/r02sc
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "head" tests/test_gpu_pipeline.py -k "head or grand or fused" > $O/tests.log 2>&1 || exit 1
for n in 6250 12500 25000; do
  timeout -k 10 300 python -u bench.py --n $n --steps 3 --warmup 1 --no-cpu-baseline --json-out $O/n$n.json > $O/n$n.log 2>&1 || exit 1
done
