set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=$GRAFT_REPO_ROOT/gpurun_out/r02rm
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_el2n_fast.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 16384 --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --arch resnet50 --classes 100 --ckpts 2 --n 8192 --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/c4.json > $O/c4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/c2.json > $O/c2.log 2>&1
