set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/conv_micro.py --only c1x1 > $O/c1x1.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 16384 --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --arch resnet50 --classes 100 --ckpts 2 --n 8192 --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/c4.json > $O/c4.log 2>&1
