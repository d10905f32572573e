set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r02h
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/r02h/conv1x1.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py -k "imagenet" > gpurun_out/r02h/pipe.log 2>&1
