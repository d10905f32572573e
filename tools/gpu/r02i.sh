set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r02i
timeout -k 10 500 python -u bench.py --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 16384 --steps 2 --warmup 1 --json-out gpurun_out/r02i/c5.json > gpurun_out/r02i/c5.log 2>&1
