set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k el2n > $O/el2n_tests.log 2>&1 && \
bash tools/hbm_roofline.sh $O/hbm > $O/hbm.log 2>&1 && \
timeout -k 10 700 python -u bench.py --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 1281167 --steps 1 --warmup 1 --json-out $O/c5_full.json > $O/c5_full.log 2>&1
