set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_el2n_fast.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi stats --batch 1024 --rounds 5 --iters 10 > $O/ab_conv_stats.txt 2>&1
