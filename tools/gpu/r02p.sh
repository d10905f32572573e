set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_down.py tests/test_gpu_kernels.py tests/test_gpu_el2n_fast.py > $O/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ab_conv.py --kernel down --epi stats --rounds 5 --iters 10 > $O/ab_down_stats.txt 2>&1 && \
timeout -k 10 200 python -u tools/ab_conv.py --kernel down --epi none --rounds 5 --iters 10 > $O/ab_down_none.txt 2>&1
