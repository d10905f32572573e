set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ab_conv.py --kernel c1x1 --epi stats --batch 512 --rounds 3 --iters 10 > $O/ab_stats.txt 2>&1 && \
timeout -k 10 200 python -u tools/ab_conv.py --kernel c1x1 --epi none --batch 512 --rounds 3 --iters 10 > $O/ab_none.txt 2>&1
