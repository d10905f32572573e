set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_conv.py tests/test_gpu_conv1x1.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi none --rounds 5 > $O/ab_conv_none.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi bwd --rounds 5 > $O/ab_conv_bwd.txt 2>&1 && \
timeout -k 10 300 python -u tools/conv_micro.py --only c1x1 > $O/c1x1.txt 2>&1
