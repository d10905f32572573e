set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=$GRAFT_REPO_ROOT/gpurun_out/r02xn
mkdir -p $O
timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi bwd --batch 1024 --rounds 5 --iters 10 > $O/conv_bwd.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_conv.py --kernel conv --epi stats --batch 1024 --rounds 5 --iters 10 > $O/conv_stats.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_conv.py --kernel down --epi none --batch 1024 --rounds 5 --iters 10 > $O/down.txt 2>&1
