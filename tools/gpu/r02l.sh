set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02l
mkdir -p $O
for r in 1 2; do
DD_C1_XCD=0 timeout -k 10 200 python -u tools/conv_micro.py --only c1x1 > $O/c1x1_off_$r.txt 2>&1 && \
DD_C1_XCD=1 timeout -k 10 200 python -u tools/conv_micro.py --only c1x1 > $O/c1x1_on_$r.txt 2>&1 || exit 1
done
