set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02s
mkdir -p $O
for v in c1_noload c1_nostage c1_noepi; do
  timeout -k 10 200 python -u tools/ab_conv.py --kernel c1x1 --epi stats --batch 512 --rounds 3 --iters 10 --lib-a build/abl/libfull.so --lib-b build/abl/lib$v.so > $O/$v.txt 2>&1 || exit 1
done
