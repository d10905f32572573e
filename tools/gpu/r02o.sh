set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02o
mkdir -p $O
for v in down_noepi down_nostage; do
  timeout -k 10 200 python -u tools/ab_conv.py --kernel down --epi stats --rounds 3 --iters 10 --lib-a build/abl/libfull.so --lib-b build/abl/lib$v.so > $O/$v.txt 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ab_conv.py --kernel down --epi none --rounds 3 --iters 10 --lib-a build/abl/libfull.so --lib-b build/abl/lib$v.so > $O/${v}_plain.txt 2>&1 || exit 1
done
