set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=$GRAFT_REPO_ROOT/gpurun_out/r02final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1 && \
WARMUP=1 bash tools/prof_bench.sh $O/prof --steps 2 --warmup 1 --no-cpu-baseline --json-out $O/bench_prof.json > $O/prof.log 2>&1 && \
timeout -k 10 600 python -u bench.py --arch resnet50 --classes 100 --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/c4.json > $O/c4.log 2>&1 && \
timeout -k 10 700 python -u bench.py --imagenet --arch resnet50 --classes 1000 --ckpts 1 --n 1281167 --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/c5.json > $O/c5.log 2>&1
