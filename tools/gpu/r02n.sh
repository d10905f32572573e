set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "el2n" > $O/el2n_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py > $O/pipeline_tests.log 2>&1 && \
bash tools/hbm_roofline.sh $O/hbm > $O/hbm.log 2>&1 && \
WARMUP=1 bash tools/prof_bench.sh $O/prof --steps 2 --warmup 1 --json-out $O/bench.json > $O/bench.log 2>&1 && \
WARMUP=1 bash tools/prof_cfg.sh r02n/c4 --arch resnet50 --classes 100 --steps 1 --warmup 1 > $O/c4.log 2>&1
