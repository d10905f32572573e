set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06mp
timeout -k 10 600 python -u -m pytest tests/test_gpu_el2n_fast.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -k "maxpool or imagenet" > gpurun_out/r06mp/pytest.log 2>&1 || { tail -30 gpurun_out/r06mp/pytest.log; exit 1; }
tail -2 gpurun_out/r06mp/pytest.log
bash tools/gpu_round.sh r06mp c5
