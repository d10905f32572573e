set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06s7b
timeout -k 10 300 python -u -m pytest tests/test_gpu_el2n_fast.py -m gpu -x -q --timeout 120 --timeout-method thread -k stem7 > gpurun_out/r06s7b/pytest.log 2>&1 || { tail -30 gpurun_out/r06s7b/pytest.log; exit 1; }
tail -1 gpurun_out/r06s7b/pytest.log
timeout -k 10 300 python -u tools/stem7_micro.py 2>&1 | grep -v amdgpu | tee gpurun_out/r06s7b/stem7_micro.log
