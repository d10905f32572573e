#!/bin/bash
# Scratch batch for the current gpurun call (overwritten per call; the standing steps are in
# tools/gpu_round.sh).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03g; mkdir -p $O
DD_C1_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread > $O/c1_pipe_tests.log 2>&1 || { tail -30 $O/c1_pipe_tests.log; exit 1; }
tail -1 $O/c1_pipe_tests.log
bash tools/ab_env.sh $O/c1pipe 2 c1x1 DD_C1_PIPE 0 1 || exit 1
bash tools/gpu_round.sh r03g spawn || exit 1
python3 -c "import json;d=json.load(open('$O/bench_spawn_n1.json'));print(d['value'], d['ranks'])"
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $O/pmc_pgram -o run -- python3 tools/conv_micro.py --iters 5 --only pegrad --batch 1024 > $O/pmc_pgram.log 2>&1 || exit 1
bash tools/gpu_round.sh r03g c4 || exit 1
