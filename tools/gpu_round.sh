#!/bin/bash
# One GPU-box session (run from the repo root on the box; results under gpurun_out/<tag>/):
#   tools/gpu_round.sh <tag> [step ...]      (default: tests smoke bench prof)
# steps:
#   tests    pytest -m gpu (parity; DD_PARITY_OUT records keep-set swap counts)
#   some     pytest -m gpu on the files in $TESTS, -k "$KEXPR" when set
#   smoke    __graft_entry__.smoke()
#   bench    the default bench line (config 2, N = 1)
#   dbench   the driver's bench command line (--gpus 1 --steps 20 --warmup 5)
#   pmc      FETCH_SIZE / WRITE_SIZE passes over a short bench (tools/pmc_bench.sh)
#   busy     MFMA busy of the conv and GraNd norm kernels (tools/pmc_pegrad_busy.sh)
#   spawn    bench.py --gpus 1 --spawn (self-launched rank, world-1 RCCL group + all-gather)
#   shards   bench lines at the rank-0 shard sizes of W = 2 / 4 / 8 (24960 / 12416 / 6144
#            examples): the per-rank compute side of the 1 -> 8 curve, as a projection
#   w2share  bench.py --gpus 2 --share-device (two ranks on cuda:0, gloo gather)
#   prof     rocprofv3 --kernel-trace --stats of a short single-lane bench (per-kernel durations
#            not stretched by co-scheduled lanes: they match the bench's isolated roofline)
#            + idle-gap summary
#   c4       config 4 line (ResNet-50 / CIFAR-100, N = 50k, K = 10, EL2N + GraNd)
#   c5       config 5 line (ResNet-50 ImageNet shape, 1,281,167 examples, EL2N)
#   dropin   sparse_loader timing at N = 50k (fast path vs engine EL2N pass)
#   hbm      byte-bound kernels (EL2N / normalise / select) HBM sweep under rocprofv3
# Every GPU step has its own time limit; the first failure ends the session.
set -uo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-run}
shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run <seconds> <log> cmd...
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  [ $rc -eq 0 ] || { echo "step failed rc=$rc ($log)"; exit $rc; }
}
for s in $STEPS; do
  case $s in
    tests)
      DD_PARITY_OUT="$OUT/keepset_swaps.json" run 1100 "$OUT/pytest_gpu.log" \
          python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    some)
      DD_PARITY_OUT="$OUT/keepset_swaps.json" run 900 "$OUT/pytest_some.log" \
          python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --timeout 300 \
          --timeout-method thread ;;
    shards)
      for n in 24960 12416 6144; do
        run 600 "$OUT/bench_shard_$n.log" python -u bench.py --n $n --no-cpu-baseline \
            --json-out "$OUT/bench_shard_n$n.json"
      done ;;
    shards_ab)
      # the launch plan A/B at the shard sizes: even (round 4) vs full chunks + short tail,
      # alternated twice on the same box
      for r in 1 2; do
        for n in 24960 12416 6144; do
          run 600 "$OUT/bench_shard_even_${n}_$r.log" python -u bench.py --n $n --no-cpu-baseline \
              --steps 3 --even-chunks --json-out "$OUT/bench_shard_even_n${n}_$r.json"
          run 600 "$OUT/bench_shard_tail_${n}_$r.log" python -u bench.py --n $n --no-cpu-baseline \
              --steps 3 --json-out "$OUT/bench_shard_tail_n${n}_$r.json"
        done
      done ;;
    w2share)
      run 600 "$OUT/bench_w2share.log" python -u bench.py --gpus 2 --share-device \
          --json-out "$OUT/bench_w2share.json" ;;
    smoke)
      run 300 "$OUT/smoke.log" python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' ;;
    bench)
      run 900 "$OUT/bench.log" python -u bench.py --json-out "$OUT/bench.json" ;;
    dbench)
      # the driver's own command line (BENCH_rNN: --steps 20 --warmup 5)
      run 900 "$OUT/bench_driver.log" python -u bench.py --gpus 1 --steps 20 --warmup 5 \
          --json-out "$OUT/bench_driver.json" ;;
    pmc)
      run 600 "$OUT/pmc.log" bash tools/pmc_bench.sh "$OUT/pmc" ;;
    busy)
      run 300 "$OUT/busy.log" bash tools/pmc_pegrad_busy.sh "$OUT/busy" ;;
    spawn)
      run 600 "$OUT/bench_spawn.log" python -u bench.py --gpus 1 --spawn --no-cpu-baseline \
          --json-out "$OUT/bench_spawn_n1.json" ;;
    prof)
      run 900 "$OUT/prof.log" rocprofv3 --kernel-trace --stats -T --output-format csv \
          -d "$OUT/prof" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
          --lanes 1 --json-out "$OUT/bench_under_rocprof.json"
      TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
      if [ -n "$TRACE" ]; then
        python3 tools/trace_summary.py "$TRACE" 1 > "$OUT/trace_summary.txt"  # 1 warmup step
        rm -f "$TRACE"
        head -25 "$OUT/trace_summary.txt"
      fi ;;
    c4)
      run 900 "$OUT/c4.log" python -u bench.py --arch resnet50 --classes 100 --steps 1 \
          --warmup 1 --json-out "$OUT/bench_c4.json" ;;
    c5)
      run 900 "$OUT/c5.log" python -u bench.py --imagenet --arch resnet50 --classes 1000 \
          --ckpts 1 --n 1281167 --steps 1 --warmup 1 --json-out "$OUT/bench_c5.json" ;;
    dropin)
      run 600 "$OUT/dropin.log" python -u tools/bench_dropin.py --json-out "$OUT/dropin.json" ;;
    hbm)
      run 900 "$OUT/hbm.log" bash tools/hbm_roofline.sh "$OUT/hbm" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
