#!/bin/bash
# One GPU-box session: parity tests, the bench line, a rocprofv3 kernel-trace summary of the same
# bench command, and the GEMM / Adam A/B timers.  Every GPU step has its own time limit; the script
# stops at the first fault, abort, segfault or timeout (test FAILURES -- exit 1 -- do not stop it).
# Usage (repo root on the box): tools/gpu_round.sh [OUT] [steps...]
#   steps: test smoke bench prof configs sharded rehearse gemm ab stepab small adam pmc
OUT=${1:-gpurun_out/round}
shift
STEPS=${*:-test bench prof gemm adam}
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONDONTWRITEBYTECODE=1
# bench.py raises the HIP hardware-queue count to 8 itself; under rocprofv3 the profiler initialises HIP
# before bench.py runs, so the profiled runs get it from here
export GPU_MAX_HW_QUEUES=8

run() {  # run NAME LIMIT CMD...; returns 0 on success or ordinary failure (1), else aborts
  local name=$1 lim=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with $rc"
    tail -20 "$OUT/$name.log"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    test) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ;;
    configs) for c in 3 4 5; do run bench_config$c 400 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 3; done ;;
    rehearse) for n in 2 4; do CC_BENCH_ONE_DEVICE=1 run rehearse_n$n 400 python bench.py --gpus $n --steps 5 \
                --warmup 2 --deadline 360 --no-cpu-baseline; done ;;
    sharded) run bench_sharded 300 python bench.py --no-cpu-baseline --force-sharded
             run bench_sharded_rs 300 python bench.py --no-cpu-baseline --force-sharded --comm reduce_scatter ;;
    prof) run rocprof_stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python bench.py --no-cpu-baseline ;;
    gemm) run gemm_bench 300 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    ab) run gemm_ab 400 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/exp/base.so \
          crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    stepab) run step_ab 400 python tools/step_ab.py --spans ;;
    small) run small_bench 200 python tools/small_bench.py crosscoder-model-diff-replication_amd/exp/base.so \
             crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    adam) run adam_bench 200 python tools/adam_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    pmc)
      run pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc/p1" -o pmc -- \
          python bench.py --steps 3 --warmup 1 --no-cpu-baseline
      run pmc_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc/p2" -o pmc -- \
          python bench.py --steps 3 --warmup 1 --no-cpu-baseline
      run pmc_sq 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
          --output-format csv -d "$OUT/pmc/p3" -o pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
      run pmc_mfma 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
          --output-format csv -d "$OUT/pmc/p4" -o pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
      ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done"
