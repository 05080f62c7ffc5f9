#!/bin/bash
# One GPU-box session for a change under test: GPU tests, a same-box step A/B of exp_head/ (a build of the last
# commit, tools/snapshot_head.sh) vs this tree, and the GEMM timers.  Each GPU step has its own limit; the
# script stops at the first fault / abort / timeout (an ordinary test failure, rc 1, does not stop it).
#   tools/gpu_ab.sh OUT [steps...]   steps: test ab gemm gemmdbg
OUT=${1:-gpurun_out/ab}
shift
STEPS=${*:-test ab}
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
run() {
  local name=$1 lim=$2
  shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name ended with $rc"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    test) run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    ab) run step_ab 600 bash tools/ab_trees.sh exp_head . 4 "$OUT/trees" ;;
    ab3) run step_ab3 900 bash tools/ab_multi.sh 4 "$OUT/trees3" exp_prev exp_head . ;;
    gemm) run gemm 300 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    gemmdbg) run gemmdbg 300 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip_dbg.so@5 \
               crosscoder-model-diff-replication_amd/libcrosscoder_hip_dbg.so@7 ;;
    bench) run bench 300 python bench.py ;;
    sprof) run sprof 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sprof" -o run -- \
             python bench.py --no-cpu-baseline --steps 20 --force-sharded
           f=$(find "$OUT/sprof" -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && python tools/step_timeline.py "$f" 12 > "$OUT/timeline_sharded.txt" ;;
    sbench) run sbench 400 bash -c "python bench.py --no-cpu-baseline --force-sharded > $OUT/sh4.json && python bench.py --no-cpu-baseline --force-sharded --recon-chunks 2 > $OUT/sh2.json && python bench.py --no-cpu-baseline --force-sharded --recon-chunks 1 > $OUT/sh1.json && python bench.py --no-cpu-baseline > $OUT/single.json" ;;
    probe) run probe 400 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so \
             $(ls crosscoder-model-diff-replication_amd/exp/*.so) ;;
    prof) run prof_new 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_new" -o run -- \
            python bench.py --no-cpu-baseline --steps 20
          run prof_old 300 bash -c "cd exp_head && rocprofv3 --kernel-trace --output-format csv -d ../$OUT/prof_old -o run -- python bench.py --no-cpu-baseline --steps 20"
          for t in new old; do f=$(find "$OUT/prof_$t" -name '*kernel_trace.csv' | head -1); \
            [ -n "$f" ] && python tools/step_timeline.py "$f" 12 > "$OUT/timeline_$t.txt"; done ;;
  esac
done
echo done
