#!/bin/bash
# One GPU-box session for a change under test: GPU tests, a same-box step A/B of exp_head/ (a build of the last
# commit, tools/snapshot_head.sh) vs this tree, and the GEMM timers.  Each GPU step has its own limit; the
# script stops at the first fault / abort / timeout (an ordinary test failure, rc 1, does not stop it).
#   tools/gpu_ab.sh OUT [steps...]   steps: test testk(TESTK=expr) ab ab3 sab3 shab gslice lossb trp qmap gemm gemmdbg bench sprof sproft sbench host probe prof
OUT=${1:-gpurun_out/ab}
shift
STEPS=${*:-test ab}
mkdir -p "$OUT"
# (bench.py raises the hardware-queue count itself, but under rocprofv3 the profiler initialises HIP first)
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1 GPU_MAX_HW_QUEUES=8
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
    testk) run pytest_gpu_k 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$TESTK" ;;
    test) run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    ab) run step_ab 600 bash tools/ab_trees.sh exp_head . 4 "$OUT/trees" ;;
    sab3) AB_ARGS=--force-sharded run step_sab3 900 bash tools/ab_multi.sh 4 "$OUT/strees3" exp_head exp_b . ;;
    gslice) run gslice 300 bash -c "for b in 4096 2048 1024; do CC_GEMM_B=\$b CC_GEMM_ONLY=G1_encode_T,G2_decode_ws_T,G3_dacts_T python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so || exit 1; done" ;;
    shab) run shard_ab 900 bash tools/shard_ab.sh 3 "$OUT/shab" exp_head . ;;
    trp) run trp 300 python tools/transpose_probe.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so $(ls crosscoder-model-diff-replication_amd/exp/*.so) ;;
    lossb) run lossb 300 python tools/loss_bench.py $(ls crosscoder-model-diff-replication_amd/exp/*.so) crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    qmap) for q in 4 8; do for c in 1 2; do
            GPU_MAX_HW_QUEUES=$q run qmap_q${q}_c${c} 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/qmap_q${q}_c${c}" -o run -- \
              python bench.py --no-cpu-baseline --steps 20 --force-sharded --recon-chunks $c
            f=$(find "$OUT/qmap_q${q}_c${c}" -name '*kernel_trace.csv' | head -1)
            [ -n "$f" ] && python tools/step_timeline.py "$f" 12 > "$OUT/timeline_q${q}_c${c}.txt"; done; done ;;
    ab3) run step_ab3 900 bash tools/ab_multi.sh 4 "$OUT/trees3" exp_prev exp_head . ;;
    gemm) run gemm 300 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip.so ;;
    gemmdbg) run gemmdbg 300 python tools/gemm_bench.py crosscoder-model-diff-replication_amd/libcrosscoder_hip_dbg.so@5 \
               crosscoder-model-diff-replication_amd/libcrosscoder_hip_dbg.so@7 ;;
    bench) run bench 300 python bench.py ;;
    sprof) run sprof 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sprof" -o run -- \
             python bench.py --no-cpu-baseline --steps 20 --force-sharded
           f=$(find "$OUT/sprof" -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && python tools/step_timeline.py "$f" 12 > "$OUT/timeline_sharded.txt" ;;
    sbench) run sbench 400 bash -c "python bench.py --no-cpu-baseline --force-sharded > $OUT/sh4.json && python bench.py --no-cpu-baseline --force-sharded --recon-chunks 2 > $OUT/sh2.json && python bench.py --no-cpu-baseline --force-sharded --recon-chunks 1 > $OUT/sh1.json && python bench.py --no-cpu-baseline > $OUT/single.json" ;;
    host) run host 400 bash -c "python tools/host_probe.py && python tools/host_probe.py --sharded && python tools/host_probe.py --sharded --recon-chunks 1" ;;
    sproft) run sproft 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/sproft" -o run -- \
              python bench.py --no-cpu-baseline --steps 20 --force-sharded
            f=$(find "$OUT/sproft" -name '*kernel_trace.csv' | head -1); g=$(find "$OUT/sproft" -name '*hip_api_trace.csv' | head -1)
            [ -n "$f" ] && python tools/step_timeline.py "$f" 12 $g > "$OUT/timeline_sharded_api.txt" ;;
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
