set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -k "full_size_config2_trainer_steps_match_oracle or fp32_mode_matches" --timeout 300 --timeout-method thread > gpurun_out/r6e/pytest_s.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6e/pytest_s.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
tools/gpu_round.sh gpurun_out/r6e pmc
