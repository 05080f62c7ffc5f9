set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/q4e
timeout -k 10 1000 tools/ab_multi.sh 4 gpurun_out/q4e/ab exp_pp exp_q4m2 exp_q4m3 exp_q4m3s86 exp_q4m3s80 > gpurun_out/q4e/ab.txt 2>&1
rc=$?; cat gpurun_out/q4e/ab.txt; exit $rc
