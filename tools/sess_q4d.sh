set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/q4d
timeout -k 10 900 tools/ab_multi.sh 4 gpurun_out/q4d/ab exp_pp exp_q4m2 exp_q4m3 > gpurun_out/q4d/ab.txt 2>&1 || exit $?
cat gpurun_out/q4d/ab.txt
cd exp_q4m3 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/q4d/prof_q4m3 -o run -- python bench.py --no-cpu-baseline > ../gpurun_out/q4d/prof_q4m3.log 2>&1
