set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/q4c
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "q4" --timeout 300 --timeout-method thread > gpurun_out/q4c/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/q4c/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 tools/ab_multi.sh 4 gpurun_out/q4c/ab exp_pp exp_q4 > gpurun_out/q4c/ab.txt 2>&1 || exit $?
cat gpurun_out/q4c/ab.txt
cd exp_q4 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/q4c/prof_q4 -o run -- python bench.py --no-cpu-baseline > ../gpurun_out/q4c/prof_q4.log 2>&1 || exit $?
cd ../exp_pp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/q4c/prof_pp -o run -- python bench.py --no-cpu-baseline > ../gpurun_out/q4c/prof_pp.log 2>&1
