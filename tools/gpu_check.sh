set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 240 --timeout-method thread -k "config2_trainer_steps or trainer_steps" > gpurun_out/r3c/calib.log 2>&1
rc=$?; echo "calib rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3c/all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -3 gpurun_out/r3c/all.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3c/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/r3c/bench.log | cut -c1-300
