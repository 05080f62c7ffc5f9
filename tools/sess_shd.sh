set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
mkdir -p gpurun_out/shd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "sharded or g2_kernel_wait" --timeout 200 --timeout-method thread > gpurun_out/shd/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/shd/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for args in "" "--force-sharded --recon-chunks 1" "--force-sharded --recon-chunks 2"; do
  echo "== $args"
  AB_ARGS="$args" timeout -k 10 600 tools/ab_multi.sh 3 "gpurun_out/shd/ab$(echo $args | tr -d ' -')" exp_before exp_after || exit $?
done
