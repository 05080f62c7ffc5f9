#!/bin/bash
# Same-box A/B of the in-tree library vs crosscoder-model-diff-replication_amd/exp/head.so (a build of the last commit):
# targeted GPU tests, then tools/step_ab.py --only=default alternating old / new twice.
set -o pipefail
mkdir -p gpurun_out/r1q
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dec_norms or fused_decoder or full_size or trainer_steps" > gpurun_out/r1q/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python tools/step_ab.py --lib crosscoder-model-diff-replication_amd/exp/head.so > gpurun_out/r1q/old_$i.log 2>&1 || exit 1
  timeout -k 10 150 python tools/step_ab.py > gpurun_out/r1q/new_$i.log 2>&1 || exit 1
done
