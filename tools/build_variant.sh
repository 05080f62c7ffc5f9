#!/bin/bash
# Experiment build of the CURRENT sources with extra compile flags, for tools/gemm_bench.py A/Bs:
#   tools/build_variant.sh NAME "-DFLAG=1 ..."   ->  crosscoder-model-diff-replication_amd/exp/NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/crosscoder-model-diff-replication_amd/csrc
OUT=$ROOT/crosscoder-model-diff-replication_amd/exp
B=/tmp/variant_$1
mkdir -p "$OUT" "$B"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -Wall -Wno-unused-function -munsafe-fp-atomics $2"
for s in gemm step_kernels aux_kernels; do
  /opt/rocm/bin/hipcc $F -c "$SRC/$s.hip" -o "$B/$s.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script="$SRC/exports.map" "$B"/*.o -o "$OUT/$1.so"
echo "$OUT/$1.so"
