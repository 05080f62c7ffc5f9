#!/bin/bash
# Experiment build of the library with extra defines (never shipped): tools/build_variant.sh NAME -DFOO=1 ...
# -> crosscoder-model-diff-replication_amd/exp/NAME.so ; time it with tools/step_ab.py --lib <path> (tools only).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/crosscoder-model-diff-replication_amd/csrc
OUT=$ROOT/crosscoder-model-diff-replication_amd/exp
mkdir -p "$OUT/$NAME.obj"
for f in gemm step_kernels aux_kernels; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics "$@" -c "$SRC/$f.hip" \
      -o "$OUT/$NAME.obj/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$OUT/$NAME.obj/"*.o -o "$OUT/$NAME.so"
rm -rf "$OUT/$NAME.obj"
echo "$OUT/$NAME.so"
