#!/bin/bash
# Probe library for tools/tile_anatomy.py: the debug build with per-tile clock stamps (-DCC_PP_STAMPS), linked
# against the tree's step / aux objects.  Output: exp_stamps/libstamps.so (not shipped, not used by tests).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/crosscoder-model-diff-replication_amd/csrc
make -s -C "$C" -j8
mkdir -p "$ROOT/exp_stamps"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -munsafe-fp-atomics \
  -DCC_DEBUG_HOOKS -DCC_PP_STAMPS -c "$C/gemm.hip" -o "$ROOT/exp_stamps/gemm_st.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script="$C/exports.map" \
  "$ROOT/exp_stamps/gemm_st.o" "$C/step_kernels.o" "$C/aux_kernels.o" -o "$ROOT/exp_stamps/libstamps.so"
rm -f "$ROOT/exp_stamps/gemm_st.o"
echo "$ROOT/exp_stamps/libstamps.so"
