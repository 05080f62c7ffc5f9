// Experiment (tools only): per-CU store rate of 16-B-per-lane buffer stores, 512-thread workgroups
// (8 waves) writing `kb` KB each as 1-KB wave-instructions (the epilogue's pattern: each wave
// instruction = 2 rows x 512 B of a row-major tile with row stride ld), one workgroup per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__global__ __launch_bounds__(512, 1) void store_tile(char* out, int64_t ld_bytes, int pieces, int tiles_per_wg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u32x4 v = {(unsigned)threadIdx.x, 1u, 2u, 3u};
  for (int t = 0; t < tiles_per_wg; ++t) {
    const int64_t tile = (int64_t)blockIdx.x * tiles_per_wg + t;
    // tile = 256 rows x 512 B at (tile row block, column block): place tiles side by side in rows of ld
    char* base = out + (tile / 16) * 256 * ld_bytes + (tile % 16) * 512;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7ffffff0, 0x00020000);
    for (int q = 0; q < pieces; ++q) {
      const int ci = q * 8 + wave;
      const int row = 2 * ci + (lane >> 5);
      const uint32_t off = (uint32_t)(row * ld_bytes + (lane & 31) * 16);
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
    }
  }
}

extern "C" int store_run(char* out, int64_t ld_bytes, int blocks, int pieces, int tiles_per_wg, void* stream) {
  hipLaunchKernelGGL(store_tile, dim3(blocks), dim3(512), 0, (hipStream_t)stream, out, ld_bytes, pieces, tiles_per_wg);
  return (int)hipGetLastError();
}
