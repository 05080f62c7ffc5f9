// EXPERIMENT (tools only): the product's 4-wave assembly K loop (csrc/gemm_q4.h, q4_kloop.inc) with a plain bf16
// store epilogue, behind the g4_gemm_bf16 entry tools/g4_bench.py and tools/gemm_ksweep.py time against hipBLASLt
// and the ping-pong.  C[M][N] (bf16) = A[M][K] . B[N][K]^T; M, N % 256 == 0, K % 64 == 0, K >= 128.
// -DG4A_NOSTORE: no output stores (the K loop alone).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CC_DEV __device__ __forceinline__
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
namespace cc {
#include "../../crosscoder-model-diff-replication_amd/csrc/gemm_q4.h"
}  // namespace cc

namespace g4a {
__device__ __forceinline__ void tile_of_block(int bid, int nbm, int nbn, int& tm, int& tn) {
  int nwg = nbm * nbn;
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GM = 4;
  int per_group = GM * nbn;
  int g = wg / per_group;
  int first = g * GM;
  int gm = nbm - first < GM ? nbm - first : GM;
  int w = wg - g * per_group;
  tm = first + w % gm;
  tn = w / gm;
}
__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }

__global__ __launch_bounds__(256, 1) void gemm_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                      char* __restrict__ C, int M, int N, int K, int64_t lda,
                                                      int64_t ldb, int64_t ldc, int nbm, int nbn) {
  __shared__ __attribute__((aligned(16))) char smem[cc::Q4_LDS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  tile_of_block(blockIdx.x, nbm, nbn, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  f32x4 acc[8][8];
  cc::q4_kloop(acc, A + (int64_t)m0 * lda * 2, B + (int64_t)n0 * ldb * 2, lda, (uint64_t)(M - m0) * lda * 2,
               (uint64_t)(N - n0) * ldb * 2, K / 64, smem, lane, wave);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C + ((int64_t)m0 * ldc + n0) * 2, (short)0,
                                                                     (int)(((uint64_t)255 * ldc + 256) * 2), 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = wc * 128 + j * 16 + 4 * (lane >> 4);
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (short)f2bf(acc[i][j][e]);
#ifndef G4A_NOSTORE
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rc, (int)(((int64_t)row * ldc + col) * 2), 0,
                                            0);
#else
      if (v[0] == 12345 && v[1] == -7) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rc, 0, 0, 0);
#endif
    }
  }
}
}  // namespace g4a

extern "C" int g4_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, void* stream) {
  if (M <= 0 || N <= 0 || K < 128 || (K % 64) || (N % 256) || (M % 256) || lda != ldb) return 1;
  const int nbm = (int)(M / 256), nbn = (int)(N / 256);
  hipLaunchKernelGGL(g4a::gemm_kernel, dim3(nbm * nbn), dim3(256), 0, (hipStream_t)stream, (const char*)A,
                     (const char*)B, (char*)C, (int)M, (int)N, (int)K, lda, ldb, ldc, nbm, nbn);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
