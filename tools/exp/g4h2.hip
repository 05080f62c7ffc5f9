// EXPERIMENT (tools only, never linked into the product): g4h.hip's 4-wave 128 x 128-per-wave bf16 GEMM with the
// LDS-DMAs spread over the whole K step.  Each K-step buffer is split by k-slice: [A kk0 | A kk1 | B kk0 | B kk1],
// 16 KB each ([256 rows][64 B], phys chunk = chunk ^ ((row >> 1) & 2): conflict-free ds_read_b128 fragments), so the
// kk1 halves of step t+1 can be loaded while the kk0 halves of step t+1 are read:
//   section 1 of step t: 64 MFMAs on F0(t); reads F1(t) (kk1 of buffer t&1); DMAs of step t+1's kk1 halves into buffer
//              (t+1)&1 (last read in section 1 of step t-1); then lgkmcnt(0), vmcnt(8) (step t+1's kk0 halves, issued
//              in section 2 of step t-1, landed), barrier.
//   section 2 of step t: 64 MFMAs on F1(t); reads F0(t+1) (kk0 of buffer (t+1)&1); DMAs of step t+2's kk0 halves into
//              buffer t&1 (last read in section 2 of step t-1); then lgkmcnt(0), vmcnt(8), barrier.
// 8 DMAs per wave per section (one per 8 MFMAs: an LDS-DMA costs ~60 issue cycles, an MFMA leaves 8 free), two
// barriers per K step.  C[M][N] (bf16) = A[M][K] . B[N][K]^T, KC/KC; M, N % 256 == 0, K % 64 == 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#ifndef G4H_GM
#define G4H_GM 4
#endif
#ifndef G4H_RD_EVERY  // MFMAs between two LDS fragment reads in a section (64 MFMAs, 16 reads)
#define G4H_RD_EVERY 2
#endif

namespace g4h2 {
constexpr int HALF = 256 * 64;  // one operand's k-slice image of a K step (16 KB)
constexpr int BUF = 4 * HALF;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint64_t bytes) {
  uint32_t n = bytes > 0x7fffffe0u ? 0x7fffffe0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

__device__ __forceinline__ void tile_of_block(int bid, int nbm, int nbn, int& tm, int& tn) {
  int nwg = nbm * nbn;
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GM = G4H_GM;
  int per_group = GM * nbn;
  int g = wg / per_group;
  int first = g * GM;
  int gm = nbm - first < GM ? nbm - first : GM;
  int w = wg - g * per_group;
  tm = first + w % gm;
  tn = w / gm;
}

__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }

__global__ __launch_bounds__(256, 1) void gemm_kernel(const void* __restrict__ A, const void* __restrict__ B,
                                                      void* __restrict__ C, int M, int N, int K, int64_t lda,
                                                      int64_t ldb, int64_t ldc, int nbm, int nbn) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  tile_of_block(blockIdx.x, nbm, nbn, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const __amdgpu_buffer_rsrc_t ra = rsrc((const char*)A + (int64_t)m0 * lda * 2, (uint64_t)256 * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc((const char*)B + (int64_t)n0 * ldb * 2, (uint64_t)256 * ldb * 2);
  // DMA piece q of a (operand, k-slice) half = rows 16q .. 16q + 15 (1 KB); wave w moves pieces 4w .. 4w + 3 of each
  // half: lane -> row 16 (4w + p) + (lane >> 2), phys chunk lane & 3 = logical chunk (lane & 3) ^ ((row >> 1) & 2)
  const int rl = lane >> 2;
  const int cl = (lane & 3) ^ ((rl >> 1) & 2);
  const uint32_t va = (uint32_t)(((int64_t)(64 * wave + rl) * lda + 8 * cl) * 2);
  const uint32_t vb = (uint32_t)(((int64_t)(64 * wave + rl) * ldb + 8 * cl) * 2);
  const int sa = (int)(16 * lda * 2), sb = (int)(16 * ldb * 2);  // one piece further (16 rows)
  const int nk = K / 64;
  // DMA q (0..7) of the kk half of step s: q < 4 -> A piece 4 wave + q, else B piece 4 wave + q - 4
  auto dma = [&](int s, int kk, int q) {
    const bool isA = q < 4;
    char* dst = smem + (s & 1) * BUF + (isA ? 0 : 2 * HALF) + kk * HALF + (4 * wave + (q & 3)) * 1024;
    const int so = (q & 3) * (isA ? sa : sb) + s * 128 + kk * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? ra : rb, (lds_void*)dst, 16, (int)(isA ? va : vb), so, 0, 0);
  };
  // fragment lane offset: row (lane & 15) of a 16-row group, chunk lane >> 4 of the 64-B k-slice row, swizzled
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane & 15) >> 1) & 2)) << 4);
  auto frag = [&](int s, int kk, int f) {  // f 0..7: A row group f of the wave; 8..15: B column group f - 8
    const char* base = smem + (s & 1) * BUF + kk * HALF +
                       (f < 8 ? (wr * 128 + 16 * f) * 64 : 2 * HALF + (wc * 128 + 16 * (f - 8)) * 64);
    return *(const bf16x8*)(base + foff);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 F0[16], F1[16];  // k-slice 0 / 1 fragments: [0..7] A row groups, [8..15] B column groups
  // prologue: step 0 (both halves) and step 1's kk0 half, then step 0's k-slice-0 fragments
#pragma unroll
  for (int q = 0; q < 8; ++q) dma(0, 0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma(0, 1, q);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(1, 0, q);
    __builtin_amdgcn_s_waitcnt((8) | (7 << 4) | (15 << 8));  // vmcnt(8)
  } else {
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));  // vmcnt(0)
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) F0[f] = frag(0, 0, f);

  // the MFMAs are inline asm on AGPR accumulators ("+a": the compiler keeps all 256 there, no copies), in program
  // order; sched_barrier pins each read / DMA between its two MFMAs
#define G4H_MFMA(ACC, BF, AF) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BF), "v"(AF))
  // DMAs and fragment reads at fixed MFMA positions: reads at m % RD == 0 (from the section's first MFMA on), DMAs at
  // m % 8 == 5
  auto step = [&](auto d1_c, auto d2_c, int t) {
    constexpr bool D1 = decltype(d1_c)::value;  // step t+1 exists: its kk1 halves now, its kk0 fragments in section 2
    constexpr bool D2 = decltype(d2_c)::value;  // step t+2 exists: its kk0 halves in section 2
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        G4H_MFMA(acc[i][j], F0[8 + j], F0[i]);
        const int m = i * 8 + j;
        if (m % G4H_RD_EVERY == 0 && m / G4H_RD_EVERY < 16) F1[m / G4H_RD_EVERY] = frag(t, 1, m / G4H_RD_EVERY);
        if (D1 && m % 8 == 5) dma(t + 1, 1, m / 8);
        __builtin_amdgcn_sched_barrier(0);
      }
    if constexpr (D1) __builtin_amdgcn_s_waitcnt((8) | (7 << 4) | (0 << 8));  // vmcnt(8) lgkmcnt(0)
    else __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));               // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        G4H_MFMA(acc[i][j], F1[8 + j], F1[i]);
        const int m = i * 8 + j;
        if (D1 && m % G4H_RD_EVERY == 0 && m / G4H_RD_EVERY < 16) F0[m / G4H_RD_EVERY] = frag(t + 1, 0, m / G4H_RD_EVERY);
        if (D2 && m % 8 == 5) dma(t + 2, 0, m / 8);
        __builtin_amdgcn_sched_barrier(0);
      }
    if constexpr (D2) __builtin_amdgcn_s_waitcnt((8) | (7 << 4) | (0 << 8));
    else __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  int t = 0;
  for (; t + 2 < nk; ++t) step(T_{}, T_{}, t);
  if (t + 1 < nk) step(T_{}, F_{}, t++);
  step(F_{}, F_{}, t);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 2" ::: "memory");  // (MFMA -> v_accvgpr_read of its result)
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
  // epilogue: lane holds row (lane & 15), 4 consecutive columns 4 * (lane >> 4) of each 16 x 16 block
  const __amdgpu_buffer_rsrc_t rc = rsrc((char*)C + ((int64_t)m0 * ldc + n0) * 2, ((uint64_t)255 * ldc + 256) * 2);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = wc * 128 + j * 16 + 4 * (lane >> 4);
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (short)f2bf(acc[i][j][e]);
#ifndef G4H_NOSTORE
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rc, (int)(((int64_t)row * ldc + col) * 2), 0,
                                            0);
#else
      if (v[0] == 12345 && v[1] == -7) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rc, 0, 0, 0);
#endif
    }
  }
}
}  // namespace g4h2

extern "C" int g4_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % 64) || (N % 256) || (M % 256)) return 1;
  const int nbm = (int)(M / 256), nbn = (int)(N / 256);
  hipLaunchKernelGGL(g4h2::gemm_kernel, dim3(nbm * nbn), dim3(256), 0, (hipStream_t)stream, A, B, C, (int)M, (int)N,
                     (int)K, lda, ldb, ldc, nbm, nbn);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
