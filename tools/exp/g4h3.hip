// EXPERIMENT (tools only, never linked into the product): the 4-wave 128 x 128-per-wave bf16 GEMM of g4h.hip with
// the K-loop schedule of the vendor library's gfx950 kernel for this shape (hipBLASLt
// Custom_Cijk_Alik_Bljk_..._MT256x256x64_MI16x16x1, read with llvm-objdump for study; slot numbers = MFMAs issued
// before the instruction, 128 MFMAs per 64-deep K step):
//   MFMAs 0-63 on the k-slice-0 fragments F0 (read at the end of the previous step), 64-127 on k-slice 1 (F1);
//   1-15 (every 2): the 8 A fragments of k-slice 1;  lgkmcnt(0) after 21, barrier after 22 (the A region of this
//   step's buffer is free) -> the 8 A DMAs of step t+2 into it (23 .. 59);  25-43: the 8 B fragments of k-slice 1;
//   lgkmcnt(0) after 51, barrier after 52 -> the 8 B DMAs of step t+2 (62 .. 125);  vmcnt(13) after 92 (every DMA
//   of the PREVIOUS step landed: this step issued 13 so far), barrier after 93 -> the 16 F0 reads of step t+1
//   (94-124);  lgkmcnt(0) after 127.  Each DMA has ~1.2-1.5 K steps to land (g4h: one, behind a vmcnt(0)).
//   C[M][N] (bf16) = A[M][K] . B[N][K]^T, both operands K-contiguous; M, N % 256 == 0, K % 64 == 0, K >= 128.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#ifndef G4H_GM
#define G4H_GM 4
#endif
// schedule knobs (G4H_TUNE): first MFMA of the section-1 / section-2 fragment reads and of the DMAs, spacing, and a
// shift for the odd waves (their SIMD pair issues its LDS traffic at other MFMAs: the vendor kernel keeps two loop
// copies, picked by the SIMD id)
#ifndef G4H_TUNE
#define G4H_TUNE 0
#endif
#ifndef G4H_R1_START
#define G4H_R1_START 0
#endif
#ifndef G4H_R2_START
#define G4H_R2_START 0
#endif
#ifndef G4H_D_START
#define G4H_D_START 1
#endif
#ifndef G4H_D_EVERY
#define G4H_D_EVERY 4
#endif
#ifndef G4H_PAR
#define G4H_PAR 0
#endif
#ifndef G4H_SPLIT  // 1: step t+1's DMAs split over section 2 of step t-1 and section 1 of step t
#define G4H_SPLIT 0
#endif
#ifndef G4H_RD_EVERY  // MFMAs between two LDS fragment reads in a section (64 MFMAs, 16 reads)
#define G4H_RD_EVERY 4
#endif

#ifndef G4H_PIN
#define G4H_PIN 0
#endif
#if G4H_PIN
#include "g4h3_pin.h"
#endif
namespace g4h {
// vendor schedule slots (after the MFMA with that 0-based index), see the header
constexpr int RA[8] = {0, 2, 4, 6, 8, 10, 12, 14};
constexpr int DA[8] = {22, 25, 28, 31, 34, 52, 55, 58};
constexpr int RB[8] = {24, 27, 30, 33, 36, 38, 40, 42};
constexpr int DB[8] = {61, 64, 85, 87, 89, 96, 100, 124};
constexpr int R0[16] = {93, 94, 95, 97, 98, 102, 103, 104, 105, 106, 109, 112, 114, 117, 120, 123};
template <int N>
constexpr int find_slot(const int (&s)[N], int m) {
  for (int q = 0; q < N; ++q)
    if (s[q] == m) return q;
  return -1;
}
template <class F, int... Ms>
__device__ __forceinline__ void for_each_slot(F& f, std::integer_sequence<int, Ms...>) {
  (f(std::integral_constant<int, Ms>{}), ...);
}
#ifndef G4H_VLAYOUT
#define G4H_VLAYOUT 0
#endif
// G4H_VLAYOUT 1: the vendor kernel's LDS image -- 1-KB pieces p = 16 h + r16 holding rows {128 h + 16 i + r16, i < 8}
// x 64 K (16 B per (i, 16-B K chunk), i-major), four pieces per 4160-B block (64 B of padding per 4 KB); a DMA moves
// one piece (8 rows 16 apart), a lane's fragment of row group i / k-slice kk sits at 128 i + 64 kk in its piece
constexpr int IMG = G4H_VLAYOUT ? 8 * 4160 : 256 * 128;  // one operand's K-step image
constexpr int BUF = 2 * IMG;

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
  // DMA: wave w moves image pieces 8w .. 8w + 7 of A and of B (piece ci = rows 8ci .. 8ci + 7, 1 KB); lane ->
  // row 8ci + (lane >> 3), logical chunk (lane & 7) ^ (lane >> 3) (the swizzle through the source address)
#if G4H_VLAYOUT
  // piece of DMA q (0..7 per operand) and wave w: p = 4 q + w -> h = q >> 2, r16 = 4 (q & 3) + w; lane -> row
  // 128 h + 16 (lane >> 3) + r16, K chunk lane & 7
  const uint32_t va = (uint32_t)(((int64_t)(16 * (lane >> 3) + wave) * lda + 8 * (lane & 7)) * 2);
  const uint32_t vb = (uint32_t)(((int64_t)(16 * (lane >> 3) + wave) * ldb + 8 * (lane & 7)) * 2);
  auto qrow = [](int q) { return 128 * (q >> 2) + 4 * (q & 3); };
  const int sa = (int)(lda * 2), sb = (int)(ldb * 2);  // (times qrow)
#else
  const int rl = lane >> 3, cl = (lane & 7) ^ rl;
  const uint32_t va = (uint32_t)(((int64_t)(64 * wave + rl) * lda + 8 * cl) * 2);
  const uint32_t vb = (uint32_t)(((int64_t)(64 * wave + rl) * ldb + 8 * cl) * 2);
  const int sa = (int)(8 * lda * 2), sb = (int)(8 * ldb * 2);  // one piece further (8 rows)
#endif
  const int nk = K / 64;
  // K stagger (G4H_SU > 1): the tile's K loop starts at K step (stagger index * G4H_SS) mod nk and wraps, so the
  // tiles that share an operand panel read different K slices of it at any moment (the vendor kernel's StaggerU);
  // stagger index = (tn + G4H_SM * tm) mod G4H_SU
#ifndef G4H_SU
#define G4H_SU 1
#endif
#ifndef G4H_SS
#define G4H_SS 1
#endif
#ifndef G4H_SM
#define G4H_SM 0
#endif
  const int koff = __builtin_amdgcn_readfirstlane((((tn + G4H_SM * tm) % G4H_SU) * G4H_SS) % nk);
  auto dma = [&](int s, int q) {  // piece q (0..7: A, 8..15: B) of step s into buffer s & 1
    const int ks = s + koff >= nk ? s + koff - nk : s + koff;  // (the stagger's wrapped K step)
#if G4H_VLAYOUT
    char* dst = smem + (s & 1) * BUF + (q < 8 ? 0 : IMG) + (q & 7) * 4160 + wave * 1024;
    const int so = qrow(q & 7) * (q < 8 ? sa : sb) + ks * 128;
#else
    char* dst = smem + (s & 1) * BUF + (q < 8 ? 0 : IMG) + (8 * wave + (q & 7)) * 1024;
    const int so = (q & 7) * (q < 8 ? sa : sb) + ks * 128;
#endif
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 8 ? ra : rb, (lds_void*)dst, 16, (int)(q < 8 ? va : vb), so, 0, 0);
  };
  // fragment lane offset: row (lane & 15) of a 16-row group, chunk 4 kk + (lane >> 4), swizzled
#if G4H_VLAYOUT
  auto pbase = [](int p) { return (p >> 2) * 4160 + (p & 3) * 1024; };
  const int vA = pbase(16 * wr + (lane & 15)) + 16 * (lane >> 4);
  const int vB = IMG + pbase(16 * wc + (lane & 15)) + 16 * (lane >> 4);
  auto frag = [&](int s, int kk, int f) {  // f 0..7: A row group f of the wave; 8..15: B column group f - 8
    const char* base = smem + (s & 1) * BUF + (f < 8 ? vA + 128 * f : vB + 128 * (f - 8)) + 64 * kk;
    return *(const bf16x8*)base;
  };
#else
  int foff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) foff[kk] = (lane & 15) * 128 + (((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4);
  auto frag = [&](int s, int kk, int f) {  // f 0..7: A row group f of the wave; 8..15: B column group f - 8
    const char* base = smem + (s & 1) * BUF + (f < 8 ? (wr * 128 + 16 * f) * 128 : IMG + (wc * 128 + 16 * (f - 8)) * 128);
    return *(const bf16x8*)(base + foff[kk]);
  };
#endif

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 F0[16], F1[16];  // k-slice 0 / 1 fragments: [0..7] A row groups, [8..15] B column groups
  // prologue: steps 0 and 1, then step 0's k-slice-0 fragments
#pragma unroll
  for (int q = 0; q < 16; ++q) dma(0, q);
  if (nk > 1) {
#if G4H_SPLIT  // (step 1's second half: section 1 of step 0)
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(1, q);
    __builtin_amdgcn_s_waitcnt((8) | (7 << 4) | (15 << 8));  // vmcnt(8)
#else
#pragma unroll
    for (int q = 0; q < 16; ++q) dma(1, q);
    __builtin_amdgcn_s_waitcnt((16 & 15) | (7 << 4) | (15 << 8) | ((16 >> 4) << 14));  // vmcnt(16)
#endif
  } else {
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));  // vmcnt(0)
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) F0[f] = frag(0, 0, f);

  // the MFMAs are inline asm on AGPR accumulators ("+a": the compiler keeps all 256 there, no copies), in program
  // order; sched_barrier pins each read / DMA between its two MFMAs
#define G4H_MFMA(ACC, BF, AF) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(BF), "v"(AF))
  // (schedule slots: g4h3::RA etc.; every slot is resolved at compile time)
  auto step = [&](auto more_c, auto dmas_c, int t) {
    constexpr bool MORE = decltype(more_c)::value, DMAS = decltype(dmas_c)::value;
    auto body = [&](auto mc) {
      constexpr int m = decltype(mc)::value;
#ifndef G4H_SRC0_CONST
#define G4H_SRC0_CONST 0
#endif
      // (G4H_SRC0_CONST: j outer, i inner -- src0, the B fragment, stays the same over 8 consecutive MFMAs, as in the
      // vendor loop; else i outer, src1 constant)
      constexpr int i = G4H_SRC0_CONST ? (m & 7) : ((m & 63) >> 3), j = G4H_SRC0_CONST ? ((m & 63) >> 3) : (m & 7);
#if G4H_PIN
      if constexpr (m < 64) mfma_pin<0, i, j>(acc[i][j], F0[8 + j], F0[i]);
      else mfma_pin<1, i, j>(acc[i][j], F1[8 + j], F1[i]);
#else
      if constexpr (m < 64) G4H_MFMA(acc[i][j], F0[8 + j], F0[i]);
      else G4H_MFMA(acc[i][j], F1[8 + j], F1[i]);
#endif
      constexpr int qa = find_slot(RA, m), qb = find_slot(RB, m), da = find_slot(DA, m), db = find_slot(DB, m),
                    r0 = find_slot(R0, m);
      if constexpr (qa >= 0) F1[qa] = frag(t, 1, qa);
      if constexpr (qb >= 0) F1[8 + qb] = frag(t, 1, 8 + qb);
      if constexpr (DMAS && da >= 0) dma(t + 2, da);
      if constexpr (DMAS && db >= 0) dma(t + 2, 8 + db);
      if constexpr (MORE && r0 >= 0) F0[r0] = frag(t + 1, 0, r0);
      if constexpr (m == 20 || m == 50 || m == 126) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      if constexpr (m == 91) {
        if constexpr (DMAS) __builtin_amdgcn_s_waitcnt((13) | (7 << 4) | (15 << 8));  // vmcnt(13)
        else __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));                   // vmcnt(0)
      }
      if constexpr (m == 21 || m == 51 || m == 92) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    for_each_slot(body, std::make_integer_sequence<int, 128>{});
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
}  // namespace g4h

extern "C" int g4_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % 64) || (N % 256) || (M % 256)) return 1;
  const int nbm = (int)(M / 256), nbn = (int)(N / 256);
  hipLaunchKernelGGL(g4h::gemm_kernel, dim3(nbm * nbn), dim3(256), 0, (hipStream_t)stream, A, B, C, (int)M, (int)N,
                     (int)K, lda, ldb, ldc, nbm, nbn);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
