// EXPERIMENT (tools only, never linked into the product): a 4-wave bf16 GEMM with a 128 x 128
// output tile per wave (all 256 accumulator registers), to measure whether that geometry beats
// the product's 8-wave 128 x 64-per-wave ping-pong loop on the G1 / G3 shape.
//   C[M][N] (bf16) = A[M][K] . B[N][K]^T, both operands K-contiguous (KC/KC).
// Tile 256 x 256, waves 2 x 2, K sub-step BK = 32 (64-B rows), NST LDS stages of 32 KB (A | B),
// prefetch NST-1 sub-steps ahead by LDS-DMA (buffer_load ... lds, 16 B per lane), counted vmcnt,
// one raw s_barrier per sub-step.  LDS row swizzle: phys chunk = chunk ^ ((row >> 2) & 3).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#ifndef G4_NST
#define G4_NST 5
#endif
#ifndef G4_GM
#define G4_GM 4
#endif

namespace g4 {
constexpr int NST = G4_NST;
constexpr int STAGE = 2 * 256 * 64;  // A + B images of one 32-deep sub-step (32 KB)
constexpr uint32_t OOB = 0x7ffffff0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint64_t bytes) {
  uint32_t n = bytes > 0x7fffffe0u ? 0x7fffffe0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

template <int N> __device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void tile_of_block(int bid, int nbm, int nbn, int& tm, int& tn) {
  int nwg = nbm * nbn;
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GM = G4_GM;
  int per_group = GM * nbn;
  int g = wg / per_group;
  int first = g * GM;
  int gm = nbm - first < GM ? nbm - first : GM;
  int w = wg - g * per_group;
  tm = first + w % gm;
  tn = w / gm;
}

// MFMA with the accumulator pinned to AGPRs (the compiler otherwise splits the 256 accumulators
// between the VGPR and AGPR files and copies them around the MFMAs).  Only accumulate chains use
// the AGPRs inside the loop (D -> C of the next MFMA on the same registers needs no wait states);
// the epilogue's first read follows a 12-state s_nop.
__device__ __forceinline__ void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }

__global__ __launch_bounds__(256, 1) void gemm4w_kernel(const void* __restrict__ A, const void* __restrict__ B,
                                                        void* __restrict__ C, int M, int N, int K, int64_t lda,
                                                        int64_t ldb, int64_t ldc, int nbm, int nbn) {
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  tile_of_block(blockIdx.x, nbm, nbn, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const __amdgpu_buffer_rsrc_t ra = rsrc((const char*)A + (int64_t)m0 * lda * 2, (uint64_t)(M - m0) * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc((const char*)B + (int64_t)n0 * ldb * 2, (uint64_t)(N - n0) * ldb * 2);
  // Sub-step image: 32 pieces of 1 KB (one wave-instruction each): pieces 0..15 = A rows 16p..16p+15,
  // 16..31 = B rows.  Waves 0, 1 load A, waves 2, 3 load B, 8 pieces each (q = 0..7).  Lane ->
  // row 16*piece + lane/4, phys chunk lane & 3, logical chunk lc = (lane & 3) ^ ((lane >> 4) & 3)
  // (= phys ^ ((row >> 2) & 3), the same for every piece).  (Experiment: M, N % 256 == 0, K % 32 == 0.)
  const bool loadsA = wave < 2;
  const int64_t ld = loadsA ? lda : ldb;
  const int row0 = (wave & 1) * 128 + (lane >> 2);
  const uint32_t voff0 = (uint32_t)((int64_t)row0 * ld * 2 + (((lane & 3) ^ ((lane >> 4) & 3)) << 4));
  const uint32_t vstep = (uint32_t)(16 * ld * 2);
  const __amdgpu_buffer_rsrc_t rl = loadsA ? ra : rb;
  char* const dst0 = smem + (loadsA ? 0 : 256 * 64) + (wave & 1) * 8 * 1024;
  const int nk = K / 32;
  auto issue = [&](int s) {  // DMAs of sub-step s into stage s % NST (past the end: zero-fill)
    char* dst = dst0 + (s % NST) * STAGE;
    const uint32_t kb = (uint32_t)(s * 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t off = s < nk ? voff0 + q * vstep + kb : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_void*)(dst + q * 1024), 16, (int)off, 0, 0, 0);
    }
  };
  // fragment lane offset within a 16-row group: row (lane & 15), logical chunk lane >> 4
  const int r16 = lane & 15;
  const int foff = r16 * 64 + (((lane >> 4) ^ ((r16 >> 2) & 3)) << 4);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // B fragments double-buffered in registers (Bf[cur] for this sub-step, Bf[nxt] filled for the next
  // one), A fragments streamed one row group ahead (Af[i & 1])
  bf16x8 Bf[2][8], Af[4];
  auto frag = [&](int s, int f) {  // f 0..7: A row group f; 8..15: B column group f - 8
    const char* st = smem + (s % NST) * STAGE;
    const char* base = f < 8 ? st + wr * 128 * 64 + f * 16 * 64 : st + 256 * 64 + wc * 128 * 64 + (f - 8) * 16 * 64;
    return *(const bf16x8*)(base + foff);
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s);
  wait_vmcnt<8 * (NST - 2)>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) Bf[0][j] = frag(0, 8 + j);
  Af[0] = frag(0, 0);
  Af[1] = frag(0, 1);

  // sub-step s: row group i = MFMAs A_i x B_0..7, then the reads of A_{i+2} (stage s, or s + 1 past row 5) and
  // B_i (stage s + 1).  Stage s is read during sub-steps s - 1 (B, A row 0) and s (A rows 1..7).  After row 0
  // the barrier: stage s + 1 landed everywhere (RAW for the B reads that follow), and every wave is
  // past sub-step s - 1, the last reader of stage s - 1, which takes the DMAs of sub-step s + NST - 1
  // (WAR).  Prefetch distance NST - 2 sub-steps.
  auto substep = [&](auto cur_c, int s) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
    char* dst = dst0 + ((s + NST - 1) % NST) * STAGE;
    const uint32_t kb = (uint32_t)((s + NST - 1) * 64);
    const bool live = s + NST - 1 < nk;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bf16x8 a = Af[i & 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#ifdef G4_ASM_MFMA
        mfma_a(acc[i][j], Bf[cur][j], a);
#else
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Bf[cur][j], a, acc[i][j], 0, 0, 0);
#endif
        __builtin_amdgcn_sched_barrier(0);
        // the 8 DMAs of sub-step s + NST - 1 spread one per row group (two in row 1) after the
        // barrier: an LDS-DMA piece costs ~60 issue cycles, hidden only behind ~4 queued MFMAs
        if (i >= 1 && (j == 3 || (i == 1 && j == 7))) {
          const int q = (i == 1 && j == 7) ? 0 : i;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_void*)(dst + q * 1024), 16,
                                                   (int)(live ? voff0 + q * vstep + kb : OOB), 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
        // the fragment reads: A two row groups ahead after MFMA 2, B of s + 1 after MFMA 5
        if (j == 2) {
          Af[(i + 2) & 3] = i < 6 ? frag(s, i + 2) : frag(s + 1, i - 6);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (j == 5 && i >= 1) {
          Bf[nxt][i - 1] = frag(s + 1, 8 + i - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (i == 0) {  // the barrier of sub-step s + 1 (see above)
        wait_vmcnt<8 * (NST - 3)>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    Bf[nxt][7] = frag(s + 1, 15);
    __builtin_amdgcn_sched_barrier(0);
  };
  int s = 0;
  for (; s + 1 < nk; s += 2) {
    substep(std::integral_constant<int, 0>{}, s);
    substep(std::integral_constant<int, 1>{}, s + 1);
  }
  if (s < nk) substep(std::integral_constant<int, 0>{}, s);
  wait_vmcnt<0>();
#ifdef G4_ASM_MFMA
  asm volatile("s_nop 11\n\ts_nop 4" ::: "memory");
#endif
  // epilogue: lane holds row (lane & 15), 4 consecutive columns 4 * (lane >> 4) of each 16 x 16 block
  const __amdgpu_buffer_rsrc_t rc = rsrc((char*)C + ((int64_t)m0 * ldc + n0) * 2,
                                         ((uint64_t)(M - m0 - 1) * ldc + (N - n0)) * 2);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr * 128 + i * 16 + r16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = wc * 128 + j * 16 + 4 * (lane >> 4);
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (short)f2bf(acc[i][j][e]);
      const uint32_t off = (row < M - m0 && col < N - n0) ? (uint32_t)(((int64_t)row * ldc + col) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rc, (int)off, 0, 0);
    }
  }
}
}  // namespace g4

extern "C" int g4_gemm_bf16(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                            int64_t ldb, int64_t ldc, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % 32) || (N % 256) || (M % 256)) return 1;
  const int nbm = (int)((M + 255) / 256), nbn = (int)((N + 255) / 256);
  hipLaunchKernelGGL(g4::gemm4w_kernel, dim3(nbm * nbn), dim3(256), 0, (hipStream_t)stream, A, B, C, (int)M, (int)N,
                     (int)K, lda, ldb, ldc, nbm, nbn);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
