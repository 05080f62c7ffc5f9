// MFMA GEMM for the five contractions of one crosscoder training step, with the step's
// elementwise/reduction work fused into the epilogues.  gfx950 (CDNA4) only.
//
//   G1 encode   acts[B,h]   = relu(x[B,K] . W_enc[h][K]^T + b_enc)   A:KC  B:KC   (crosscoder.py:69-80)
//   G2 decode   recon[B,K]  = acts[B,h] . W_dec[h][K]                A:KC  B:MN   (crosscoder.py:82-89)
//   G3 d_acts   g_pre[B,h]  = (g_recon . W_dec^T + l1 term) * mask   A:KC  B:KC   (autograd of :84-89,126,77)
//   G4 dW_dec   [h][K]      = acts^T . g_recon + norm-grad term      A:MN  B:MN
//   G5 dW_enc   [h][K]      = g_pre^T . x                            A:MN  B:MN
//
// Geometry: 256x256 output tile per 512-thread workgroup (8 waves = 2 per SIMD, 2(M) x 4(N)),
// each wave 128x64 = 8x4 tiles of v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32
// (fp32 mode, exact-f32 MFMA).  K-step: 64 bf16 / 32 fp32 elements = 128 B per KC row, so
// every operand tile is 32 KB; two stages (A+B) = 128 KB of the CU's 160 KB LDS.
// Staging is LDS-DMA (buffer_load ... lds, 16 B per lane) through a buffer descriptor whose
// range check zero-fills out-of-range lanes (M/N/K tails: the offset is pushed past the
// descriptor's record count).  The LDS image is lane-linear per 1 KB wave-instruction, so the
// bank-conflict swizzle lives in the per-lane SOURCE address and the matching read address:
//   KC tile  [256 rows][8 x 16 B chunks]:   phys chunk = chunk ^ (row & 7)        (ds_read_b128)
//   MN tile  [k rows][rows/8 x 16 B chunks]: phys chunk = chunk ^ f(k)            (ds_read_b64_tr_b16)
// One s_barrier per K-step: wait own DMA (vmcnt 0) -> barrier -> issue DMA of step t+1 into the
// other stage -> MFMA on stage t.  All LDS is one __shared__ array (no vmcnt(0) before ds_read).
#include "cc_common.h"

namespace cc {

constexpr int BM = 256, BN = 256, NTHR = 512;
constexpr int TILE_BYTES = 256 * 128;           // one operand tile per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;     // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 128 KB
constexpr uint32_t OOB = 0x7ffffff0u;           // voffset that the range check always rejects
constexpr uint32_t MAX_RECORDS = 0x7fffffe0u;

enum Epi { EPI_F32 = 0, EPI_ENC = 1, EPI_DEC = 2, EPI_DACTS = 3, EPI_WGDEC = 4, EPI_WGENC = 5 };

struct GemmArgs {
  const void* A;
  const void* B;
  int64_t lda, ldb;
  int M, N, K;
  int nbm, nbn;
  void* out;            // primary output (dtype), or fp32 for EPI_F32
  int64_t ldo;
  float* out_f32;       // EPI_DEC fp32 output
  const void* bias;     // b_enc / b_dec, indexed by column
  const float* tn;      // per-column total decoder norm
  const void* mask_src; // acts (EPI_DACTS), indexed like out
  const void* w_src;    // W_dec (EPI_WGDEC), indexed like out
  const float* norms;   // [h][n]
  const float* colsum;  // [h] sum_b acts
  float* col_part;      // [2*nbm][N]
  float* wave_part0;    // [nbm*nbn*8]
  float* wave_part1;
  float scale0;
  int flag;             // apply_relu
  int d_model, n_models;
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

CC_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  uint32_t nrec = bytes > MAX_RECORDS ? MAX_RECORDS : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec, 0x00020000);
}

CC_DEV void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_base, 16, (int)voff, 0, 0, 0);
}

// MN-tile swizzle (16-B chunk index XOR, depends on the k row); conflict-free for the
// ds_read_b64_tr_b16 fragment reads of the 16x16x32 operands (bf16), and for the fp32
// ds_read_b32 reads (toggles 64 B by k row bit 2).
CC_DEV int mn_swz_bf16(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }
CC_DEV int mn_swz_f32(int k) { return ((k >> 2) & 1) << 2; }

// ---- global -> LDS staging of one operand tile (4 x 1 KB DMA per thread) ----
// KC: tile rows = the operand's M (or N) rows [row0, row0+256), 128 B of contraction each.
template <int DT>
CC_DEV void stage_kc(__amdgpu_buffer_rsrc_t r, char* lds, int rows_left, int k0, int K, int64_t ld, int wave,
                     int lane) {
  constexpr int EPC = DT == CC_BF16 ? 8 : 4;  // elements per 16-B chunk
  constexpr int ES = DT == CC_BF16 ? 2 : 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int ci = i * 8 + wave;
    int row = ci * 8 + (lane >> 3);
    int c = (lane & 7) ^ (row & 7);
    int k = k0 + c * EPC;
    bool ok = row < rows_left && k < K;
    uint32_t voff = ok ? (uint32_t)(((int64_t)row * ld + k) * ES) : OOB;
    dma16(r, lds + ci * 1024, voff);
  }
}
// MN: tile = contraction rows [k0, k0+BK) x 256 contiguous columns [col0, col0+256).
template <int DT>
CC_DEV void stage_mn(__amdgpu_buffer_rsrc_t r, char* lds, int cols_left, int k0, int K, int64_t ld, int wave,
                     int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int ci = i * 8 + wave;
    int k, q, col;
    if constexpr (DT == CC_BF16) {  // 1 KB = 2 k rows of 512 B
      k = ci * 2 + (lane >> 5);
      q = (lane & 31) ^ mn_swz_bf16(k);
      col = q * 8;
    } else {  // 1 KB = 1 k row of 256 fp32
      k = ci;
      q = lane ^ mn_swz_f32(k);
      col = q * 4;
    }
    constexpr int ES = DT == CC_BF16 ? 2 : 4;
    bool ok = (k0 + k) < K && col < cols_left;
    uint32_t voff = ok ? (uint32_t)(((int64_t)(k0 + k) * ld + col) * ES) : OOB;
    dma16(r, lds + ci * 1024, voff);
  }
}

// ---- fragment reads (bf16, v_mfma_f32_16x16x32_bf16 operand maps) ----
// lane l holds X[row = l&15][k = 8*(l>>4) + j], j = 0..7, for the 16-row tile at `row0`,
// k half `kk` (k 0..31 or 32..63 of the step).
CC_DEV bf16x8 frag_kc_bf16(const char* tile, int row0, int kk, int lane) {
  int row = row0 + (lane & 15);
  int c = (lane >> 4) + 4 * kk;
  int off = row * 128 + ((c ^ (row & 7)) << 4);
  return *(const bf16x8*)(tile + off);
}
CC_DEV bf16x8 frag_mn_bf16(const char* tile, int col0, int kk, int lane) {
  int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
  int col = col0 + 4 * pp;
  bf16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    int k = 32 * kk + 8 * g + 4 * t + qq;
    int off = k * 512 + ((((col >> 3) ^ mn_swz_bf16(k))) << 4) + 8 * (pp & 1);
    bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + off));
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * t + e] = v[e];
  }
  return out;
}
// ---- fragment reads (fp32, v_mfma_f32_16x16x4_f32: lane holds X[l&15][k = l>>4]) ----
// The 32-k step is consumed as 8 MFMAs (kk = 0..1, e = 0..3); lane group g = l>>4 supplies
// k = 4*(g + 4*kk) + e, the same mapping on both operands.
CC_DEV f32x4 frag_kc_f32(const char* tile, int row0, int kk, int lane) {
  int row = row0 + (lane & 15);
  int c = (lane >> 4) + 4 * kk;
  int off = row * 128 + ((c ^ (row & 7)) << 4);
  return *(const f32x4*)(tile + off);
}
CC_DEV f32x4 frag_mn_f32(const char* tile, int col0, int kk, int lane) {
  int g = lane >> 4;
  int col = col0 + (lane & 15);
  f32x4 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int k = 4 * (g + 4 * kk) + e;
    int off = k * 1024 + ((((col >> 2) ^ mn_swz_f32(k))) << 4) + 4 * (col & 3);
    out[e] = *(const float*)(tile + off);
  }
  return out;
}

// Bijective XCD-aware block remap (blocks b and b+8 share an XCD: give each XCD a contiguous
// range of tile ids), then grouped tile order (GM tile rows per group) for L2 reuse.
CC_DEV void tile_of_block(int bid, int nbm, int nbn, int& tm, int& tn) {
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

template <int DT, bool AKC, bool BKC, int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(const GemmArgs args) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  using E = Elem<DT>;
  using T = typename E::T;
  constexpr int BK = DT == CC_BF16 ? 64 : 32;
  constexpr int ES = DT == CC_BF16 ? 2 : 4;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int tm, tn;
  tile_of_block(blockIdx.x, args.nbm, args.nbn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int M = args.M, N = args.N, K = args.K;

  // descriptors based at the block's panel; offsets stay < 2^31 for every supported shape
  __amdgpu_buffer_rsrc_t ra, rb;
  {
    const char* a = (const char*)args.A;
    const char* b = (const char*)args.B;
    if constexpr (AKC) {
      a += (int64_t)m0 * args.lda * ES;
      ra = make_rsrc(a, (uint64_t)(M - m0) * args.lda * ES);
    } else {
      a += (int64_t)m0 * ES;
      ra = make_rsrc(a, ((uint64_t)(K - 1) * args.lda + (M - m0)) * ES);
    }
    if constexpr (BKC) {
      b += (int64_t)n0 * args.ldb * ES;
      rb = make_rsrc(b, (uint64_t)(N - n0) * args.ldb * ES);
    } else {
      b += (int64_t)n0 * ES;
      rb = make_rsrc(b, ((uint64_t)(K - 1) * args.ldb + (N - n0)) * ES);
    }
  }

  auto stage = [&](int kt, int s) {
    char* la = smem + s * STAGE_BYTES;
    char* lb = la + TILE_BYTES;
    int k0 = kt * BK;
    if constexpr (AKC) stage_kc<DT>(ra, la, M - m0, k0, K, args.lda, wave, lane);
    else stage_mn<DT>(ra, la, M - m0, k0, K, args.lda, wave, lane);
    if constexpr (BKC) stage_kc<DT>(rb, lb, N - n0, k0, K, args.ldb, wave, lane);
    else stage_mn<DT>(rb, lb, N - n0, k0, K, args.ldb, wave, lane);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const char* la = smem + (kt & 1) * STAGE_BYTES;
    const char* lb = la + TILE_BYTES;
    if constexpr (DT == CC_BF16) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a[8], b[4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          a[i] = AKC ? frag_kc_bf16(la, wr * 128 + i * 16, kk, lane) : frag_mn_bf16(la, wr * 128 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b[j] = BKC ? frag_kc_bf16(lb, wc * 64 + j * 16, kk, lane) : frag_mn_bf16(lb, wc * 64 + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        f32x4 a[8], b[4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          a[i] = AKC ? frag_kc_f32(la, wr * 128 + i * 16, kk, lane) : frag_mn_f32(la, wr * 128 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b[j] = BKC ? frag_kc_f32(lb, wc * 64 + j * 16, kk, lane) : frag_mn_f32(lb, wc * 64 + j * 16, kk, lane);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
      }
    }
  }

  // ------------------------------- epilogue (C-fragment layout) ------------------------------
  // acc[i][j][e] = C[row = m0 + wr*128 + i*16 + 4*(lane>>4) + e][col = n0 + wc*64 + j*16 + (lane&15)]
  const int rbase = m0 + wr * 128 + 4 * (lane >> 4);
  const int cbase = n0 + wc * 64 + (lane & 15);
  const int wave_slot = blockIdx.x * 8 + wave;

  if constexpr (EPI == EPI_F32) {
    float* C = (float*)args.out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int col = cbase + j * 16;
      if (col >= N) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int row = rbase + i * 16 + e;
          if (row < M) C[(int64_t)row * args.ldo + col] = acc[i][j][e];
        }
    }
  } else if constexpr (EPI == EPI_DEC) {
    const T* bias = (const T*)args.bias;
    T* out = (T*)args.out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int col = cbase + j * 16;
      if (col >= N) continue;
      float bc = bias ? E::to_f(bias[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int row = rbase + i * 16 + e;
          if (row >= M) continue;
          float v = acc[i][j][e] + bc;
          int64_t o = (int64_t)row * args.ldo + col;
          if (args.out_f32) args.out_f32[o] = v;
          if (out) out[o] = E::from_f(v);
        }
    }
  } else if constexpr (EPI == EPI_ENC || EPI == EPI_DACTS) {
    const T* bias = (const T*)args.bias;
    const T* mask = (const T*)args.mask_src;
    T* out = (T*)args.out;
    float s_l1 = 0.f, s_l0 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int col = cbase + j * 16;
      bool cv = col < N;
      float csum = 0.f;
      float add = 0.f, tnc = 0.f;
      if (cv) {
        if constexpr (EPI == EPI_ENC) {
          add = bias ? E::to_f(bias[col]) : 0.f;
          tnc = args.tn ? args.tn[col] : 0.f;
        } else {
          add = args.tn ? args.scale0 * args.tn[col] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int row = rbase + i * 16 + e;
          if (!cv || row >= M) continue;
          int64_t o = (int64_t)row * args.ldo + col;
          float v = acc[i][j][e] + add;
          if constexpr (EPI == EPI_ENC) {
            if (args.flag) v = fmaxf(v, 0.f);
          } else {
            v = E::to_f(mask[o]) > 0.f ? v : 0.f;
          }
          T q = E::from_f(v);
          out[o] = q;
          float vq = E::to_f(q);
          csum += vq;
          if constexpr (EPI == EPI_ENC) {
            s_l1 += vq * tnc;
            s_l0 += vq > 0.f ? 1.f : 0.f;
          }
        }
      if (args.col_part) {
        csum += __shfl_xor(csum, 16, 64);
        csum += __shfl_xor(csum, 32, 64);
        if (lane < 16 && cv) args.col_part[(int64_t)(2 * tm + wr) * N + col] = csum;
      }
    }
    if constexpr (EPI == EPI_ENC) {
      if (args.wave_part0) {
        float t = wave_sum(s_l1);
        if (lane == 0) args.wave_part0[wave_slot] = t;
      }
      if (args.wave_part1) {
        float t = wave_sum(s_l0);
        if (lane == 0) args.wave_part1[wave_slot] = t;
      }
    }
  } else if constexpr (EPI == EPI_WGDEC || EPI == EPI_WGENC) {
    T* out = (T*)args.out;
    const T* w = (const T*)args.w_src;
    float sq = 0.f;
    const bool l1term = EPI == EPI_WGDEC && args.scale0 != 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int row = rbase + i * 16 + e;
        if (row >= M) continue;
        float cs = l1term ? args.scale0 * args.colsum[row] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int col = cbase + j * 16;
          if (col >= N) continue;
          int64_t o = (int64_t)row * args.ldo + col;
          float v = acc[i][j][e];
          if (l1term) {
            float nrm = args.norms[(int64_t)row * args.n_models + col / args.d_model];
            v += nrm > 0.f ? cs * E::to_f(w[o]) / nrm : 0.f;
          }
          T q = E::from_f(v);
          out[o] = q;
          float vq = E::to_f(q);
          sq += vq * vq;
        }
      }
    if (args.wave_part0) {
      float t = wave_sum(sq);
      if (lane == 0) args.wave_part0[wave_slot] = t;
    }
  }
}

template <int DT, bool AKC, bool BKC, int EPI>
static int launch(GemmArgs a, hipStream_t st) {
  a.nbm = (a.M + BM - 1) / BM;
  a.nbn = (a.N + BN - 1) / BN;
  dim3 grid(a.nbm * a.nbn), block(NTHR);
  hipLaunchKernelGGL((gemm_kernel<DT, AKC, BKC, EPI>), grid, block, 0, st, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

template <int EPI, bool AKC, bool BKC>
static int launch_dt(int dtype, GemmArgs a, hipStream_t st) {
  if (dtype == CC_BF16) return launch<CC_BF16, AKC, BKC, EPI>(a, st);
  if (dtype == CC_F32) return launch<CC_F32, AKC, BKC, EPI>(a, st);
  return CC_ERR_DTYPE;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Shape / alignment validation shared by all GEMM entries.
static int check_gemm(const GemmArgs& a, int dtype, bool akc, bool bkc) {
  if (!a.A || !a.B) return CC_ERR_NULL;
  if (dtype != CC_BF16 && dtype != CC_F32) return CC_ERR_DTYPE;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return CC_ERR_SHAPE;
  int epc = dtype == CC_BF16 ? 8 : 4;
  // vector (16 B) granularity: contiguous dims and leading dims
  if (akc && (a.K % epc)) return CC_ERR_SHAPE;
  if (!akc && (a.M % epc)) return CC_ERR_SHAPE;
  if (bkc && (a.K % epc)) return CC_ERR_SHAPE;
  if (!bkc && (a.N % epc)) return CC_ERR_SHAPE;
  if ((a.lda % epc) || (a.ldb % epc)) return CC_ERR_ALIGN;
  if (!al16(a.A) || !al16(a.B)) return CC_ERR_ALIGN;
  int es = dtype == CC_BF16 ? 2 : 4;
  // per-block descriptor ranges must fit the 31-bit offsets
  uint64_t ra = akc ? (uint64_t)BM * a.lda * es : (uint64_t)a.K * a.lda * es;
  uint64_t rb = bkc ? (uint64_t)BN * a.ldb * es : (uint64_t)a.K * a.ldb * es;
  if (ra >= MAX_RECORDS || rb >= MAX_RECORDS) return CC_ERR_TOO_LARGE;
  return CC_OK;
}

}  // namespace cc

using namespace cc;

extern "C" {

int64_t cc_col_part_rows(int64_t M) { return 2 * ((M + BM - 1) / BM); }
int64_t cc_wave_parts(int64_t M, int64_t N) { return 8 * ((M + BM - 1) / BM) * ((N + BN - 1) / BN); }

int cc_gemm_f32out(const void* A, int a_layout, int64_t lda, const void* Bm, int b_layout, int64_t ldb, float* C,
                   int64_t ldc, int64_t M, int64_t N, int64_t K, int dtype, void* stream) {
  GemmArgs a = {};
  a.A = A; a.B = Bm; a.lda = lda; a.ldb = ldb; a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.out = C; a.ldo = ldc;
  if (!C) return CC_ERR_NULL;
  bool akc = a_layout == CC_LAYOUT_KC, bkc = b_layout == CC_LAYOUT_KC;
  int rc = check_gemm(a, dtype, akc, bkc);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (akc && bkc) return launch_dt<EPI_F32, true, true>(dtype, a, st);
  if (akc && !bkc) return launch_dt<EPI_F32, true, false>(dtype, a, st);
  if (!akc && bkc) return launch_dt<EPI_F32, false, true>(dtype, a, st);
  return launch_dt<EPI_F32, false, false>(dtype, a, st);
}

int cc_encode_fwd(const void* x, const void* W_enc, const void* b_enc, const float* tn, void* acts, int apply_relu,
                  float* colsum_part, float* l1_part, float* l0_part, int64_t B, int64_t K, int64_t h, int dtype,
                  void* stream) {
  if (!acts) return CC_ERR_NULL;
  if (l1_part && !tn) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = x; a.lda = K; a.B = W_enc; a.ldb = K;
  a.M = (int)B; a.N = (int)h; a.K = (int)K;
  a.out = acts; a.ldo = h; a.bias = b_enc; a.tn = tn; a.flag = apply_relu;
  a.col_part = colsum_part; a.wave_part0 = l1_part; a.wave_part1 = l0_part;
  int rc = check_gemm(a, dtype, true, true);
  if (rc) return rc;
  return launch_dt<EPI_ENC, true, true>(dtype, a, (hipStream_t)stream);
}

int cc_decode_fwd(const void* acts, const void* W_dec, const void* b_dec, float* recon_f32, void* recon_t, int64_t B,
                  int64_t h, int64_t K, int dtype, void* stream) {
  if (!recon_f32 && !recon_t) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = acts; a.lda = h; a.B = W_dec; a.ldb = K;
  a.M = (int)B; a.N = (int)K; a.K = (int)h;
  a.out = recon_t; a.out_f32 = recon_f32; a.ldo = K; a.bias = b_dec;
  int rc = check_gemm(a, dtype, true, false);
  if (rc) return rc;
  return launch_dt<EPI_DEC, true, false>(dtype, a, (hipStream_t)stream);
}

int cc_dacts_bwd(const void* g_recon, const void* W_dec, const void* acts, const float* tn, float l1_scale,
                 void* g_pre, float* colsum_part, int64_t B, int64_t K, int64_t h, int dtype, void* stream) {
  if (!g_pre || !acts) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = g_recon; a.lda = K; a.B = W_dec; a.ldb = K;
  a.M = (int)B; a.N = (int)h; a.K = (int)K;
  a.out = g_pre; a.ldo = h; a.mask_src = acts; a.tn = tn; a.scale0 = l1_scale;
  a.col_part = colsum_part;
  int rc = check_gemm(a, dtype, true, true);
  if (rc) return rc;
  return launch_dt<EPI_DACTS, true, true>(dtype, a, (hipStream_t)stream);
}

int cc_wgrad_dec(const void* acts, const void* g_recon, const void* W_dec, const float* norms, const float* colsum_acts,
                 float l1_scale, void* grad_W_dec, float* sq_part, int64_t B, int64_t h, int64_t n, int64_t d, int dtype,
                 void* stream) {
  if (!grad_W_dec) return CC_ERR_NULL;
  if (l1_scale != 0.f && (!W_dec || !norms || !colsum_acts)) return CC_ERR_NULL;
  GemmArgs a = {};
  int64_t K = n * d;
  a.A = acts; a.lda = h; a.B = g_recon; a.ldb = K;
  a.M = (int)h; a.N = (int)K; a.K = (int)B;
  a.out = grad_W_dec; a.ldo = K; a.w_src = W_dec; a.norms = norms; a.colsum = colsum_acts;
  a.scale0 = l1_scale; a.wave_part0 = sq_part; a.d_model = (int)d; a.n_models = (int)n;
  int rc = check_gemm(a, dtype, false, false);
  if (rc) return rc;
  return launch_dt<EPI_WGDEC, false, false>(dtype, a, (hipStream_t)stream);
}

int cc_wgrad_enc(const void* g_pre, const void* x, void* grad_W_enc, float* sq_part, int64_t B, int64_t h, int64_t K,
                 int dtype, void* stream) {
  if (!grad_W_enc) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = g_pre; a.lda = h; a.B = x; a.ldb = K;
  a.M = (int)h; a.N = (int)K; a.K = (int)B;
  a.out = grad_W_enc; a.ldo = K; a.wave_part0 = sq_part;
  int rc = check_gemm(a, dtype, false, false);
  if (rc) return rc;
  return launch_dt<EPI_WGENC, false, false>(dtype, a, (hipStream_t)stream);
}

}  // extern "C"
