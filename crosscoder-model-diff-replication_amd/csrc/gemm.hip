// MFMA GEMM for the five contractions of one crosscoder training step, with the step's
// elementwise/reduction work fused into the epilogues.  gfx950 (CDNA4) only.
//
//   G1 encode   acts[B,h]   = relu(x[B,K] . W_enc[h][K]^T + b_enc)   A:KC  B:KC   (crosscoder.py:69-80)
//   G2 decode   recon[B,K]  = acts[B,h] . W_dec[h][K]                A:KC  B:MN   (crosscoder.py:82-89)
//   G3 d_acts   g_pre[B,h]  = (g_recon . W_dec^T + l1 term) * mask   A:KC  B:KC   (autograd of :84-89,126,77)
//   G4 dW_dec   [h][K]      = acts^T . g_recon + norm-grad term      A:MN  B:MN
//   G5 dW_enc   [h][K]      = g_pre^T . x                            A:MN  B:MN
//
// Geometry: 512-thread workgroups (8 waves = 2 per SIMD), output tile 256 x BN with
//   BN = 256: waves 2(M) x 4(N), 128 x 64 per wave (8 x 4 MFMA tiles)
//   BN = 288: waves 4(M) x 2(N),  64 x 144 per wave (4 x 9 MFMA tiles) -- used when N = n*d is a
//             multiple of 288 (n*2304 at the Gemma-2-2b width): 4096 x 4608 -> exactly 256 tiles.
// MFMA: v_mfma_f32_16x16x32_bf16 (bf16) / v_mfma_f32_16x16x4_f32 (fp32 mode, exact f32), issued
// with the operands swapped (B fragment as src A) so each lane's 4 accumulator registers are 4
// CONSECUTIVE output columns of one row: 8-16 B vector epilogue loads/stores.
// K-step: 64 bf16 / 32 fp32 elements = 128 B per KC row.  Two LDS stages (A+B).
// Staging is LDS-DMA (buffer_load ... lds, 16 B per lane) through buffer descriptors whose range
// check zero-fills out-of-range lanes (M/N/K tails: the offset is pushed past the record count).
// The LDS image is lane-linear per 1 KB wave-instruction, so the bank-conflict swizzle lives in
// the per-lane SOURCE address and the matching read address:
//   KC tile [rows][8 x 16 B]:   phys chunk = chunk ^ (row & 7)                  (ds_read_b128)
//   MN tile [k][cols]:          phys chunk = (chunk + rot(k)) mod chunks/row      (ds_read_b64_tr_b16
//                               bf16 / ds_read_b32 fp32), rot chosen conflict-free per geometry.
// One s_barrier per K-step: wait own DMA (vmcnt 0) -> barrier -> issue DMA of step t+1 into the
// other stage -> MFMA on stage t.  All LDS is one __shared__ array.
#include <mutex>

#include <hip/hip_ext.h>

#include "cc_common.h"

namespace cc {

#include "grad_tail.h"
#include "loss_tail.h"

constexpr int BM = 256, NTHR = 512;
constexpr uint32_t OOB = 0x7ffffff0u;  // voffset that the range check always rejects
constexpr uint32_t MAX_RECORDS = 0x7fffffe0u;

enum Epi { EPI_F32 = 0, EPI_ENC = 1, EPI_DEC = 2, EPI_DACTS = 3, EPI_WGDEC = 4, EPI_WGENC = 5, EPI_SPLIT = 6, EPI_DLOSS = 7 };

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
  const float* norms;   // [h][n] inverse decoder norms (0 where the norm is 0)
  const float* colsum;  // [h] sum_b acts
  float* col_part;      // [nbm * WARPS_M][N]
  float* wave_part0;    // [nbm*nbn*8]
  float* wave_part1;
  float scale0;
  int flag;             // apply_relu
  int d_model, n_models;
  int k_step0, k_steps; // ping-pong split-K: contraction steps [k_step0, k_step0 + k_steps) (0 steps: all)
  void* out_t;          // ping-pong bf16 epilogue: also store the tile transposed, out_t[n][m] (ld ldt)
  int64_t ldt;
  float* row_part;      // EPI_DLOSS: loss row terms [2][n * d/64][M]
  uint32_t* mask_bits;  // ping-pong EPI_ENC (out) / EPI_DACTS FAST (in): the activation mask, 1 bit per output
                        // in accumulator order: [tile tm*nbn + tn][thread][4] u32, bit 4(4i+j)+e of fragment (i,j)
  uint32_t* tile_ctr;   // persistent ping-pong launches: 8 per-XCD tile counters (dynamic order), NULL: static
  uint32_t* wave_sync;  // probe only: 8 zeroed per-XCD arrival words (TileLoop::wave_wait), NULL: off
  uint64_t* stamps;     // probe build only (-DCC_PP_STAMPS): [tile][12] clock stamps of a ping-pong tile (pp_tile)
  // wait in the kernel for a producer on another stream (cc_decode_loss: the side-stream Adam's done counter,
  // AdamArgs::done_ctr) before the first operand load: until *wait_ctr - wait_target >= 0 (mod 2^32); a wait
  // past ~1 s gives up, sets *wait_err (host-visible) and runs on (NULL wait_ctr: none)
  const uint32_t* wait_ctr;
  uint32_t wait_target;
  uint32_t* wait_err;
  RedSeg pre;           // a column reduction the launch runs before its tiles (cc_colsum_job), pre_blocks > 0
  int pre_blocks;
  LossTailArgs tail;    // the forward's loss tail the launch runs before its tiles (cc_loss_tail_job), tail_items > 0
  int tail_items;
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

// ---- Pipeline geometry.  KROW = bytes of contraction per KC row per K-step (64 or 128);
// BK = KROW / element size; NST = LDS stages (prefetch distance NST-1 K-steps).
// MN tile: [BK k rows][COLS columns], row bytes RB, CH 16-B chunks per row.
template <int DT, int COLS, int KROW>
struct MnTile {
  static constexpr int ES = DT == CC_BF16 ? 2 : 4;
  static constexpr int EPC = 16 / ES;                 // elements per chunk
  static constexpr int BK = KROW / ES;
  static constexpr int RB = COLS * ES;
  static constexpr int CH = RB / 16;
  static constexpr int BYTES = BK * RB;
  static constexpr int NDMA = BYTES / 1024;
  // chunk rotation per k row: conflict-free fragment reads (checked exhaustively offline for
  // the 16x16x32 bf16 / 16x16x4 f32 read patterns of both column counts)
  static CC_DEV int rot(int k) {
    if constexpr (DT == CC_BF16) {
      if constexpr (COLS == 256) return 2 * ((k & 3) | ((k >> 1) & 4));
      else return 2 * ((k >> 3) & 1);
    } else {
      return 4 * ((k >> 2) & 1);
    }
  }
};
// KC tile: [ROWS][KROW bytes]; phys chunk = chunk ^ swz(row), conflict-free for ds_read_b128
template <int KROW>
struct KcTile {
  static constexpr int CPR = KROW / 16;     // chunks per row
  static constexpr int RPD = 1024 / KROW;   // rows per 1 KB DMA
  static CC_DEV int swz(int row) { return KROW == 128 ? (row & 7) : ((row >> 1) & 3); }
};

// ---- global -> LDS staging: the q-th 1 KB DMA of this wave for one operand tile ----
// KC: tile rows [row0, row0+ROWS), KROW bytes of contraction each.
template <int DT, int ROWS, int KROW>
CC_DEV void dma_kc(__amdgpu_buffer_rsrc_t r, char* lds, char* junk, int q, bool live, int rows_left, int k0, int K,
                   int64_t ld, int wave, int lane) {
  using T = KcTile<KROW>;
  constexpr int EPC = DT == CC_BF16 ? 8 : 4;
  constexpr int ES = DT == CC_BF16 ? 2 : 4;
  constexpr int NDMA = ROWS * KROW / 1024;
  const int ci = q * 8 + wave;
  // branch-free: a DMA beyond the tile (or of a step past the end) lands in the junk slot,
  // so every wave issues the same count every step (uniform counted vmcnt)
  const bool use = live && (NDMA % 8 == 0 || ci < NDMA);
  const int row = ci * T::RPD + lane / T::CPR;
  const int c = (lane % T::CPR) ^ T::swz(row);
  const int k = k0 + c * EPC;
  const bool ok = use && row < rows_left && k < K;
  const uint32_t voff = ok ? (uint32_t)(((int64_t)row * ld + k) * ES) : OOB;
  dma16(r, use ? lds + ci * 1024 : junk, voff);
}
// MN: contraction rows [k0, k0+BK) x COLS contiguous columns, lane-linear image.
template <int DT, int COLS, int KROW>
CC_DEV void dma_mn(__amdgpu_buffer_rsrc_t r, char* lds, char* junk, int q, bool live, int cols_left, int k0, int K,
                   int64_t ld, int wave, int lane) {
  using G = MnTile<DT, COLS, KROW>;
  const int ci = q * 8 + wave;
  const bool use = live && (G::NDMA % 8 == 0 || ci < G::NDMA);
  const int b = ci * 1024 + lane * 16;
  const int k = b / G::RB;
  const int cph = (b - k * G::RB) >> 4;
  int clog = cph - G::rot(k);
  clog += clog < 0 ? G::CH : 0;
  const int col = clog * G::EPC;
  const bool ok = use && (k0 + k) < K && col < cols_left;
  const uint32_t voff = ok ? (uint32_t)(((int64_t)(k0 + k) * ld + col) * G::ES) : OOB;
  dma16(r, use ? lds + ci * 1024 : junk, voff);
}

// Step-invariant part of the q-th DMA's per-lane source offset (bytes from the panel origin at
// k0 = 0), or OOB; the step adds k0 through the scalar soffset (k0*ES for KC, k0*ld*ES for MN),
// so the steady-state K loop spends no VALU on DMA addressing.  Valid when the whole K step is
// in range (k0 + BK <= K); the K-tail step uses dma_kc / dma_mn.
template <int DT, int ROWS, int KROW>
CC_DEV uint32_t dma_kc_base(int q, int rows_left, int64_t ld, int wave, int lane) {
  using T = KcTile<KROW>;
  constexpr int EPC = DT == CC_BF16 ? 8 : 4;
  constexpr int ES = DT == CC_BF16 ? 2 : 4;
  constexpr int NDMA = ROWS * KROW / 1024;
  const int ci = q * 8 + wave;
  const int row = ci * T::RPD + lane / T::CPR;
  const int c = (lane % T::CPR) ^ T::swz(row);
  const bool ok = (NDMA % 8 == 0 || ci < NDMA) && row < rows_left;
  return ok ? (uint32_t)(((int64_t)row * ld + c * EPC) * ES) : OOB;
}
template <int DT, int COLS, int KROW>
CC_DEV uint32_t dma_mn_base(int q, int cols_left, int64_t ld, int wave, int lane) {
  using G = MnTile<DT, COLS, KROW>;
  const int ci = q * 8 + wave;
  const int b = ci * 1024 + lane * 16;
  const int k = b / G::RB;
  const int cph = (b - k * G::RB) >> 4;
  int clog = cph - G::rot(k);
  clog += clog < 0 ? G::CH : 0;
  const int col = clog * G::EPC;
  const bool ok = (G::NDMA % 8 == 0 || ci < G::NDMA) && col < cols_left;
  return ok ? (uint32_t)(((int64_t)k * ld + col) * G::ES) : OOB;
}
CC_DEV void dma16s(__amdgpu_buffer_rsrc_t r, char* lds_base, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_base, 16, (int)voff, (int)soff, 0, 0);
}

// Step-invariant LDS byte offset of a lane's MN fragment read for the 16-column group at col0
// (the k rows 8*(l>>4) + (l&3)... of the slice go to immediates): rot(k) depends only on the
// lane's row-within-slice bits, so the whole address is lane part + compile-time constant.
template <int DT, int COLS, int KROW>
CC_DEV int mn_frag_off(int col0, int lane) {
  using G = MnTile<DT, COLS, KROW>;
  if constexpr (DT == CC_BF16) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
    const int k = 8 * g + qq;  // + 32*kk + 4*t (immediates; rot() is invariant under them)
    int cph = ((col0 + 4 * pp) >> 3) + G::rot(k);
    cph -= cph >= G::CH ? G::CH : 0;
    return k * G::RB + cph * 16 + 8 * (pp & 1);
  } else {
    const int g = lane >> 4;
    const int col = col0 + (lane & 15);
    const int k = 4 * g;  // + 16*kk + e
    int cph = (col >> 2) + G::rot(k);
    cph -= cph >= G::CH ? G::CH : 0;
    return k * G::RB + cph * 16 + 4 * (col & 3);
  }
}
template <int COLS, int KROW>
CC_DEV bf16x8 frag_mn_bf16_at(const char* tile, int off, int kk) {
  using G = MnTile<CC_BF16, COLS, KROW>;
  bf16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + off + (32 * kk + 4 * t) * G::RB));
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * t + e] = v[e];
  }
  return out;
}
template <int COLS, int KROW>
CC_DEV f32x4 frag_mn_f32_at(const char* tile, int off, int kk) {
  using G = MnTile<CC_F32, COLS, KROW>;
  f32x4 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) out[e] = *(const float*)(tile + off + (16 * kk + e) * G::RB);
  return out;
}

// ---- fragment reads, bf16 (16x16x32 operand map: lane l holds X[r = l&15][k = 8*(l>>4) + j]);
// kk selects the 32-k slice of the K-step.
template <int KROW>
CC_DEV bf16x8 frag_kc_bf16(const char* tile, int row0, int kk, int lane) {
  using T = KcTile<KROW>;
  int row = row0 + (lane & 15);
  int c = (lane >> 4) + 4 * kk;
  return *(const bf16x8*)(tile + row * KROW + ((c ^ T::swz(row)) << 4));
}
template <int COLS, int KROW>
CC_DEV bf16x8 frag_mn_bf16(const char* tile, int col0, int kk, int lane) {
  using G = MnTile<CC_BF16, COLS, KROW>;
  int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
  int clog = (col0 + 4 * pp) >> 3;
  bf16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    int k = 32 * kk + 8 * g + 4 * t + qq;
    int cph = clog + G::rot(k);
    cph -= cph >= G::CH ? G::CH : 0;
    bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(tile + k * G::RB + cph * 16 + 8 * (pp & 1)));
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * t + e] = v[e];
  }
  return out;
}
// ---- fragment reads, fp32 (16x16x4: lane holds X[l&15][k = l>>4]); a 16-k slice kk is 4 MFMAs
// (e = 0..3), lane group g = l>>4 supplies k = 4*(g + 4*kk) + e on both operands.
template <int KROW>
CC_DEV f32x4 frag_kc_f32(const char* tile, int row0, int kk, int lane) {
  using T = KcTile<KROW>;
  int row = row0 + (lane & 15);
  int c = (lane >> 4) + 4 * kk;
  return *(const f32x4*)(tile + row * KROW + ((c ^ T::swz(row)) << 4));
}
template <int COLS, int KROW>
CC_DEV f32x4 frag_mn_f32(const char* tile, int col0, int kk, int lane) {
  using G = MnTile<CC_F32, COLS, KROW>;
  int g = lane >> 4;
  int col = col0 + (lane & 15);
  f32x4 out;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int k = 4 * (g + 4 * kk) + e;
    int cph = (col >> 2) + G::rot(k);
    cph -= cph >= G::CH ? G::CH : 0;
    out[e] = *(const float*)(tile + k * G::RB + cph * 16 + 4 * (col & 3));
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

template <int BNT>
struct WaveGeom {
  static constexpr int WARPS_M = BNT == 256 ? 2 : 4;
  static constexpr int WARPS_N = 8 / WARPS_M;
  static constexpr int WTM = BM / WARPS_M;    // wave tile rows
  static constexpr int WTN = BNT / WARPS_N;   // wave tile cols
  static constexpr int TM = WTM / 16, TN = WTN / 16;
};

// bf16x4 / f32x4 vector access of 4 consecutive elements
template <int DT> CC_DEV void ld4(const void* p, int64_t idx, float v[4]) {
  if constexpr (DT == CC_BF16) {
    bf16x4 r = *(const bf16x4*)((const bf16_t*)p + idx);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = bf2f((bf16_t)r[e]);
  } else {
    f32x4 r = *(const f32x4*)((const float*)p + idx);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = r[e];
  }
}
template <int DT> CC_DEV void st4(void* p, int64_t idx, const float v[4]) {
  if constexpr (DT == CC_BF16) {
    bf16x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = (short)f2bf(v[e]);
    *(bf16x4*)((bf16_t*)p + idx) = r;
  } else {
    *(f32x4*)((float*)p + idx) = f32x4{v[0], v[1], v[2], v[3]};
  }
}

// raw 4-element vectors held across an epilogue batch (8 B bf16 / 16 B fp32 per lane)
template <int DT> struct V4;
template <> struct V4<CC_BF16> {
  typedef bf16x4 T;
  static CC_DEV T load(const void* p, int64_t idx) { return *(const bf16x4*)((const bf16_t*)p + idx); }
  static CC_DEV T zero() { return bf16x4{0, 0, 0, 0}; }
  static CC_DEV float get(T v, int e) { return bf2f((bf16_t)v[e]); }
};
template <> struct V4<CC_F32> {
  typedef f32x4 T;
  static CC_DEV T load(const void* p, int64_t idx) { return *(const f32x4*)((const float*)p + idx); }
  static CC_DEV T zero() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
  static CC_DEV float get(T v, int e) { return v[e]; }
};
// epilogue load batch: JB column groups x TM row groups of vectors in flight per batch
template <int DT, int BNT>
struct EPB {
  static constexpr int JB = DT == CC_F32 ? 1 : (WaveGeom<BNT>::TM * WaveGeom<BNT>::TN <= 32 ? WaveGeom<BNT>::TN : 3);
  // W_dec term (vector + per-row factor each): half the batch within 256 VGPRs
  static constexpr int JB_W = DT == CC_F32 ? 1 : (WaveGeom<BNT>::TN == 4 ? 2 : 3);
  // activation mask of d_acts (kept beside the per-fragment output offsets)
  static constexpr int JB_M = DT == CC_F32 ? 1 : (WaveGeom<BNT>::TN == 4 ? 1 : 3);
  static_assert(WaveGeom<BNT>::TN % JB == 0 && WaveGeom<BNT>::TN % JB_W == 0, "batch must divide the column groups");
};

template <int N> CC_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

#include "gemm_epilogue.h"

// The general two-stage kernel (fp32 mode, BN 288, shapes off the ping-pong path): K-step = KROW bytes of
// contraction per KC row, NST LDS stages (prefetch distance 1).
template <int DT, bool AKC, bool BKC, int EPI, int BNT>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(const GemmArgs args) {
  using WG = WaveGeom<BNT>;
  constexpr int KROW = 128, NST = 2;
  constexpr int ES = DT == CC_BF16 ? 2 : 4;
  constexpr int BK = KROW / ES;
  constexpr int KK = KROW / 64;  // 32-element (bf16) / 16-element (fp32) slices per K-step
  constexpr int A_BYTES = AKC ? BM * KROW : MnTile<DT, BM, KROW>::BYTES;
  constexpr int B_BYTES = BKC ? BNT * KROW : MnTile<DT, BNT, KROW>::BYTES;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int DA = (A_BYTES / 1024 + 7) / 8, DB = (B_BYTES / 1024 + 7) / 8;  // DMAs per wave per step
  constexpr int D = DA + DB;
  constexpr bool SPREAD = AKC;
  static_assert(!BKC || BNT == 256, "BN=288 tiles are built for MN-contiguous B only");
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE + 1024];  // + junk DMA target
  char* const junk = smem + NST * STAGE;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WG::WARPS_N, wc = wave % WG::WARPS_N;
  int tm, tn;
  tile_of_block(blockIdx.x, args.nbm, args.nbn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BNT;
  const int M = args.M, N = args.N, K = args.K;

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

  // q-th DMA (0..D-1) of this wave for K-step kt into stage s
  // q-th DMA (0..D-1) of this wave for K-step kt into stage s; steps >= nk go to the junk slot
  uint32_t vo[D];  // step-invariant per-lane DMA source offsets (see dma_kc_base / dma_mn_base)
#pragma unroll
  for (int q = 0; q < D; ++q) {
    if (q < DA)
      vo[q] = AKC ? dma_kc_base<DT, BM, KROW>(q, M - m0, args.lda, wave, lane)
                  : dma_mn_base<DT, BM, KROW>(q, M - m0, args.lda, wave, lane);
    else
      vo[q] = BKC ? dma_kc_base<DT, BNT, KROW>(q - DA, N - n0, args.ldb, wave, lane)
                  : dma_mn_base<DT, BNT, KROW>(q - DA, N - n0, args.ldb, wave, lane);
  }
  auto dma = [&](int q, int kt, int s, bool live) {
    char* la = smem + s * STAGE;
    char* lb = la + A_BYTES;
    const int k0 = kt * BK;
    // MN operands, whole step in range: precomputed offsets + scalar k0 offset (measured slower
    // than the per-step address math for KC operands, which keep it)
    if (!(q < DA ? AKC : BKC) && k0 + BK <= K) {
      const bool isA = q < DA;
      const int ci = (isA ? q : q - DA) * 8 + wave;
      const int ndma = (isA ? A_BYTES : B_BYTES) / 1024;
      const bool use = live && ((isA ? A_BYTES : B_BYTES) / 1024 % 8 == 0 || ci < ndma);
      char* dst = use ? (isA ? la : lb) + ci * 1024 : junk;
      const bool kc = isA ? AKC : BKC;
      const int64_t ld = isA ? args.lda : args.ldb;
      const uint32_t soff = live ? (uint32_t)(kc ? (int64_t)k0 * ES : (int64_t)k0 * ld * ES) : 0u;
      dma16s(isA ? ra : rb, dst, live ? vo[q] : OOB, soff);
      return;
    }
    if (q < DA) {
      if constexpr (AKC) dma_kc<DT, BM, KROW>(ra, la, junk, q, live, M - m0, k0, K, args.lda, wave, lane);
      else dma_mn<DT, BM, KROW>(ra, la, junk, q, live, M - m0, k0, K, args.lda, wave, lane);
    } else {
      if constexpr (BKC) dma_kc<DT, BNT, KROW>(rb, lb, junk, q - DA, live, N - n0, k0, K, args.ldb, wave, lane);
      else dma_mn<DT, BNT, KROW>(rb, lb, junk, q - DA, live, N - n0, k0, K, args.ldb, wave, lane);
    }
  };

  // acc[i][j][e] = C[row = m0 + wr*WTM + 16i + (lane&15)][col = n0 + wc*WTN + 16j + 4*(lane>>4) + e]
  f32x4 acc[WG::TM][WG::TN];
#pragma unroll
  for (int i = 0; i < WG::TM; ++i)
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // step-invariant per-lane LDS offsets of the MN fragment reads (transposed-read operands)
  int offA[WG::TM], offB[WG::TN];
#pragma unroll
  for (int i = 0; i < WG::TM; ++i) offA[i] = AKC ? 0 : mn_frag_off<DT, BM, KROW>(wr * WG::WTM + i * 16, lane);
#pragma unroll
  for (int j = 0; j < WG::TN; ++j) offB[j] = BKC ? 0 : mn_frag_off<DT, BNT, KROW>(wc * WG::WTN + j * 16, lane);

  const int nk = (K + BK - 1) / BK;
  // prologue: steps 0 .. NST-2 in flight
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) dma(q, p, p, p < nk);

  for (int kt = 0; kt < nk; ++kt) {
    // step kt landed (this wave's DMAs): every step issues exactly D DMAs per wave, so the
    // NST-2 younger steps may stay in flight
    wait_vmcnt<(NST - 2) * D>();
    __builtin_amdgcn_s_barrier();  // ... for every wave; stage (kt-1)%NST is free again
    const int nxt = kt + NST - 1;
    const bool pf = nxt < nk;
    const int snx = nxt % NST;
    const char* la = smem + (kt % NST) * STAGE;
    const char* lb = la + A_BYTES;
    // KC-A kernels spread the next step's D DMAs over the TM A-fragment groups of the first
    // slice; MN-A kernels (transposed reads) issue them all here (measured faster for each).
    if constexpr (!SPREAD) {
#pragma unroll
      for (int q = 0; q < D; ++q) dma(q, nxt, snx, pf);
    }
    if constexpr (DT == CC_BF16) {
      // all fragments of each 32-k slice are read first, so a wave waits for LDS once per slice and
      // then issues its MFMAs back to back
      constexpr int KB = 1;
#pragma unroll
      for (int k0 = 0; k0 < KK; k0 += KB) {
        bf16x8 a[KB][WG::TM], b[KB][WG::TN];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
#pragma unroll
          for (int j = 0; j < WG::TN; ++j) {
            const int c0 = wc * WG::WTN + j * 16;
            b[u][j] = BKC ? frag_kc_bf16<KROW>(lb, c0, k0 + u, lane) : frag_mn_bf16_at<BNT, KROW>(lb, offB[j], k0 + u);
          }
#pragma unroll
          for (int i = 0; i < WG::TM; ++i) {
            const int r0 = wr * WG::WTM + i * 16;
            a[u][i] = AKC ? frag_kc_bf16<KROW>(la, r0, k0 + u, lane) : frag_mn_bf16_at<BM, KROW>(la, offA[i], k0 + u);
          }
        }
        if (SPREAD && k0 == 0) {
#pragma unroll
          for (int q = 0; q < D; ++q) dma(q, nxt, snx, pf);
        }
#pragma unroll
        for (int u = 0; u < KB; ++u)
#pragma unroll
          for (int i = 0; i < WG::TM; ++i)
#pragma unroll
            for (int j = 0; j < WG::TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[u][j], a[u][i], acc[i][j], 0, 0, 0);
        // keep the reads ahead of the MFMAs (the scheduler otherwise sinks them for pressure)
        __builtin_amdgcn_sched_group_barrier(0x100, KB * (WG::TM * (AKC ? 1 : 2) + WG::TN * (BKC ? 1 : 2)), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, KB * WG::TM * WG::TN, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        f32x4 b[WG::TN];
#pragma unroll
        for (int j = 0; j < WG::TN; ++j) {
          const int c0 = wc * WG::WTN + j * 16;
          b[j] = BKC ? frag_kc_f32<KROW>(lb, c0, kk, lane) : frag_mn_f32_at<BNT, KROW>(lb, offB[j], kk);
        }
#pragma unroll
        for (int i = 0; i < WG::TM; ++i) {
          if (SPREAD && kk == 0) {
#pragma unroll
            for (int q = 0; q < D; ++q)
              if (q * WG::TM / D == i) dma(q, nxt, snx, pf);
          }
          const int r0 = wr * WG::WTM + i * 16;
          f32x4 a = AKC ? frag_kc_f32<KROW>(la, r0, kk, lane) : frag_mn_f32_at<BM, KROW>(la, offA[i], kk);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < WG::TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][e], a[e], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  wait_vmcnt<0>();  // drain the junk-slot DMAs of the last NST-1 steps

  gemm_epilogue<DT, EPI, BNT>(args, acc, tm, m0, n0, wr, wc, lane, blockIdx.x * 8 + wave);
}

#include "gemm_pp.h"
#include "gemm_q4_tile.h"

// ---- G4 + G5 with the gradient tail in the same launch (the single-GPU step's backward end).
// What the stand-alone tail kernel (cc_grad_tail) runs after the weight-gradient GEMMs, here inside
// their persistent launch, so the step loses a kernel boundary and a launch:
//   (1) before its first tile, 256-thread group g of workgroup b runs bias reduction blocks
//       2b + g, 2b + g + 2 * grid, ... (b_enc.grad / b_dec.grad column sums of the G3 / loss partial
//       slabs + their sq partials: reduce_rows_phase1/2, the bits cc_grad_tail writes);
//   (2) the dual tile loop of gemm_pp_dual_kernel (static or dynamic order, TileLoop); after each tile the
//       8 waves' squared-sum partials are added in wave order through LDS into tile_sum[tile];
//   (3) the last workgroup to arrive (device-scope arrival counter, reset by it for the next launch) sums,
//       per parameter, tile_sum over the tiles (G5 -> W_enc, G4 -> W_dec) and the bias blocks' partials in a
//       fixed order -- whichever workgroups ran which tiles, the same bits -- into clip_grad_norm_'s
//       coefficient;
//   (4) that workgroup also adds its own lifetime -- s_memtime (shader clock) and s_memrealtime (100 MHz) ticks
//       from its start to the finaliser, which spans the launch: persistent workgroups all start in the first
//       dispatch wave -- into clock[0] / clock[1] and counts the launch in clock[2], so the host reads the clock
//       the chip held over the roofline launches (bench.py `effective_sclk_ghz`).
constexpr int CC_WGRAD_CLOCK_WORDS = 8;  // (floats: the 4 uint64 clock words after the tile sums)
struct WgradTail {
  RedSeg red[2];
  int red_blocks[2];
  ClipArgs clip;
  unsigned* counter;
  float* tile_sum;  // [2 * nb0]: the per-tile squared sums, dW_dec's tiles first
  uint64_t* clock;  // [4] after tile_sum's tile sums: shader ticks, 100 MHz ticks, launches, (reserved)
};

template <bool AKC, bool BKC, int EPI0, int EPI1>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp_dual_tail_kernel(const GemmArgs a0, const GemmArgs a1,
                                                                   const WgradTail tl) {
  __shared__ __attribute__((aligned(16))) char smem[EPI0 == EPI_WGDEC || EPI1 == EPI_WGDEC ? PP_LDS_W : PP_LDS];
  // (scalar reads, uniform over the workgroup: they stay in SGPRs through the tile loop)
  const uint64_t clk0 = __builtin_amdgcn_s_memtime(), wall0 = __builtin_amdgcn_s_memrealtime();
  {
    const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
    float(*red)[RED_COLS] = (float(*)[RED_COLS])(smem + grp * 4 * RED_COLS * sizeof(float));
    const int nred = tl.red_blocks[0] + tl.red_blocks[1];
    for (int base = 2 * (int)blockIdx.x; base < nred; base += 2 * (int)gridDim.x) {  // uniform per workgroup
      const int b = base + grp;
      const int role = b < tl.red_blocks[0] ? 0 : 1, rb = role ? b - tl.red_blocks[0] : b;
      if (b < nred) reduce_rows_phase1(tl.red[role], rb, t, red);
      __syncthreads();
      if (b < nred) reduce_rows_phase2<CC_BF16>(tl.red[role], rb, t, red);
      __syncthreads();
    }
  }
  const int nb0 = a0.nbm * a0.nbn;
  float* wsum_lds = (float*)(smem + PP_SLOT + 64);  // (beside the claim word: free until the next prologue barrier)
  const int wave = threadIdx.x >> 6;
  for (TileLoop L(2 * nb0, a0.tile_ctr, a0.wave_sync); L.more();) {
    const int t = L.begin();
    const int tid = pp_opaque_tid();
    float w;
    if (t < nb0) w = pp_tile<AKC, BKC, EPI0>(a0, smem, t, tid);
    else w = pp_tile<AKC, BKC, EPI1>(a1, smem, t - nb0, tid);
    pp_tile_boundary();
    if ((threadIdx.x & 63) == 0) wsum_lds[wave] = w;
    L.advance(smem);
    if (!L.ctr) __syncthreads();  // (the dynamic advance has its own barrier)
    if (threadIdx.x == 0) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += wsum_lds[k];
      tl.tile_sum[t] = s;
    }
  }
  // publish: the tile sums' stores drained, the barrier joins the waves, ONE agent-scope release writes this
  // XCD's L2 back before the arrival count
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int* last = (int*)smem;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const bool is_last = atomicAdd(tl.counter, 1u) == gridDim.x - 1;
    if (is_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop stale lines before the reads
    *last = is_last;
  }
  __syncthreads();
  if (!*last) return;
  {
    // fixed order: thread j adds each GEMM's tiles j, j + NTHR, ... and bias blocks j, j + NTHR, ...;
    // clip_finish combines the threads in a fixed order
    double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < nb0; k += NTHR) s[1] += (double)tl.tile_sum[k];
    for (int k = threadIdx.x; k < nb0; k += NTHR) s[0] += (double)tl.tile_sum[nb0 + k];
    for (int k = threadIdx.x; k < tl.red_blocks[0]; k += NTHR) s[2] += (double)tl.red[0].sq_part[k];
    for (int k = threadIdx.x; k < tl.red_blocks[1]; k += NTHR) s[3] += (double)tl.red[1].sq_part[k];
    clip_finish<NTHR>(tl.clip, s, (double(*)[NTHR / 64])(smem + 64),
                      (float*)(smem + 64 + 8 * (NTHR / 64) * sizeof(double)));
  }
  if (threadIdx.x == 0) {
    atomicExch(tl.counter, 0u);
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), wall1 = __builtin_amdgcn_s_memrealtime();
    if (tl.clock) {  // (one writer per launch; launches sharing the words are ordered by their stream)
      tl.clock[0] += clk1 - clk0;
      tl.clock[1] += wall1 - wall0;
      tl.clock[2] += 1;
    }
  }
}

// Launch-form switches.  The product library fixes them; the test-only debug build (-DCC_DEBUG_HOOKS,
// libcrosscoder_hip_dbg.so) exports setters so the parity tests can run the alternate forms in one process
// and compare their bits.
//   pp_mask     bf16 GEMM layouts that run the ping-pong kernel (gemm_pp.h, 256 x 256 tiles): bit 0 KC/KC
//               (G1, G3), bit 1 KC/MN (G2), bit 2 MN/MN (G4, G5); the others run gemm_kernel
//   pp_fast     the whole-tile ReLU epilogue form of G1 / G3 (same bits as the general form)
//   dec_one     G2's main tiles and split-K units as one launch (0: two launches, same bits)
//   q4          GEMMs on the 4-wave assembly K loop (gemm_q4_tile.h): bit 0 G1 (EPI_ENC, whole tiles), bit 1 G3 (EPI_DACTS,
//               whole tiles); the same bits as their ping-pong launches.  The product runs G3 on it (its kernel -10 us, the
//               step -2.5 / -4 us); G1 on it is faster alone but slows the side-stream decoder-half Adam beside it, +14 to
//               +27 us per step (profiles/r06_ab_q4_step.txt)
#ifndef CC_Q4_MASK
#define CC_Q4_MASK 2
#endif
#ifdef CC_DEBUG_HOOKS
static int g_pp_mask = 7, g_pp_fast = 1, g_dec_one_launch = 1, g_q4 = CC_Q4_MASK;
#define CC_DEBUG_API extern "C" __attribute__((visibility("default")))
CC_DEBUG_API void cc_debug_set_q4(int mask) { g_q4 = mask; }
CC_DEBUG_API int cc_debug_get_q4() { return CC_Q4_MASK; }
CC_DEBUG_API void cc_debug_set_pp_mask(int mask) { g_pp_mask = mask; }
CC_DEBUG_API void cc_debug_set_pp_fast(int on) { g_pp_fast = on; }
CC_DEBUG_API void cc_debug_set_dec_one_launch(int on) { g_dec_one_launch = on; }
// G4G5 (cc_wgrad_both_t / the _clip_t, _sums_t forms) in the static order with each XCD's waves of tiles
// started together (TileLoop::wave_wait): the L2 panel-reuse probe of VERDICT r03 item 4
static int g_wave_sync = 0;
// per-tile clock stamps of the ping-pong GEMMs (probe build -DCC_PP_STAMPS; NULL: off): pp_tile's anatomy probe
static uint64_t* g_stamps = nullptr;
CC_DEBUG_API void cc_debug_set_stamps(void* buf) { g_stamps = (uint64_t*)buf; }
// ping-pong GEMMs without their output tiles' HBM stores (the epilogue still runs into LDS): the store-exposure probe
static int g_epi_store = 1;
CC_DEBUG_API void cc_debug_set_epi_store(int on) { g_epi_store = on; }
static void debug_epi_store(GemmArgs& a, int64_t stamp_tile0 = 0) {
  if (!g_epi_store) a.out = a.out_t = nullptr;
  if (g_stamps) a.stamps = g_stamps + stamp_tile0 * 12;
}
CC_DEBUG_API void cc_debug_set_wave_sync(int on) { g_wave_sync = on; }
static void debug_wave_sync(GemmArgs& a, hipStream_t st) {
  static uint32_t* words = nullptr;
  if (!g_wave_sync) return;
  if (!words && hipMalloc((void**)&words, 64) != hipSuccess) return;
  if (hipMemsetAsync(words, 0, 32, st) != hipSuccess) return;
  a.wave_sync = words;
  a.tile_ctr = nullptr;
}
// Test / probe kernel: `blocks` workgroups of 512 threads that each hold `lds_bytes` of LDS and spin for `ns`
// nanoseconds of the 100 MHz wall clock (s_sleep between reads) -- a stand-in for another stream's kernel that
// holds CUs (a delayed producer, or RCCL's collective kernel beside a GEMM).  Every wave exits on the clock.
__global__ __launch_bounds__(NTHR) void debug_spin_kernel(int64_t ticks) {
  extern __shared__ char hold[];
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) hold[0] = 0;
  while (wall_clock64() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(8);
}
CC_DEBUG_API int cc_debug_spin(int64_t blocks, int64_t lds_bytes, int64_t ns, void* stream) {
  if (blocks <= 0 || blocks > 4096 || lds_bytes < 0 || lds_bytes > 160 * 1024 || ns < 0 || ns > 1000000000)
    return CC_ERR_SHAPE;
  if (lds_bytes > 65536 && hipFuncSetAttribute((const void*)debug_spin_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes) != hipSuccess)
    return CC_ERR_SHAPE;
  hipLaunchKernelGGL(debug_spin_kernel, dim3((unsigned)blocks), dim3(NTHR), (unsigned)lds_bytes, (hipStream_t)stream,
                     (int64_t)(ns / 10));
  CC_LAUNCH_CHECK();
  return CC_OK;
}
// The same launch through hipExtLaunchKernel with a stop event (probe: whether an event recorded by the launch
// itself costs the stream the idle gap of a separate hipEventRecord)
CC_DEBUG_API int cc_debug_spin_ev(int64_t blocks, int64_t ns, void* stream, void* stop_event) {
  if (blocks <= 0 || blocks > 4096 || ns < 0 || ns > 1000000000) return CC_ERR_SHAPE;
  hipExtLaunchKernelGGL(debug_spin_kernel, dim3((unsigned)blocks), dim3(NTHR), 0, (hipStream_t)stream, nullptr,
                        (hipEvent_t)stop_event, 0, (int64_t)(ns / 10));
  CC_LAUNCH_CHECK();
  return CC_OK;
}
#else
constexpr int g_pp_mask = 7, g_pp_fast = 1, g_dec_one_launch = 1, g_q4 = CC_Q4_MASK;
#endif
// N = n*d multiple of 288 (and an MN-contiguous bf16 B operand): 256 x 288 tiles.  (The fp32
// parity mode keeps 256 x 256: its 288-wide variant exceeds 256 VGPRs.)
static bool use_pp(int64_t N, bool akc, bool bkc, int dtype) {
  // (N % 8: the ping-pong epilogue moves whole 16-byte column chunks through LDS)
  if (dtype != CC_BF16 || (!akc && bkc) || N % 8) return false;
  const int bit = akc && bkc ? 0 : (akc ? 1 : 2);
  return (g_pp_mask >> bit) & 1;
}
// 1 when the transposed-operand entries (cc_encode_fwd_t, cc_dacts_bwd_t, cc_wgrad_both_t's fused
// form) serve this step shape.
// A cc_colsum_job as the launch's prologue reduction (reduce_rows' fields: out_f32 only).
static int set_pre(GemmArgs& a, const cc_colsum_job* job) {
  if (!job) return CC_OK;
  if (!job->part || !job->out) return CC_ERR_NULL;
  if (job->rows <= 0 || job->cols <= 0 || job->ld < job->cols) return CC_ERR_SHAPE;
  a.pre = {job->part, (int)job->rows, (int)job->cols, job->ld, job->scale, job->out, nullptr, nullptr, nullptr, nullptr};
  a.pre_blocks = (int)((job->cols + RED_COLS - 1) / RED_COLS);
  return CC_OK;
}

// A cc_loss_tail_job as the launch's prologue work.
static int set_tail(GemmArgs& a, const cc_loss_tail_job* j) {
  if (!j) return CC_OK;
  if (!j->colsum_acts || !j->tn || !j->l1_part || !j->row_part || !j->scalars || !j->counter) return CC_ERR_NULL;
  if (j->h <= 0 || j->B <= 0 || j->n <= 0 || j->ncb <= 0) return CC_ERR_SHAPE;
  a.tail = make_loss_tail_args(j->colsum_acts, j->tn, j->h, j->l1_part, j->row_part, j->ncb, j->l0_part, j->n_l0, j->ev,
                               j->ev_a, j->ev_b, j->scalars, j->l1l0_out, j->host_out, j->seq, j->B, j->n, j->counter);
  a.tail_items = a.tail.l1_wgs + a.tail.ev.nblk;
  return CC_OK;
}

extern "C" int cc_transposed_ok(int64_t B, int64_t K, int64_t h, int dtype) {
  return dtype == CC_BF16 && B % 8 == 0 && K % 8 == 0 && h % 8 == 0 && use_pp(h, true, true, dtype) &&
         use_pp(K, true, true, dtype);
}
static int pick_bn(int64_t N, bool akc, bool bkc, int dtype) {
  if (use_pp(N, akc, bkc, dtype)) return 256;
  return (!bkc && dtype == CC_BF16 && N % 288 == 0) ? 288 : 256;
}
static int64_t n_blocks(int64_t M, int64_t N, int bn) { return ((M + BM - 1) / BM) * ((N + bn - 1) / bn); }

template <int DT, bool AKC, bool BKC, int EPI, int BNT>
static int launch(GemmArgs a, hipStream_t st) {
  a.nbm = (a.M + BM - 1) / BM;
  a.nbn = (a.N + BNT - 1) / BNT;
  dim3 grid(a.nbm * a.nbn), block(NTHR);
  hipLaunchKernelGGL((gemm_kernel<DT, AKC, BKC, EPI, BNT>), grid, block, 0, st, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

// grid of a ping-pong launch over `tiles` output tiles: one workgroup per tile, or (persistent tile loop)
// at most one per CU
static int pp_grid(int64_t tiles) {
  static int cus = 0;
  static std::once_flag once;
  std::call_once(once, [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  });
  return (int)(tiles < cus ? tiles : cus);
}

template <bool AKC, bool BKC, int EPI>
static int launch_pp(GemmArgs a, hipStream_t st) {
#ifdef CC_DEBUG_HOOKS
  debug_epi_store(a);
#endif
  a.nbm = (a.M + BM - 1) / BM;
  a.nbn = (a.N + 255) / 256;
  if constexpr (EPI == EPI_ENC || EPI == EPI_DACTS) {
    // whole tiles, ReLU on (encode: no l1 partials; d_acts: with G1's mask bits)
    if (g_pp_fast && a.M % BM == 0 && a.N % 256 == 0 &&
        (EPI == EPI_DACTS ? a.mask_bits != nullptr : a.flag && !a.wave_part0)) {
      if constexpr (AKC && BKC) {
        if ((g_q4 >> (EPI == EPI_ENC ? 0 : 1)) & 1 && a.K % 64 == 0 && a.K >= 128 && a.lda == a.ldb) {
          if constexpr (EPI == EPI_ENC)
            hipLaunchKernelGGL((gemm_q4_enc_kernel<true>), dim3(pp_grid(a.nbm * a.nbn)), dim3(Q4_THREADS), 0, st, a);
          else
            hipLaunchKernelGGL((gemm_q4_kernel<EPI, true>), dim3(pp_grid(a.nbm * a.nbn)), dim3(Q4_THREADS), 0, st, a);
          CC_LAUNCH_CHECK();
          return CC_OK;
        }
      }
      hipLaunchKernelGGL((gemm_pp_kernel<AKC, BKC, EPI, true>), dim3(pp_grid(a.nbm * a.nbn)), dim3(NTHR), 0, st, a);
      CC_LAUNCH_CHECK();
      return CC_OK;
    }
  }
  hipLaunchKernelGGL((gemm_pp_kernel<AKC, BKC, EPI>), dim3(pp_grid(a.nbm * a.nbn)), dim3(NTHR), 0, st, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

template <int EPI, bool AKC, bool BKC>
static int launch_dt(int dtype, GemmArgs a, hipStream_t st) {
  if constexpr (!(!AKC && BKC)) {
    if (use_pp(a.N, AKC, BKC, dtype)) return launch_pp<AKC, BKC, EPI>(a, st);
  }
  if constexpr (!BKC) {
    if (pick_bn(a.N, AKC, BKC, dtype) == 288) return launch<CC_BF16, AKC, BKC, EPI, 288>(a, st);
  }
  if (dtype == CC_BF16) return launch<CC_BF16, AKC, BKC, EPI, 256>(a, st);
  if (dtype == CC_F32) return launch<CC_F32, AKC, BKC, EPI, 256>(a, st);
  return CC_ERR_DTYPE;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Shape / alignment validation shared by all GEMM entries.
static int check_gemm(const GemmArgs& a, int dtype, bool akc, bool bkc) {
  if (!a.A || !a.B) return CC_ERR_NULL;
  if (dtype != CC_BF16 && dtype != CC_F32) return CC_ERR_DTYPE;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) return CC_ERR_SHAPE;
  int epc = dtype == CC_BF16 ? 8 : 4;
  // vector (16 B) granularity of contiguous dims / leading dims; epilogue vectors of 4 columns
  if (akc && (a.K % epc)) return CC_ERR_SHAPE;
  if (!akc && (a.M % epc)) return CC_ERR_SHAPE;
  if (bkc && (a.K % epc)) return CC_ERR_SHAPE;
  if (!bkc && (a.N % epc)) return CC_ERR_SHAPE;
  if (a.N % 4 || a.ldo % 4) return CC_ERR_SHAPE;
  if ((a.lda % epc) || (a.ldb % epc)) return CC_ERR_ALIGN;
  if (!al16(a.A) || !al16(a.B)) return CC_ERR_ALIGN;
  int es = dtype == CC_BF16 ? 2 : 4;
  uint64_t ra = akc ? (uint64_t)BM * a.lda * es : (uint64_t)a.K * a.lda * es;
  uint64_t rb = bkc ? (uint64_t)288 * a.ldb * es : (uint64_t)a.K * a.ldb * es;
  if (ra >= MAX_RECORDS || rb >= MAX_RECORDS) return CC_ERR_TOO_LARGE;
  return CC_OK;
}

}  // namespace cc

using namespace cc;

extern "C" {

int64_t cc_col_part_rows(int64_t M) { return 2 * ((M + BM - 1) / BM); }
int64_t cc_wave_parts(int64_t M, int64_t N) { return 8 * n_blocks(M, N, 256); }
// exactly the partials the weight-gradient GEMMs write (the clip sums all of them)
int64_t cc_wgrad_parts(int64_t h, int64_t K, int dtype) { return 8 * n_blocks(h, K, pick_bn(K, false, false, dtype)); }
int64_t cc_wgrad_tile_sums(int64_t h, int64_t K) { return 2 * n_blocks(h, K, 256) + CC_WGRAD_CLOCK_WORDS; }

int cc_gemm_f32out(const void* A, int a_layout, int64_t lda, const void* Bm, int b_layout, int64_t ldb, float* C,
                   int64_t ldc, int64_t M, int64_t N, int64_t K, int dtype, void* stream) {
  GemmArgs a = {};
  a.A = A; a.B = Bm; a.lda = lda; a.ldb = ldb; a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.out = C; a.ldo = ldc;
  if (!C) return CC_ERR_NULL;
  if (((uintptr_t)C & 15) != 0) return CC_ERR_ALIGN;
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

// cc_encode_fwd that also stores acts transposed, acts_t [h][B] (the batch-contiguous operand of
// the KC/KC weight-gradient GEMM, cc_wgrad_both_t).  bf16, B % 8 == 0, ping-pong path only.
int64_t cc_mask_bits_words(int64_t B, int64_t h) { return n_blocks(B, h, 256) * NTHR * 4; }

int cc_encode_fwd_t(const void* x, const void* W_enc, const void* b_enc, const float* tn, void* acts, void* acts_t,
                    int apply_relu, float* colsum_part, float* l1_part, float* l0_part, uint32_t* mask_bits,
                    uint32_t* tile_ctr, const cc_colsum_job* pre, int64_t B, int64_t K, int64_t h, int dtype,
                    void* stream) {
  if (!acts || !acts_t) return CC_ERR_NULL;
  if (l1_part && !tn) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = x; a.lda = K; a.B = W_enc; a.ldb = K;
  a.M = (int)B; a.N = (int)h; a.K = (int)K;
  a.out = acts; a.ldo = h; a.bias = b_enc; a.tn = tn; a.flag = apply_relu;
  a.col_part = colsum_part; a.wave_part0 = l1_part; a.wave_part1 = l0_part;
  a.out_t = acts_t; a.ldt = B; a.mask_bits = mask_bits; a.tile_ctr = tile_ctr;
  int rc = check_gemm(a, dtype, true, true);
  if (rc) return rc;
  if ((rc = set_pre(a, pre))) return rc;
  if (B % 8 || !al16(acts_t) || !use_pp(a.N, true, true, dtype)) return CC_ERR_SHAPE;
  if (mask_bits && !al16(mask_bits)) return CC_ERR_ALIGN;
  return launch_pp<true, true, EPI_ENC>(a, (hipStream_t)stream);
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

}  // extern "C"

// ---- G2 with the leftover tiles split over K (bf16, fp32 output, no bias) ----
// 256-tile waves: the tiles of the first `nbn_main` column blocks fill whole waves (ping-pong
// kernel, full contraction); the remaining column blocks' tiles (a partial wave, e.g. 32 of 288
// at 4096 x 4608) run as S-way split-K passes (S * tiles <= 256 blocks, one wave of 1/S length)
// whose fp32 partials a fixed-order reduce sums: deterministic, and ~1/S of a wave instead of a
// whole one.
struct DecPlan {
  int nbn_main;   // column blocks (of 256) in the whole-wave launch
  int tail_cols;  // columns handled by the split passes
  int nsplit, steps_per, nk;
};
static bool dec_plan(int64_t B, int64_t h, int64_t K, int dtype, DecPlan& p) {
  p = DecPlan{};
  if (dtype != CC_BF16 || K % 8 || h % 8) return false;
  const int64_t nbm = (B + BM - 1) / BM, nbn = (K + 255) / 256, tiles = nbm * nbn;
  const int64_t waves = tiles / 256;
  if (waves == 0 || tiles % 256 == 0 || (256 * waves) % nbm) return false;
  p.nbn_main = (int)(256 * waves / nbm);
  if (p.nbn_main >= nbn) return false;
  p.tail_cols = (int)(K - (int64_t)p.nbn_main * 256);
  const int64_t tail_tiles = nbm * (nbn - p.nbn_main);
  p.nk = (int)((h + 63) / 64);
  int S = (int)(256 / tail_tiles);
  if (S < 2) return false;
  if (S > p.nk) S = p.nk;
  p.steps_per = (p.nk + S - 1) / S;
  p.nsplit = (p.nk + p.steps_per - 1) / p.steps_per;
  return p.nsplit >= 2;
}

// Sum of the S split-K partial slabs (fixed order) into out[m][n] (ldo): the slabs hold each tile
// in accumulator-fragment order (EPI_SPLIT: tile, wave, fragment, lane -> 4 floats), so the split
// passes store whole 1-KB pieces; one thread per (tile, wave, fragment, lane).
// The decoder norms' finaliser as extra blocks of a launch (NormFin::part NULL: none): finaliser block b does rows
// 256 b .. +255, one per thread (norms_finalize_row) -- the norms are first read after the launch, their partials
// are complete before.  The finaliser's blocks come FIRST in the grid, so they run beside the launch's own blocks
// instead of as a tail after them (appended, the split reduction + finaliser took 31 us vs 21 us as two launches).
struct NormFin {
  const float* part;
  int h, n, bpm;
  float* norms;
  float* total;
  float* inv;
};
CC_DEV void norm_fin_block(const NormFin& nf, int b) {
  const int row = b * 256 + (int)threadIdx.x;
  if (row < nf.h) norms_finalize_row(nf.part, row, nf.n, nf.bpm, nf.norms, nf.total, nf.inv);
}
CC_DEV int norm_fin_blocks(const NormFin& nf) { return nf.part ? (nf.h + 255) / 256 : 0; }

__global__ __launch_bounds__(256) void reduce_splits_kernel(const float* __restrict__ part, int S, int64_t split_stride,
                                                            int M, int N, int nbm, int nbn, float* __restrict__ out,
                                                            int64_t ldo, const NormFin nf) {
  const int nfb = norm_fin_blocks(nf);
  if ((int)blockIdx.x < nfb) {  // (the norm finaliser's blocks, cc_decode_partial)
    norm_fin_block(nf, (int)blockIdx.x);
    return;
  }
  const int64_t t = (int64_t)(blockIdx.x - nfb) * 256 + threadIdx.x;
  if (t >= (int64_t)nbm * nbn * 8 * 32 * 64) return;
  const int lane = (int)(t & 63), f = (int)((t >> 6) & 31), wave = (int)((t >> 11) & 7);
  const int tile = (int)(t >> 14);  // slab tile index tm * nbn + tn (EPI_SPLIT)
  const int tm = tile / nbn, tn = tile - tm * nbn;
  const int row = tm * BM + (wave >> 2) * 128 + 16 * (f >> 2) + (lane & 15);
  const int col = tn * 256 + (wave & 3) * 64 + 16 * (f & 3) + 4 * (lane >> 4);
  if (row >= M || col >= N) return;
  f32x4 a = *(const f32x4*)(part + t * 4);
  for (int q = 1; q < S; ++q) a += *(const f32x4*)(part + q * split_stride + t * 4);
  *(f32x4*)(out + (int64_t)row * ldo + col) = a;
}

extern "C" {

// floats of one split's partial slab: whole 256 x 256 tiles of the leftover columns
static int64_t split_stride_of(int64_t B, const DecPlan& p) {
  return ((B + BM - 1) / BM) * ((p.tail_cols + 255) / 256) * (int64_t)BM * 256;
}

int64_t cc_decode_ws_floats(int64_t B, int64_t h, int64_t K, int dtype) {
  DecPlan p;
  if (!dec_plan(B, h, K, dtype, p)) return 0;
  return (int64_t)p.nsplit * split_stride_of(B, p);
}

}  // extern "C"

// BKC: W_dec given transposed, W_dec_t [K][h] (both operands contract over h contiguously)
template <bool BKC>
static int decode_fwd_ws(const void* acts, const void* W_dec, float* recon_f32, float* ws, int64_t ws_floats,
                         int64_t B, int64_t h, int64_t K, int dtype, hipStream_t st, const cc_colsum_job* pre = nullptr,
                         const NormFin& nf = NormFin{}, const uint32_t* wait_ctr = nullptr, uint32_t wait_target = 0,
                         uint32_t* wait_err = nullptr) {
  if (!recon_f32) return CC_ERR_NULL;
  // (the in-kernel wait: the ping-pong kernels' pp_wait_ready, bf16 only)
  if (wait_ctr && (dtype != CC_BF16 || !use_pp(K, true, BKC, dtype))) return CC_ERR_SHAPE;
  DecPlan p;
  const bool split = dec_plan(B, h, K, dtype, p);
  const int64_t ldb = BKC ? h : K;
  const int nf_blocks = nf.part ? (nf.h + 255) / 256 : 0;
  if (!split) {
    GemmArgs a = {};
    a.A = acts; a.lda = h; a.B = W_dec; a.ldb = ldb;
    a.M = (int)B; a.N = (int)K; a.K = (int)h;
    a.out_f32 = recon_f32; a.ldo = K;
    a.wait_ctr = wait_ctr; a.wait_target = wait_target; a.wait_err = wait_err;
    int rc = check_gemm(a, dtype, true, BKC);
    if (rc) return rc;
    if (pre) {  // (the job runs in the ping-pong kernels' prologue only: else its stand-alone launches first)
      if (!use_pp(a.N, true, BKC, dtype)) {
        if ((rc = cc_reduce_rows(pre->part, pre->rows, pre->cols, pre->ld, pre->scale, pre->out, nullptr, CC_F32,
                                 nullptr, nullptr, nullptr, st)))
          return rc;
      } else if ((rc = set_pre(a, pre))) {
        return rc;
      }
    }
    rc = launch_dt<EPI_DEC, true, BKC>(dtype, a, st);
    if (rc || !nf_blocks) return rc;
    hipLaunchKernelGGL(reduce_splits_kernel, dim3((unsigned)nf_blocks), dim3(256), 0, st, nullptr, 0, (int64_t)0, 0, 0,
                       0, 0, nullptr, (int64_t)0, nf);
    CC_LAUNCH_CHECK();
    return CC_OK;
  }
  if (!ws) return CC_ERR_NULL;
  const int64_t split_stride = split_stride_of(B, p);
  if (ws_floats < (int64_t)p.nsplit * split_stride) return CC_ERR_SHAPE;
  if (((uintptr_t)ws & 15) || ((uintptr_t)recon_f32 & 15)) return CC_ERR_ALIGN;
  GemmArgs a = {};
  a.A = acts; a.lda = h; a.B = W_dec; a.ldb = ldb;
  a.M = (int)B; a.N = p.nbn_main * 256; a.K = (int)h;
  a.out_f32 = recon_f32; a.ldo = K;
  a.wait_ctr = wait_ctr; a.wait_target = wait_target; a.wait_err = wait_err;
  int rc = check_gemm(a, dtype, true, BKC);
  if (rc) return rc;
  if (pre && (rc = set_pre(a, pre))) return rc;
  GemmArgs t = {};
  t.A = acts; t.lda = h; t.B = (const bf16_t*)W_dec + (int64_t)p.nbn_main * 256 * (BKC ? h : 1); t.ldb = ldb;
  t.M = (int)B; t.N = p.tail_cols; t.K = (int)h;
  t.out = ws; t.ldo = p.tail_cols;
  t.wait_ctr = wait_ctr; t.wait_target = wait_target; t.wait_err = wait_err;
  t.nbm = (t.M + BM - 1) / BM;
  t.nbn = (t.N + 255) / 256;
  if (g_dec_one_launch) {
    // main tiles and split units in one grid (gemm_pp_main_splitk_kernel)
    a.nbm = (a.M + BM - 1) / BM;
    a.nbn = (a.N + 255) / 256;
    hipLaunchKernelGGL((gemm_pp_main_splitk_kernel<true, BKC, EPI_DEC>),
                       dim3(a.nbm * a.nbn + p.nsplit * t.nbm * t.nbn), dim3(NTHR), 0, st, a, t, p.steps_per, p.nk,
                       split_stride);
    CC_LAUNCH_CHECK();
  } else {
    rc = launch_pp<true, BKC, EPI_DEC>(a, st);  // whole waves
    if (rc) return rc;
    hipLaunchKernelGGL((gemm_pp_splitk_kernel<true, BKC>), dim3(p.nsplit * t.nbm * t.nbn), dim3(NTHR), 0, st, t,
                       p.steps_per, p.nk, split_stride);
    CC_LAUNCH_CHECK();
  }
  const int64_t threads = (int64_t)t.nbm * t.nbn * 8 * 32 * 64;
  hipLaunchKernelGGL(reduce_splits_kernel, dim3((unsigned)((threads + 255) / 256 + nf_blocks)), dim3(256), 0, st, ws,
                     p.nsplit, split_stride, t.M, t.N, t.nbm, t.nbn, recon_f32 + (int64_t)p.nbn_main * 256, (int64_t)K,
                     nf);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

extern "C" {

int cc_decode_fwd_ws(const void* acts, const void* W_dec, float* recon_f32, float* ws, int64_t ws_floats, int64_t B,
                     int64_t h, int64_t K, int dtype, void* stream) {
  return decode_fwd_ws<false>(acts, W_dec, recon_f32, ws, ws_floats, B, h, K, dtype, (hipStream_t)stream);
}

int cc_decode_fwd_ws_t(const void* acts, const void* W_dec_t, float* recon_f32, float* ws, int64_t ws_floats,
                       int64_t B, int64_t h, int64_t K, int dtype, void* stream) {
  return decode_fwd_ws<true>(acts, W_dec_t, recon_f32, ws, ws_floats, B, h, K, dtype, (hipStream_t)stream);
}

int cc_decode_partial(const void* acts, const void* W_dec, float* recon_f32, float* ws, int64_t ws_floats,
                      const float* norm_part, float* norms, float* tn, float* inv_norms, const cc_colsum_job* pre,
                      const uint32_t* wait_ctr, uint32_t wait_target, uint32_t* wait_err, int64_t B, int64_t h,
                      int64_t n, int64_t d, int dtype, void* stream) {
  if (norm_part && (!norms || !tn || d % 64)) return norms && tn ? CC_ERR_SHAPE : CC_ERR_NULL;
  NormFin nf = {};
  if (norm_part) nf = NormFin{norm_part, (int)h, (int)n, (int)(d / 64), norms, tn, inv_norms};
  return decode_fwd_ws<false>(acts, W_dec, recon_f32, ws, ws_floats, B, h, n * d, dtype, (hipStream_t)stream, pre, nf,
                              wait_ctr, wait_target, wait_err);
}

}  // extern "C"

// ---- G2 + the reconstruction loss in one pass (bf16) ----
// The whole-contraction tiles run the loss as their epilogue (EPI_DLOSS: the fp32 reconstruction never
// reaches HBM); the split-K leftover columns are summed here in the fixed order of reduce_splits_kernel
// and run the same per-element arithmetic (loss_kernel's): g_recon is bit-identical to decode + loss.
// Block: 128 rows x 64 columns of the leftover region (tail-relative column ct0 = 64 * blockIdx.x), 16
// waves: lane -> 8 columns (lane & 7) of row 8 * wave + (lane >> 3).  Row terms per 64-column block
// (row_part[2][n * d/64][B]), column sums of g_recon per 128-row group (col_part[B/128][K]), g_recon^T
// through an LDS tile.  B % 8 == 0, d % 64 == 0.
// Blocks with blockIdx.y >= part_rows (= cc_col_part_rows(B)) instead finalise the decoder norms from their
// per-block partials (norms_finalize_row, 64 rows per block, one per lane of its first wave -- the stand-alone
// finaliser's spread; 1024 rows per block took 70 us; nf_part NULL: none): the norms are first read
// by G3 and by the side stream's loss tail, both after this launch, and their partials (the decoder-half
// Adam's) are complete before G2 -- the finaliser rides here at no cost on the compute stream instead of
// running on the side stream behind an event the compute stream must wait for.
struct LossSplitArgs {
  const float* part;
  int S, t_nbn, col0, B, K, n, d;
  int64_t split_stride;
  const bf16_t* b_dec;
  const bf16_t* x;
  const float* x_mean;
  float gs;
  bf16_t* g_recon;
  bf16_t* g_t;
  float* row_part;
  float* col_part;
  int part_rows;
  const float* nf_part;  // decoder-norm partials [h][n * nf_bpm] (NULL: no finaliser blocks)
  int nf_h, nf_n, nf_bpm;
  float* nf_norms;
  float* nf_total;
  float* nf_inv;
};
constexpr int LSPLIT_THREADS = 1024;
__global__ __launch_bounds__(LSPLIT_THREADS) void loss_split_kernel(const LossSplitArgs a) {
  constexpr int TP = 128 + 8;  // padded LDS row (rows of one column of the transposed tile)
  constexpr int NW = LSPLIT_THREADS / 64;
  __shared__ __attribute__((aligned(16))) bf16_t tt[64 * TP];
  __shared__ float red[NW][64];
  if ((int)blockIdx.y >= a.part_rows) {  // (64 rows per block, wave 0: the finaliser spread over many CUs)
    const int row = (((int)blockIdx.y - a.part_rows) * (int)gridDim.x + (int)blockIdx.x) * 64 + (int)threadIdx.x;
    if (threadIdx.x < 64 && row < a.nf_h)
      norms_finalize_row(a.nf_part, row, a.nf_n, a.nf_bpm, a.nf_norms, a.nf_total, a.nf_inv);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cq = lane & 7;
  const int ct = blockIdx.x * 64 + cq * 8;  // tail-relative column of this lane's 8
  const int c = a.col0 + ct;                // global column
  const int r0 = blockIdx.y * 128;
  const int cblk = a.col0 + blockIdx.x * 64;
  const int m = cblk / a.d, ncb = a.d / 64, cb = (cblk - m * a.d) / 64;
  const int rl = w * 8 + (lane >> 3);
  const int r = r0 + rl;
  float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r0 + w * 8 < a.B) {  // wave-uniform (B % 8 == 0)
    // slab coordinates of (r, ct): tile (tm, tn), wave, fragment (i, j), lane (lr + 16 lg)
    const int tn = ct >> 8, cc2 = ct & 255;
    const int tm = r >> 8, rr2 = r & 255;
    const int wave = (rr2 >> 7) * 4 + (cc2 >> 6), i = (rr2 & 127) >> 4, j = (cc2 & 63) >> 4;
    const int lr = rr2 & 15, lg = (cc2 & 15) >> 2;
    const int64_t off = ((int64_t)(tm * a.t_nbn + tn) * 8 + wave) * 8192 + ((i * 4 + j) * 64 + lr + 16 * lg) * 4;
    float bd[8], mu[8], xv[8];
    load8<CC_BF16>(a.b_dec, c, bd);
    load8f(a.x_mean, c, mu);
    load8<CC_BF16>(a.x, (int64_t)r * a.K + c, xv);
    f32x4 u = *(const f32x4*)(a.part + off), v = *(const f32x4*)(a.part + off + 64);
    for (int s = 1; s < a.S; ++s) {  // reduce_splits' order
      u += *(const f32x4*)(a.part + s * a.split_stride + off);
      v += *(const f32x4*)(a.part + s * a.split_stride + off + 64);
    }
    float l2 = 0.f, tv = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float rv = e < 4 ? u[e] : v[e - 4];
      const float diff = (rv + bd[e]) - xv[e];
      l2 += diff * diff;
      const float q = xv[e] - mu[e];
      tv += q * q;
      g[e] = Elem<CC_BF16>::round(a.gs * diff);
      tt[(cq * 8 + e) * TP + rl] = f2bf(g[e]);
    }
    store8<CC_BF16>(a.g_recon, (int64_t)r * a.K + c, g);
    l2 = block8_sum(l2);
    tv = block8_sum(tv);
    if (cq == 0) {
      const int64_t plane = (int64_t)a.n * ncb * a.B;
      a.row_part[(int64_t)(m * ncb + cb) * a.B + r] = l2;
      a.row_part[plane + (int64_t)(m * ncb + cb) * a.B + r] = tv;
    }
  }
  // column sums over the block's 128 rows: the 8 row lanes of each column group, then the waves
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float s = g[e];
    s += __shfl_xor(s, 8, 64);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane < 8) red[w][cq * 8 + e] = s;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    float s = red[0][t];
    for (int q = 1; q < NW; ++q) s += red[q][t];
    a.col_part[(int64_t)blockIdx.y * a.K + cblk + t] = s;
  }
  // g_recon^T: column cblk + cc gets rows [r0, r0 + 128) as 16 chunks of 16 B (one per thread)
  const int cc = threadIdx.x >> 4, ch = threadIdx.x & 15;
  if (a.g_t && r0 + ch * 8 < a.B)
    *(u32x4*)(a.g_t + (int64_t)(cblk + cc) * a.B + r0 + ch * 8) = *(const u32x4*)(tt + cc * TP + ch * 8);
}

extern "C" {

// Row-term column blocks per model of cc_decode_loss_t's row_part (d / 64), or 0 when the fused entry
// does not serve the shape (then: cc_decode_fwd_ws_t + cc_loss_fwd_bwd_rows_t).
int64_t cc_decode_loss_ncb(int64_t B, int64_t h, int64_t n, int64_t d, int dtype) {
  const int64_t K = n * d;
  if (dtype != CC_BF16 || B <= 0 || h <= 0 || n <= 0 || d <= 0) return 0;
  if (B % 8 || h % 8 || d % 64 || !use_pp(K, true, true, dtype)) return 0;
  return d / 64;
}

}  // extern "C"

// BKC: W_dec given transposed (W_dec_t [K][h], KC/KC); otherwise W_dec [h][K] itself (KC/MN)
template <bool BKC>
static int decode_loss(const void* acts, const void* W_dec, const void* b_dec, const void* x, const float* x_mean,
                       float grad_scale, void* g_recon, void* g_recon_t, float* row_part, float* col_part, float* ws,
                       int64_t ws_floats, const float* norm_part, float* norms, float* tn, float* inv_norms,
                       const cc_colsum_job* pre, const uint32_t* wait_ctr, uint32_t wait_target, uint32_t* wait_err,
                       int64_t B, int64_t h, int64_t n, int64_t d, int dtype, hipStream_t st) {
  if (!acts || !W_dec || !b_dec || !x || !x_mean || !g_recon || !row_part || !col_part) return CC_ERR_NULL;
  if (BKC && !g_recon_t) return CC_ERR_NULL;
  if (!cc_decode_loss_ncb(B, h, n, d, dtype) || !use_pp(n * d, true, BKC, dtype)) return CC_ERR_SHAPE;
  if (!al16(x) || !al16(g_recon) || !al16(g_recon_t) || !al16(x_mean) || !al16(b_dec)) return CC_ERR_ALIGN;
  if (norm_part && (!norms || !tn)) return CC_ERR_NULL;
  const int64_t K = n * d;
  const int64_t ldb = BKC ? h : K;
  DecPlan p;
  const bool split = dec_plan(B, h, K, dtype, p);
  GemmArgs a = {};
  a.A = acts; a.lda = h; a.B = W_dec; a.ldb = ldb;
  a.M = (int)B; a.N = split ? p.nbn_main * 256 : (int)K; a.K = (int)h;
  a.out = g_recon; a.ldo = K; a.out_t = g_recon_t; a.ldt = B;
  a.mask_src = x; a.bias = b_dec; a.tn = x_mean; a.scale0 = grad_scale;
  a.col_part = col_part; a.row_part = row_part; a.d_model = (int)d; a.n_models = (int)n;
  int rc = check_gemm(a, dtype, true, BKC);
  if (rc) return rc;
  if ((rc = set_pre(a, pre))) return rc;
  a.wait_ctr = wait_ctr; a.wait_target = wait_target; a.wait_err = wait_err;
  a.nbm = (a.M + BM - 1) / BM;
  a.nbn = (a.N + 255) / 256;
  const bool fast = B % BM == 0 && a.N % 256 == 0;
  if (!split) {
    const dim3 grid(pp_grid(a.nbm * a.nbn));
    if (fast) hipLaunchKernelGGL((gemm_pp_kernel<true, BKC, EPI_DLOSS, true>), grid, dim3(NTHR), 0, st, a);
    else hipLaunchKernelGGL((gemm_pp_kernel<true, BKC, EPI_DLOSS>), grid, dim3(NTHR), 0, st, a);
    CC_LAUNCH_CHECK();
    // (no leftover launch to carry it: the stand-alone finaliser after the GEMM, which reads no norms -- and,
    // with wait_ctr, after the GEMM's wait for the partials' producer)
    return norm_part ? cc_dec_norms_finalize(norm_part, h, n, d, norms, tn, inv_norms, st) : CC_OK;
  }
  if (!ws) return CC_ERR_NULL;
  const int64_t split_stride = split_stride_of(B, p);
  if (ws_floats < (int64_t)p.nsplit * split_stride) return CC_ERR_SHAPE;
  if (!al16(ws)) return CC_ERR_ALIGN;
  GemmArgs t = {};
  t.A = acts; t.lda = h; t.B = (const bf16_t*)W_dec + (int64_t)p.nbn_main * 256 * (BKC ? h : 1); t.ldb = ldb;
  t.M = (int)B; t.N = p.tail_cols; t.K = (int)h;
  t.out = ws; t.ldo = p.tail_cols;
  t.wait_ctr = wait_ctr; t.wait_target = wait_target; t.wait_err = wait_err;
  t.nbm = (t.M + BM - 1) / BM;
  t.nbn = (t.N + 255) / 256;
  const dim3 grid(a.nbm * a.nbn + p.nsplit * t.nbm * t.nbn);
  if (fast) hipLaunchKernelGGL((gemm_pp_main_splitk_kernel<true, BKC, EPI_DLOSS, true>), grid, dim3(NTHR), 0, st, a, t,
                               p.steps_per, p.nk, split_stride);
  else hipLaunchKernelGGL((gemm_pp_main_splitk_kernel<true, BKC, EPI_DLOSS>), grid, dim3(NTHR), 0, st, a, t,
                          p.steps_per, p.nk, split_stride);
  CC_LAUNCH_CHECK();
  LossSplitArgs l = {};
  l.part = ws; l.S = p.nsplit; l.t_nbn = t.nbn; l.col0 = p.nbn_main * 256; l.B = (int)B; l.K = (int)K; l.n = (int)n;
  l.d = (int)d; l.split_stride = split_stride;
  l.b_dec = (const bf16_t*)b_dec; l.x = (const bf16_t*)x; l.x_mean = x_mean; l.gs = grad_scale;
  l.g_recon = (bf16_t*)g_recon; l.g_t = (bf16_t*)g_recon_t; l.row_part = row_part; l.col_part = col_part;
  // one block per 128-row half of every 256-row tile (cc_col_part_rows(B) groups, like the main tiles' column-sum
  // rows): a half past B writes zero column sums, so every partial row the backward reduces is written; then
  // the norm finaliser's rows of blocks
  const int gx = p.tail_cols / 64;
  l.part_rows = (int)cc_col_part_rows(B);
  int fin_rows = 0;
  if (norm_part) {
    l.nf_part = norm_part; l.nf_h = (int)h; l.nf_n = (int)n; l.nf_bpm = (int)(d / 64);
    l.nf_norms = norms; l.nf_total = tn; l.nf_inv = inv_norms;
    fin_rows = (int)((h + (int64_t)gx * 64 - 1) / ((int64_t)gx * 64));
  }
  hipLaunchKernelGGL(loss_split_kernel, dim3((unsigned)gx, (unsigned)(l.part_rows + fin_rows)), dim3(LSPLIT_THREADS), 0,
                     st, l);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

extern "C" {

int cc_decode_loss_t(const void* acts, const void* W_dec_t, const void* b_dec, const void* x, const float* x_mean,
                     float grad_scale, void* g_recon, void* g_recon_t, float* row_part, float* col_part, float* ws,
                     int64_t ws_floats, int64_t B, int64_t h, int64_t n, int64_t d, int dtype, void* stream) {
  return decode_loss<true>(acts, W_dec_t, b_dec, x, x_mean, grad_scale, g_recon, g_recon_t, row_part, col_part, ws,
                           ws_floats, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, B, h, n, d,
                           dtype, (hipStream_t)stream);
}

int cc_decode_loss(const void* acts, const void* W_dec, const void* b_dec, const void* x, const float* x_mean,
                   float grad_scale, void* g_recon, void* g_recon_t, float* row_part, float* col_part, float* ws,
                   int64_t ws_floats, const float* norm_part, float* norms, float* tn, float* inv_norms,
                   const cc_colsum_job* pre, const uint32_t* wait_ctr, uint32_t wait_target, uint32_t* wait_err,
                   int64_t B, int64_t h, int64_t n, int64_t d, int dtype, void* stream) {
  return decode_loss<false>(acts, W_dec, b_dec, x, x_mean, grad_scale, g_recon, g_recon_t, row_part, col_part, ws,
                            ws_floats, norm_part, norms, tn, inv_norms, pre, wait_ctr, wait_target, wait_err, B, h, n,
                            d, dtype, (hipStream_t)stream);
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

}  // extern "C"

extern "C" {
// cc_dacts_bwd storing d pre-activations TRANSPOSED only: g_pre_t[j][b] for b < B (row stride ldt
// >= B; a batch slice passes g_pre_t + r0).  bf16, B % 8 == 0, ldt % 8 == 0, ping-pong path only.
int cc_dacts_bwd_t(const void* g_recon, const void* W_dec, const void* acts, const float* tn, float l1_scale,
                   const uint32_t* mask_bits, void* g_pre_t, int64_t ldt, float* colsum_part, uint32_t* tile_ctr,
                   const cc_loss_tail_job* tail, int64_t B, int64_t K, int64_t h, int dtype, void* stream) {
  if (!g_pre_t || !acts) return CC_ERR_NULL;
  GemmArgs a = {};
  a.A = g_recon; a.lda = K; a.B = W_dec; a.ldb = K;
  a.M = (int)B; a.N = (int)h; a.K = (int)K;
  a.out = nullptr; a.ldo = h; a.mask_src = acts; a.tn = tn; a.scale0 = l1_scale;
  a.col_part = colsum_part; a.out_t = g_pre_t; a.ldt = ldt; a.mask_bits = const_cast<uint32_t*>(mask_bits);
  a.tile_ctr = tile_ctr;
  int rc = check_gemm(a, dtype, true, true);
  if (rc) return rc;
  if ((rc = set_tail(a, tail))) return rc;
  if (mask_bits && !al16(mask_bits)) return CC_ERR_ALIGN;
  if (B % 8 || ldt % 8 || ldt < B || !al16(g_pre_t) || !use_pp(a.N, true, true, dtype)) return CC_ERR_SHAPE;
  return launch_pp<true, true, EPI_DACTS>(a, (hipStream_t)stream);
}
}  // extern "C"

// tr: the batch-major operands are given transposed ([h][B] / [K][B], the contraction index B
// contiguous): both GEMM operands are then KC (row-contiguous LDS images, ds_read_b128).
static int wgrad_dec_args(GemmArgs& a, const void* acts, const void* g_recon, const void* W_dec, const float* inv_norms,
                          const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_part, int64_t B,
                          int64_t h, int64_t n, int64_t d, int dtype, bool tr = false) {
  if (!grad_W_dec) return CC_ERR_NULL;
  if (l1_scale != 0.f && (!W_dec || !inv_norms || !colsum_acts)) return CC_ERR_NULL;
  a = GemmArgs{};
  int64_t K = n * d;
  a.A = acts; a.lda = tr ? B : h; a.B = g_recon; a.ldb = tr ? B : K;
  a.M = (int)h; a.N = (int)K; a.K = (int)B;
  a.out = grad_W_dec; a.ldo = K; a.w_src = W_dec; a.norms = inv_norms; a.colsum = colsum_acts;
  a.scale0 = l1_scale; a.wave_part0 = sq_part; a.d_model = (int)d; a.n_models = (int)n;
  return check_gemm(a, dtype, tr, tr);
}

static int wgrad_enc_args(GemmArgs& a, const void* g_pre, const void* x, void* grad_W_enc, float* sq_part, int64_t B,
                          int64_t h, int64_t K, int dtype, bool tr = false) {
  if (!grad_W_enc) return CC_ERR_NULL;
  a = GemmArgs{};
  a.A = g_pre; a.lda = tr ? B : h; a.B = x; a.ldb = tr ? B : K;
  a.M = (int)h; a.N = (int)K; a.K = (int)B;
  a.out = grad_W_enc; a.ldo = K; a.wave_part0 = sq_part;
  return check_gemm(a, dtype, tr, tr);
}

extern "C" {

int cc_wgrad_dec(const void* acts, const void* g_recon, const void* W_dec, const float* inv_norms,
                 const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_part, int64_t B, int64_t h,
                 int64_t n, int64_t d, int dtype, void* stream) {
  GemmArgs a;
  int rc = wgrad_dec_args(a, acts, g_recon, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_part, B, h, n, d,
                          dtype);
  if (rc) return rc;
  return launch_dt<EPI_WGDEC, false, false>(dtype, a, (hipStream_t)stream);
}

int cc_wgrad_enc(const void* g_pre, const void* x, void* grad_W_enc, float* sq_part, int64_t B, int64_t h, int64_t K,
                 int dtype, void* stream) {
  GemmArgs a;
  int rc = wgrad_enc_args(a, g_pre, x, grad_W_enc, sq_part, B, h, K, dtype);
  if (rc) return rc;
  return launch_dt<EPI_WGENC, false, false>(dtype, a, (hipStream_t)stream);
}

int cc_wgrad_both_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                    const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                    const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                    int dtype, void* stream) {
  GemmArgs a0, a1;
  int rc = wgrad_dec_args(a0, actsT, g_reconT, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, B, h, n,
                          d, dtype, true);
  if (rc) return rc;
  rc = wgrad_enc_args(a1, g_preT, xT, grad_W_enc, sq_enc, B, h, n * d, dtype, true);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (!use_pp(a0.N, true, true, dtype)) {
    rc = launch_dt<EPI_WGDEC, true, true>(dtype, a0, st);
    return rc ? rc : launch_dt<EPI_WGENC, true, true>(dtype, a1, st);
  }
  a0.nbm = a1.nbm = (a0.M + BM - 1) / BM;
  a0.nbn = a1.nbn = (a0.N + 255) / 256;
#ifdef CC_DEBUG_HOOKS
  debug_wave_sync(a0, st);
  debug_epi_store(a0);
  debug_epi_store(a1, (int64_t)a0.nbm * a0.nbn);
#endif
  hipLaunchKernelGGL((gemm_pp_dual_kernel<true, true, EPI_WGDEC, EPI_WGENC>), dim3(pp_grid(2 * a0.nbm * a0.nbn)), dim3(NTHR),
                     0, st, a0, a1);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

// (step_kernels.hip, library-internal: cc_grad_tail / cc_grad_tail_sums with the step's abort word)
extern "C" int cc_grad_tail_sums_abort(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc,
                                       float* sq_b_enc, const float* loss_colpart, int64_t R_dec, int64_t K,
                                       void* g_b_dec, float* sq_b_dec, int dtype, const float* sq, const int64_t* off,
                                       int nparams, int zero_mask, float* out, uint32_t* counter,
                                       const uint32_t* abort, void* stream);
extern "C" int cc_grad_tail_abort(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                                  const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec,
                                  int dtype, const float* sq, const int64_t* off, int nparams, float max_norm,
                                  int emulate_bf16, float* clip_out, uint32_t* counter, const uint32_t* abort,
                                  void* stream);

static int wgrad_both_tail(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                           const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                           const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                           const float* gpre_colpart, int64_t R_enc, void* g_b_enc, float* sq_b_enc,
                           const float* loss_colpart, int64_t R_dec, void* g_b_dec, float* sq_b_dec, const float* sq,
                           const int64_t* off, int nparams, float max_norm, int emulate_bf16, int sums_only,
                           int zero_mask, float* out, uint32_t* counter, float* tile_sum, uint32_t* tile_ctr,
                           const uint32_t* abort, int dtype, void* stream) {
  const int64_t K = n * d;
  if (!gpre_colpart || !g_b_enc || !sq_b_enc || !loss_colpart || !g_b_dec || !sq_b_dec || !sq || !off || !out ||
      !counter || !tile_sum || !sq_dec || !sq_enc)  // (the clip's W_dec / W_enc sums come from sq_dec / sq_enc's tiles)
    return CC_ERR_NULL;
  if (R_enc <= 0 || R_dec <= 0) return CC_ERR_SHAPE;
  if (nparams != 4) return CC_ERR_SHAPE;  // W_enc, W_dec, b_enc, b_dec: the segments of sq
  GemmArgs a0, a1;
  int rc = wgrad_dec_args(a0, actsT, g_reconT, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, B, h, n,
                          d, dtype, true);
  if (rc) return rc;
  rc = wgrad_enc_args(a1, g_preT, xT, grad_W_enc, sq_enc, B, h, K, dtype, true);
  if (rc) return rc;
  if (dtype != CC_BF16 || !use_pp(a0.N, true, true, dtype)) {  // the two GEMMs, then the stand-alone tail
    rc = cc_wgrad_both_t(actsT, g_reconT, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, g_preT, xT,
                         grad_W_enc, sq_enc, B, h, n, d, dtype, stream);
    if (rc) return rc;
    if (sums_only)
      return cc_grad_tail_sums_abort(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec,
                                     sq_b_dec, dtype, sq, off, nparams, zero_mask, out, counter, abort, stream);
    return cc_grad_tail_abort(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec, sq_b_dec,
                              dtype, sq, off, nparams, max_norm, emulate_bf16, out, counter, abort, stream);
  }
  a0.nbm = a1.nbm = (a0.M + BM - 1) / BM;
  a0.nbn = a1.nbn = (a0.N + 255) / 256;
  WgradTail tl = {};
  tl.red[0] = {gpre_colpart, (int)R_enc, (int)h, h, 1.f, nullptr, g_b_enc, sq_b_enc, nullptr, nullptr};
  tl.red[1] = {loss_colpart, (int)R_dec, (int)K, K, 1.f, nullptr, g_b_dec, sq_b_dec, nullptr, nullptr};
  tl.red_blocks[0] = (int)((h + RED_COLS - 1) / RED_COLS);
  tl.red_blocks[1] = (int)((K + RED_COLS - 1) / RED_COLS);
  tl.clip.sq = sq;
  for (int i = 0; i <= nparams; ++i) tl.clip.off[i] = off[i];
  tl.clip.nparams = nparams;
  tl.clip.max_norm = max_norm;
  tl.clip.emulate_bf16 = emulate_bf16;
  tl.clip.out = out;
  tl.clip.sums_only = sums_only;
  tl.clip.zero_mask = zero_mask;
  tl.clip.abort = abort;
  tl.counter = counter;
  tl.tile_sum = tile_sum;
  tl.clock = (uint64_t*)(tile_sum + 2 * a0.nbm * a0.nbn);  // (2 * nb0 is even: 8-byte aligned)
  a0.tile_ctr = tile_ctr;
#ifdef CC_DEBUG_HOOKS
  debug_wave_sync(a0, (hipStream_t)stream);
  debug_epi_store(a0);
  debug_epi_store(a1, (int64_t)a0.nbm * a0.nbn);
#endif
  const int grid = pp_grid(2 * a0.nbm * a0.nbn);
  hipLaunchKernelGGL((gemm_pp_dual_tail_kernel<true, true, EPI_WGDEC, EPI_WGENC>), dim3(grid), dim3(NTHR), 0,
                     (hipStream_t)stream, a0, a1, tl);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_wgrad_both_clip_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                         const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                         const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                         const float* gpre_colpart, int64_t R_enc, void* g_b_enc, float* sq_b_enc,
                         const float* loss_colpart, int64_t R_dec, void* g_b_dec, float* sq_b_dec, const float* sq,
                         const int64_t* off, int nparams, float max_norm, int emulate_bf16, float* clip_out,
                         uint32_t* counter, float* tile_sum, uint32_t* tile_ctr, const uint32_t* abort_flag, int dtype,
                         void* stream) {
  return wgrad_both_tail(actsT, g_reconT, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, g_preT, xT,
                         grad_W_enc, sq_enc, B, h, n, d, gpre_colpart, R_enc, g_b_enc, sq_b_enc, loss_colpart, R_dec,
                         g_b_dec, sq_b_dec, sq, off, nparams, max_norm, emulate_bf16, 0, 0, clip_out, counter, tile_sum,
                         tile_ctr, abort_flag, dtype, stream);
}

int cc_wgrad_both_sums_t(const void* actsT, const void* g_reconT, const void* W_dec, const float* inv_norms,
                         const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_preT,
                         const void* xT, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                         const float* gpre_colpart, int64_t R_enc, void* g_b_enc, float* sq_b_enc,
                         const float* loss_colpart, int64_t R_dec, void* g_b_dec, float* sq_b_dec, const float* sq,
                         const int64_t* off, int nparams, int zero_mask, float* out, uint32_t* counter, float* tile_sum,
                         uint32_t* tile_ctr, const uint32_t* abort, int dtype, void* stream) {
  return wgrad_both_tail(actsT, g_reconT, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, g_preT, xT,
                         grad_W_enc, sq_enc, B, h, n, d, gpre_colpart, R_enc, g_b_enc, sq_b_enc, loss_colpart, R_dec,
                         g_b_dec, sq_b_dec, sq, off, nparams, 0.f, 0, 1, zero_mask, out, counter, tile_sum, tile_ctr,
                         abort, dtype, stream);
}

int cc_wgrad_both(const void* acts, const void* g_recon, const void* W_dec, const float* inv_norms,
                  const float* colsum_acts, float l1_scale, void* grad_W_dec, float* sq_dec, const void* g_pre,
                  const void* x, void* grad_W_enc, float* sq_enc, int64_t B, int64_t h, int64_t n, int64_t d,
                  int dtype, void* stream) {
  GemmArgs a0, a1;
  int rc = wgrad_dec_args(a0, acts, g_recon, W_dec, inv_norms, colsum_acts, l1_scale, grad_W_dec, sq_dec, B, h, n, d,
                          dtype);
  if (rc) return rc;
  rc = wgrad_enc_args(a1, g_pre, x, grad_W_enc, sq_enc, B, h, n * d, dtype);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (!use_pp(a0.N, false, false, dtype)) {
    rc = launch_dt<EPI_WGDEC, false, false>(dtype, a0, st);
    return rc ? rc : launch_dt<EPI_WGENC, false, false>(dtype, a1, st);
  }
  a0.nbm = a1.nbm = (a0.M + BM - 1) / BM;
  a0.nbn = a1.nbn = (a0.N + 255) / 256;
  hipLaunchKernelGGL((gemm_pp_dual_kernel<false, false, EPI_WGDEC, EPI_WGENC>), dim3(pp_grid(2 * a0.nbm * a0.nbn)),
                     dim3(NTHR),
                     0, st, a0, a1);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

}  // extern "C"
