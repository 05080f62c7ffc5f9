// Ping-pong bf16 main loop (included by gemm.hip inside namespace cc).
//
// Tile 256 x 256, BK 64, 8 waves 2(M) x 4(N), 128 x 64 outputs per wave (the same accumulator
// map as gemm_kernel<.., 256>, so the epilogues are shared).  The two wave rows form two groups
// (waves 0-3 and 4-7: one wave of each per SIMD) that run half a phase apart: while one group
// issues its MFMAs the other reads its next fragments from LDS and issues its share of the
// LDS-DMA traffic, so each SIMD's matrix pipe alternates between its two waves.
//
// Per K-step each wave runs 4 phases p; phase p = 16 MFMAs (A tiles i = 2p, 2p+1 x the 4 B
// tiles x 2 k-slices).  Fragment reads: all B fragments in phase 0 (kept for the step), the two
// A fragments of the phase in each phase.  Each phase is
//     [ds_read fragments][issue 2 LDS-DMAs][vmcnt(6)] barrier [16 MFMA] barrier
// and group 1 starts one barrier late (group 0 ends with one extra barrier).
//
// LDS: 2 buffers x (A tile 32 KB | B tile 32 KB).  The DMA traffic of one K-step (64 x 1 KB)
// is split over the 4 phases by LDS region, in the order the regions free up:
//   phase 0: A rows {0..63, 128..191} of step t+1     (freed: last read in phase 1 of step t-1)
//   phase 1: A rows {64..127, 192..255} of step t+1   (freed: last read in phase 3 of step t-1)
//   phase 2: B cols/rows 0..127 of step t+2            (freed: last read in phase 0 of step t)
//   phase 3: B cols/rows 128..255 of step t+2
// Every region is read >= 4 phases after its DMA was issued and >= 1 phase after its last
// reader's lgkmcnt-wait + barrier, so a per-phase vmcnt(6) (the DMAs of the last three phases
// may stay in flight) before the phase's barrier orders every read after the data landed.
// Steps past the end load zeros (range-checked offsets), so the loop needs no tail case.
//
// MN operands use 64-column blocks, [4 blocks][64 k][128 B], phys 16-B chunk =
// chunk ^ 2*h(k), h(k) = bit1(k) | bit3(k) << 1: conflict-free for ds_read_b64_tr_b16 (each
// 32-lane group reads 8 k rows x 32 B = all 64 banks once) and full 128-B lines per DMA row.
// KC operands keep [256 rows][128 B] with chunk ^ (row & 7).

#include <type_traits>

// cache-policy bits (buffer-store aux) of the LDS epilogue's output-tile stores: direct and transposed (build
// switches; 0 = default policy)
#ifndef CC_EPI_STORE_AUX
#define CC_EPI_STORE_AUX 0
#endif
#ifndef CC_EPI_STORE_T_AUX
#define CC_EPI_STORE_T_AUX 0
#endif
// dW_dec's W_dec tile (the L1 term's input, prefetched into LDS) is read non-temporal: the next reader of W_dec is
// the decoder-half Adam of the next step, which streams it non-temporal itself; not allocated in the Infinity
// Cache it leaves room for the GEMM's operands (step -3.1 / -4.7 us in two same-box A/Bs, 10 of 12 rounds lower,
// profiles/r04_ab_epilogue_store_policy.txt)
#ifndef CC_WDEC_TILE_AUX
#define CC_WDEC_TILE_AUX 2
#endif
#ifndef CC_WG_OPERAND_AUX  // cache policy of the weight-gradient GEMMs' operand DMAs (the activations' last reads)
#define CC_WG_OPERAND_AUX 0
#endif
#define PP_OPERAND_AUX(E) ((E) == EPI_WGDEC || (E) == EPI_WGENC ? CC_WG_OPERAND_AUX : 0)
#ifndef CC_EPI_STORE_T_AUX_ENC  // (G1's acts^T)
#define CC_EPI_STORE_T_AUX_ENC CC_EPI_STORE_T_AUX
#endif
#ifndef CC_EPI_STORE_T_AUX_DLOSS  // (G2's g_recon^T)
#define CC_EPI_STORE_T_AUX_DLOSS CC_EPI_STORE_T_AUX
#endif
// The weight gradients go out non-temporal: the Adam launches read them once, and kept out of the Infinity Cache
// they leave it to the parameters and activations the step reads next (step -8 / -21 us in two same-box A/Bs,
// profiles/r04_ab_epilogue_store_policy.txt; the same policy on acts^T / g_pre^T / g_recon^T was slower)
#ifndef CC_EPI_STORE_WG_AUX
#define CC_EPI_STORE_WG_AUX 2
#endif
// Tile anatomy probe (build with -DCC_PP_STAMPS; GemmArgs::stamps set by the debug build's cc_debug_set_stamps):
// thread 0 keeps s_memtime at tile entry (0), after the prologue's barrier (1), after the K loop (2), after the
// drain before the epilogue (3) and after the epilogue's stores are issued (4), plus the 100 MHz wall clock at
// entry (5) and end (6), and writes them with one store per value after the epilogue (no store inside the
// K loop: it would sit in the loop's counted vmcnt waits); the LDS epilogue adds s_memtime after its element
// work (7), after the direct stores (8) and after the transposed stores (9).  12 slots per tile.
#ifdef CC_PP_STAMPS
#define PP_STAMP_DECL uint64_t pp_st[7] = {(uint64_t)__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, (uint64_t)wall_clock64(), 0}
#define PP_STAMP(k) pp_st[k] = __builtin_amdgcn_s_memtime()
#define PP_STAMP_WRITE(args, bid)                                                         \
  do {                                                                                    \
    pp_st[6] = wall_clock64();                                                            \
    if ((args).stamps && threadIdx.x == 0)                                                \
      for (int k_ = 0; k_ < 7; ++k_) (args).stamps[(int64_t)(bid) * 12 + k_] = pp_st[k_]; \
  } while (0)
#else
#define PP_STAMP_DECL
#define PP_STAMP(k)
#define PP_STAMP_WRITE(args, bid)
#endif
// (PP_EPI_STAMP: gemm_epilogue.h)
CC_DEV int pp_h(int k) { return ((k >> 1) & 1) | ((k >> 2) & 2); }

// Per-lane source offset (bytes, step k0 = 0) of DMA ci (0..31) of a 256 x 64 operand tile, or
// OOB for rows / columns past the matrix edge.
template <bool KC>
CC_DEV uint32_t pp_dma_off(int ci, int lim, int64_t ld, int lane) {
  if constexpr (KC) {
    const int row = ci * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (lane >> 3);
    return row < lim ? (uint32_t)((int64_t)row * ld * 2 + c * 16) : OOB;
  } else {
    const int k = 8 * (ci & 7) + (lane >> 3);
    const int c = (lane & 7) ^ (2 * pp_h(k));
    const int col = (ci >> 3) * 64 + 8 * c;
    return col < lim ? (uint32_t)(((int64_t)k * ld + col) * 2) : OOB;
  }
}
// Per-lane k (elements, within the step) of this lane's 16 B in every DMA of the operand (the
// K-tail mask): the same for all of a wave's DMAs by construction of the ci schedule.
template <bool KC>
CC_DEV int pp_dma_k(int wave, int lane) {
  return KC ? 8 * ((lane & 7) ^ (lane >> 3)) : 8 * wave + (lane >> 3);
}

// ci of DMA q (0/1) of phase p for this wave (see the schedule above)
CC_DEV int pp_ci(int p, int q, int wave) {
  switch (p) {
    case 0: return (q ? 16 : 0) + wave;
    case 1: return (q ? 24 : 8) + wave;
    case 2: return (q ? 8 : 0) + wave;
    default: return (q ? 24 : 16) + wave;
  }
}

// 16x16x32 operand fragment for the 16 rows/cols starting at r0 (multiple of 16), slice kk.
// KC: lane l holds X[r0 + (l&15)][32kk + 8(l>>4) .. +7]; kc_off[kk] = the lane part.
CC_DEV bf16x8 pp_frag_kc(const char* tile, int r0, int off) {
  return *(const bf16x8*)(tile + r0 * 128 + off);
}
// MN: two transposed 8-byte reads (k rows 32kk + 8g + qq and +4); mn_off[m] = the lane part for
// column groups with (r0 >> 4) & 3 == m.
//
// The reads go through a __restrict__ pointer on purpose.  While an LDS-DMA is in flight hipcc (ROCm 7.2)
// puts an `s_waitcnt vmcnt(0)` before every transposed LDS read whose address carries no alias scope: it
// cannot tell the read apart from the DMA's LDS destination.  In the K loop that drained the whole DMA
// pipeline twice per K step (MN operands ran 18-28 % slower than KC ones).  With the restrict-derived scope
// the read is ordered after the DMA only by the loop's own counted vmcnt + barrier, like the KC reads.
CC_DEV bf16x8 pp_frag_mn(const char* __restrict__ tile, int r0, int kk, int off) {
  const char* p = tile + (r0 >> 6) * 8192 + kk * 32 * 128 + off;
  bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)p);
  bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p + 4 * 128));
  return bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
}

// ---- LDS-staged epilogue (bf16 output tiles, N % 8 == 0) ----
// Tile image: 4 quarters of [64 rows][512 B] (32 KB each, quarter Q = tile rows 64Q..64Q+63 at LDS
// offset qb[Q]), phys 16-B chunk = chunk ^ (row & 15): a fragment access (per 32-lane group 16
// rows x one chunk) hits 16 distinct bank groups.  The image moves between HBM and LDS in whole
// 512-B rows (1 KB piece ci = tile rows 2ci, 2ci+1 = 2 rows per wave instruction, 16 B per lane),
// so every HBM line of the epilogue's input (activation mask / W_dec) and output is transferred
// once and whole -- the fragment-shaped 8-byte accesses of the register path fetch up to 4x the
// bytes (PMC FETCH_SIZE).  Normally qb = {0, 32K, 64K, 96K}; dW_dec's W_dec tile is instead
// prefetched into LDS regions the K loop frees before it ends (pp_tile).
struct LdsIO {
  char* lo;    // quarter of fragments i = 0..3 (rows wr*128 + 0..63)
  char* hi;    // quarter of fragments i = 4..7
  int off[4];  // lane byte offset of fragment (i & 3 = 0, j) within its quarter
  CC_DEV LdsIO(char* s, const int (&qb)[4], int wr, int wc, int lane)
      : lo(s + (wr ? qb[2] : qb[0])), hi(s + (wr ? qb[3] : qb[1])) {  // (no runtime array index: scratch)
    const int r = lane & 15;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 64 + 4 * (lane >> 4) + 16 * j;
      off[j] = r * 512 + (((col >> 3) ^ r) << 4) + (col & 4) * 2;
    }
  }
  CC_DEV char* at(int i, int j) const { return (i < 4 ? lo : hi) + off[j] + (i & 3) * 16 * 512; }
  CC_DEV bf16x4 in4(int i, int j) const { return *(const bf16x4*)at(i, j); }
  CC_DEV void out4(int i, int j, const float v[4]) const { *(bf16x4*)at(i, j) = pack4<CC_BF16>(v); }
  CC_DEV void out4p(int i, int j, bf16x4 p) const { *(bf16x4*)at(i, j) = p; }
};

// Source/destination offset (bytes, in a tile-anchored descriptor) of this lane's 16 B of 1-KB
// image piece ci (tile rows 2ci, 2ci+1), or OOB past the matrix edge.
CC_DEV uint32_t piece_off(int ci, int lane, int rows, int cols, int ldo) {
  const int row = 2 * ci + (lane >> 5);
  const int c = (lane & 31) ^ (row & 15);
  return (row < rows && 8 * c < cols) ? (uint32_t)((row * ldo + 8 * c) * 2) : OOB;
}

// The tile image stored transposed: out_t[n0 + c][m0 + r] (row stride ldt; M % 8 == 0, so an
// 8-row chunk is all in or all out).  ds_read_b64_tr_b16 turns 4 image rows x 16 columns into
// 16 lanes x 4 rows; two of them give a lane 8 consecutive rows (16 B) of one column.  Wave w
// writes transposed rows (tile columns) 32w .. 32w+31, 16 at a time; per store a row gets 64
// contiguous bytes (lane groups g = 0..3 take row chunks 8g.. of a 32-row band), and a wave's 8
// bands complete its 16 rows of 512 B.
template <int AUX, int NW = 8>  // (NW: waves of the workgroup; each writes 256 / NW tile columns)
CC_DEV void pp_store_transposed(const GemmArgs& args, const char* smem, const int (&qb)[4], int m0, int n0, int rows,
                                int cols, int lane, int wave) {
  const int64_t ldt = args.ldt;
  const __amdgpu_buffer_rsrc_t rt =
      make_rsrc((const char*)args.out_t + ((int64_t)n0 * ldt + m0) * 2, ((uint64_t)(cols - 1) * ldt + rows) * 2);
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
#pragma unroll
  for (int s = 0; s < 16 / NW; ++s) {
    const int c0 = wave * (256 / NW) + s * 16;
    const int ca = c0 + 4 * p;  // address column of this lane
    const int c = c0 + i;       // column delivered to this lane
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int r = t * 32 + g * 8;  // first of the lane's 8 rows
      const int l0 = (r + q) & 63, l1 = (r + 4 + q) & 63;
      const char* base = smem + qb[t >> 1] + (ca & 4) * 2;
      const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(base + l0 * 512 + (((ca >> 3) ^ (l0 & 15)) << 4)));
      const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(base + l1 * 512 + (((ca >> 3) ^ (l1 & 15)) << 4)));
      const bf16x8 v = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const uint32_t off = (c < cols && r < rows) ? (uint32_t)(((int64_t)c * ldt + r) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rt, (int)off, 0, AUX);
    }
  }
}

template <int EPI, bool FAST>
CC_DEV float pp_epilogue_lds(const GemmArgs& args, const f32x4 (&acc)[8][4], char* smem, const int (&qb)[4],
                            bool input_staged, int tm, int m0, int n0, int wr, int wc, int lane, int wave,
                            int wave_slot, const FragGeom<256>& fg, const EpiCols<CC_BF16, 256>& ecols,
                            const float (&cw)[8][4]) {
  const int rows = args.M - m0, cols = args.N - n0, ldo = (int)args.ldo;
  // the epilogue's input tile: d_acts' activation mask (the general form; FAST reads G1's mask bits instead),
  // the fused loss's x tile, dW_dec's W_dec tile (prefetched by the K loop)
  const void* in = (EPI == EPI_DACTS && !FAST) || EPI == EPI_DLOSS
                       ? args.mask_src
                       : (EPI == EPI_WGDEC && args.scale0 != 0.f ? args.w_src : nullptr);
  // (cw: dW_dec's L1-term factors, loaded by pp_tile under the K loop's drain; EPI_WGDEC's W_dec tile is
  // staged by the K loop too, so only the other epilogues' input tiles move here)
  if (in && !input_staged) {
    const __amdgpu_buffer_rsrc_t rin = tile_rsrc(in, args.ldo, m0, n0, args.M, args.N, 2);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ci = q * 8 + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void*)(smem + qb[q >> 2] + (ci & 31) * 1024), 16,
                                               (int)piece_off(ci, lane, rows, cols, ldo), 0, 0, 0);
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  }
  const LdsIO io(smem, qb, wr, wc, lane);
  const float wsum = epilogue_core<CC_BF16, EPI, 256, FAST>(args, acc, fg, io, tm, m0, n0, wr, lane, wave_slot, ecols,
                                                            cw);
  __syncthreads();
  PP_EPI_STAMP(args, wave_slot, 7);
  if (args.out) {
    const __amdgpu_buffer_rsrc_t rout = tile_rsrc(args.out, args.ldo, m0, n0, args.M, args.N, 2);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ci = q * 8 + wave;
      const bf16x8 v = *(const bf16x8*)(smem + qb[q >> 2] + (ci & 31) * 1024 + lane * 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout,
                                             (int)piece_off(ci, lane, rows, cols, ldo), 0,
                                             EPI == EPI_WGDEC || EPI == EPI_WGENC ? CC_EPI_STORE_WG_AUX : CC_EPI_STORE_AUX);
    }
  }
  PP_EPI_STAMP(args, wave_slot, 8);
  if (args.out_t)
    pp_store_transposed<EPI == EPI_ENC     ? CC_EPI_STORE_T_AUX_ENC
                        : EPI == EPI_DLOSS ? CC_EPI_STORE_T_AUX_DLOSS
                                           : CC_EPI_STORE_T_AUX>(args, smem, qb, m0, n0, rows, cols, lane, wave);
  PP_EPI_STAMP(args, wave_slot, 9);
  return wsum;
}

constexpr int PP_LDS = 4 * 256 * 128;  // 2 buffers x (A | B) K-step images
// + one 32 KB quarter of the W_dec tile, prefetched at tile start (dW_dec kernels: 160 KB in all)
constexpr int PP_LDS_W = PP_LDS + 256 * 128;

// One output tile of one GEMM; bid = the tile's block index within that GEMM's grid.  FAST: every tile
// of the launch lies inside the matrix and the ReLU is on (EPI_ENC / EPI_DACTS epilogue fast form).
// Returns the wave's squared-sum partial of a weight-gradient tile (epilogue_core), else 0.
template <bool AKC, bool BKC, int EPI, bool FAST = false>
CC_DEV float pp_tile(const GemmArgs& args, char* smem, int bid, int tid = threadIdx.x) {
  using WG = WaveGeom<256>;
  static_assert(WG::TM == 8 && WG::TN == 4, "ping-pong geometry");
  constexpr int TILE = 256 * 128;  // one operand's K-step image
  constexpr int BUF = 2 * TILE;

  PP_STAMP_DECL;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int tm, tn;
  tile_of_block(bid, args.nbm, args.nbn, tm, tn);
  const int m0 = tm * BM, n0 = tn * 256;
  const int M = args.M, N = args.N, K = args.K;

  __amdgpu_buffer_rsrc_t ra, rb;
  {
    const char* a = (const char*)args.A;
    const char* b = (const char*)args.B;
    if constexpr (AKC) {
      a += (int64_t)m0 * args.lda * 2;
      ra = make_rsrc(a, (uint64_t)(M - m0) * args.lda * 2);
    } else {
      a += (int64_t)m0 * 2;
      ra = make_rsrc(a, ((uint64_t)(K - 1) * args.lda + (M - m0)) * 2);
    }
    if constexpr (BKC) {
      b += (int64_t)n0 * args.ldb * 2;
      rb = make_rsrc(b, (uint64_t)(N - n0) * args.ldb * 2);
    } else {
      b += (int64_t)n0 * 2;
      rb = make_rsrc(b, ((uint64_t)(K - 1) * args.ldb + (N - n0)) * 2);
    }
  }

  // DMA offsets: vo[p][q] for the 4 phases x 2 DMAs (p 0,1: A; p 2,3: B)
  uint32_t vo[4][2];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      vo[p][q] = p < 2 ? pp_dma_off<AKC>(pp_ci(p, q, wave), M - m0, args.lda, lane)
                       : pp_dma_off<BKC>(pp_ci(p, q, wave), N - n0, args.ldb, lane);
  const int kA = pp_dma_k<AKC>(wave, lane), kB = pp_dma_k<BKC>(wave, lane);
  // this block's contraction steps (split-K passes run a slice of them)
  const int nk = args.k_steps ? args.k_steps : (K + 63) / 64;
  const int kb0 = args.k_step0;

  // dW_dec's epilogue input (the W_dec tile, 128 KB) is prefetched instead of loaded after the
  // loop: quarter 3 at tile start into the extra 32 KB of LDS, quarters 0-2 by the DMA slots of
  // the steps past the end (T >= nk), which would otherwise zero-fill regions the loop no longer
  // reads (buffer nk&1's B and A images, buffer (nk+1)&1's B image).
  const bool pf = EPI == EPI_WGDEC && args.scale0 != 0.f;
  const int erows = M - m0, ecols = N - n0, eldo = (int)args.ldo;
  __amdgpu_buffer_rsrc_t rw = ra;
  int qb[4] = {0, TILE, 2 * TILE, 3 * TILE};
  if (pf) {
    rw = tile_rsrc(args.w_src, args.ldo, m0, n0, M, N, 2);
    qb[0] = (nk & 1) * BUF + TILE;
    qb[1] = (nk & 1) * BUF;
    qb[2] = ((nk + 1) & 1) * BUF + TILE;
    qb[3] = 2 * BUF;
  }

  // issue phase p's DMAs for step T (target buffer T & 1)
  // tail: 1 = the step may lie past the end (prologue and the last two K steps only: the steady-state
  // loop stays free of the branch); 0 = steady state; 2 = steady state of a K % 64 == 0 contraction:
  // every lane's step lies inside K, so the K advance rides in the scalar offset (no per-DMA VALU)
  auto issue_t = [&](auto tail, int p, int T) {
    constexpr int TL = decltype(tail)::value;
    const bool isA = p < 2;
    const int k0 = (kb0 + T) * 64;
    char* dst = smem + (T & 1) * BUF + (isA ? 0 : TILE);
    if constexpr (TL == 2) {
      const int64_t ld = isA ? args.lda : args.ldb;
      const bool kc = isA ? AKC : BKC;
      const int kadd = (int)(kc ? (int64_t)k0 * 2 : (int64_t)k0 * ld * 2);
#pragma unroll
      for (int q = 0; q < 2; ++q)  // (vo[p][q] == OOB lanes stay past the record count)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? ra : rb, (lds_void*)(dst + pp_ci(p, q, wave) * 1024), 16,
                                                 (int)vo[p][q], kadd, 0, PP_OPERAND_AUX(EPI));
      return;
    }
    if (TL == 1 && pf && T >= nk) {  // W_dec quarter 0 (B, T = nk), 1 (A, T = nk) or 2 (B, T = nk + 1)
      const int quarter = isA ? 1 : (T == nk ? 0 : 2);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ci = pp_ci(p, q, wave);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(dst + ci * 1024), 16,
                                                 (int)piece_off(32 * quarter + ci, lane, erows, ecols, eldo), 0, 0, CC_WDEC_TILE_AUX);
      }
      return;
    }
    const int64_t ld = isA ? args.lda : args.ldb;
    const bool kc = isA ? AKC : BKC;
    const uint32_t kadd = (uint32_t)(kc ? (int64_t)k0 * 2 : (int64_t)k0 * ld * 2);
    const bool kin = k0 + (isA ? kA : kB) < K;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t v = vo[p][q];
      const uint32_t off = (kin && v != OOB) ? v + kadd : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? ra : rb, (lds_void*)(dst + pp_ci(p, q, wave) * 1024), 16,
                                               (int)off, 0, 0, PP_OPERAND_AUX(EPI));
    }
  };
  auto issue = [&](int p, int T) { issue_t(std::integral_constant<int, 1>{}, p, T); };

  // fragment lane offsets
  int kc_off[2], mn_off[4];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) kc_off[kk] = (lane & 15) * 128 + ((((lane >> 4) + 4 * kk) ^ (lane & 7)) << 4);
  {
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int kq = 8 * g + qq;
    const int h = pp_h(kq);
#pragma unroll
    for (int m = 0; m < 4; ++m) mn_off[m] = kq * 128 + (((2 * (m ^ h)) | (pp >> 1)) << 4) + 8 * (pp & 1);
  }

  f32x4 acc[WG::TM][WG::TN];
#pragma unroll
  for (int i = 0; i < WG::TM; ++i)
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: W_dec quarter 3 (retired with the first operand DMAs), then the DMAs steady state
  // would have issued in steps -2 and -1
  if (pf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ci = q * 8 + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(smem + qb[3] + ci * 1024), 16,
                                               (int)piece_off(96 + ci, lane, erows, ecols, eldo), 0, 0, CC_WDEC_TILE_AUX);
    }
  }
  issue(2, 0);
  issue(3, 0);
  issue(0, 0);
  issue(1, 0);
  issue(2, 1);
  issue(3, 1);
  wait_vmcnt<6>();
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs half a phase behind
  PP_STAMP(1);

  bf16x8 bfr[WG::TN][2];
  // One K step: four phases.
  auto kstep = [&](auto tail, int t) {
    const char* la = smem + (t & 1) * BUF;
    const char* lb = la + TILE;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      __builtin_amdgcn_sched_barrier(0);
      // phase p: A tiles 4*(p>>1) .. +3 x k-slice p&1; the B fragments of k-slice p&1 are read in
      // phase p&1 (B read load per phase 8/8/0/0 fragments instead of 16/0/0/0).  Every output
      // still accumulates k-slice 0 before k-slice 1 of a step (bitwise the same sums).
      const int kk = p & 1, ib = (p >> 1) * 4;
      if (p < 2) {
#pragma unroll
        for (int j = 0; j < WG::TN; ++j) {
          const int c0 = wc * WG::WTN + 16 * j;
          bfr[j][kk] = BKC ? pp_frag_kc(lb, c0, kc_off[kk]) : pp_frag_mn(lb, c0, kk, mn_off[(c0 >> 4) & 3]);
        }
      }
      bf16x8 afr[4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int r0 = wr * WG::WTM + 16 * (ib + ii);
        afr[ii] = AKC ? pp_frag_kc(la, r0, kc_off[kk]) : pp_frag_mn(la, r0, kk, mn_off[(r0 >> 4) & 3]);
      }
      issue_t(tail, p, p < 2 ? t + 1 : t + 2);
      wait_vmcnt<6>();
      // the B region of this buffer is re-staged in phase 2 (one phase after these reads): retire
      // them before this phase's first barrier (WAR across the staggered wave groups)
      if (p == 1) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < WG::TN; ++j)
          acc[ib + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], afr[ii], acc[ib + ii][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
  };
  int t = 0;
  // steady state: every DMA is an operand DMA
  if (K % 64 == 0)
    for (; t < nk - 2; ++t) kstep(std::integral_constant<int, 2>{}, t);
  else
    for (; t < nk - 2; ++t) kstep(std::integral_constant<int, 0>{}, t);
  for (; t < nk; ++t) kstep(std::integral_constant<int, 1>{}, t);  // last two steps: DMAs past the end prefetch W_dec
  if (wr == 0) __builtin_amdgcn_s_barrier();
  PP_STAMP(2);
  // the epilogue's column vectors fly while the last (zero-fill) DMAs drain
  const FragGeom<256> fg(args, m0, n0, wr, wc, lane);
  EpiCols<CC_BF16, 256> evec;
  if constexpr (EPI != EPI_F32 && EPI != EPI_DEC) load_epi_cols<CC_BF16, EPI, 256, FAST>(evec, args, fg, n0, tm, tn, tid);
  // dW_dec's L1-term factors: their loads fly with the drain too (after it they would cost the epilogue a
  // memory latency of their own)
  float cw[8][4];
  if constexpr (EPI == EPI_WGDEC) {
    if (pf) wgdec_factors<256>(args, fg, m0, n0, cw);
  }
  wait_vmcnt<0>();

  if constexpr (EPI == EPI_SPLIT) {  // split-K partial: accumulator fragments stored as they are (1 KB each)
    // slab tile index tm * nbn + tn (row-major over the tiles, whatever the block order)
    float* o = (float*)args.out + ((int64_t)(tm * args.nbn + tn) * 8 + wave) * 32 * 256;
#pragma unroll
    for (int i = 0; i < WG::TM; ++i)
#pragma unroll
      for (int j = 0; j < WG::TN; ++j) *(f32x4*)(o + ((i * 4 + j) * 64 + lane) * 4) = acc[i][j];
  } else if constexpr (EPI == EPI_F32 || EPI == EPI_DEC) {
    gemm_epilogue<CC_BF16, EPI, 256>(args, acc, tm, m0, n0, wr, wc, lane, bid * 8 + wave);
  } else {  // (the host routes N % 8 != 0 to gemm_kernel)
    __builtin_amdgcn_s_barrier();  // every wave's zero-fill DMAs landed: the LDS is free
    PP_STAMP(3);
    const float wsum = pp_epilogue_lds<EPI, FAST>(args, acc, smem, qb, pf, tm, m0, n0, wr, wc, lane, wave,
                                                  bid * 8 + wave, fg, evec, cw);
    PP_STAMP(4);
    PP_STAMP_WRITE(args, bid);
    return wsum;
  }
  return 0.f;
}

// Persistent tile loop: grid = min(tiles, CUs) workgroups; tile t of a launch belongs to XCD t % 8 (the
// bijective remap tile_of_block gives each XCD a contiguous block of the grouped tile order), and the
// workgroups of XCD x (blockIdx.x % 8 == x: the dispatcher's round-robin) run that XCD's tiles
// t = x + 8 i, i = 0, 1, ... (ntx of them) in order of i:
//   static (tile_ctr NULL): workgroup w of the XCD (w = blockIdx.x / 8) runs i = w, w + nwx, w + 2 nwx, ...
//   dynamic (tile_ctr = 8 u32 per-XCD counters): i = w first, then every further tile is claimed from the XCD's
//     counter, i = nwx + claim, until a claim runs past ntx.  A workgroup that starts late -- its CU held by
//     another stream's kernel (the side stream's, or RCCL's collective in the latent-sharded step) -- then
//     takes fewer tiles instead of delaying the launch by its whole static share.  Each launch makes exactly
//     ntx claims on counter x (every claim past the end is one workgroup's last), and atomicInc wraps at
//     ntx - 1, so the counter is back at 0 when the launch ends: no reset, but launches sharing a counter
//     must be ordered (one stream).  The claim for the next tile is issued as a tile starts (its latency hides
//     under the tile's first operand DMAs) and broadcast through an LDS word after the tile: buffer 1's A
//     image, which the next tile's DMAs first write after its prologue barrier.
// Which workgroup runs a tile does not change its results: every partial-sum slot is indexed by tile.
// Between tiles every wave's LDS reads of the epilogue image must be done before any wave's DMAs
// overwrite it: lgkmcnt(0) + s_barrier (no vmcnt wait: the stores keep draining, the next tile's first
// operand DMAs fly while they do).
CC_DEV void pp_tile_boundary() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}
// threadIdx.x as a value the compiler cannot prove loop-invariant: every per-lane offset of a tile is
// then computed inside the tile (hoisted out of the tile loop they would stay live through the K loop:
// ~45 more VGPRs, which also keep the side-stream kernels off the GEMM's SIMDs)
CC_DEV int pp_opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
constexpr int PP_SLOT = 2 * 256 * 128;  // LDS byte offset of the tile-claim broadcast word (see above)
struct TileLoop {
  unsigned* ctr;
  unsigned* wsync;  // probe only (cc_debug_set_wave_sync): static order, the XCD's waves of tiles start together
  int x, nwx, ntx, i;
  unsigned nxt;
  CC_DEV TileLoop(int nt, unsigned* c, unsigned* ws = nullptr) : ctr(c), wsync(ws), nxt(0) {
    const int G = gridDim.x;
    x = blockIdx.x & 7;
    nwx = (G >> 3) + ((G & 7) > x);
    ntx = (nt >> 3) + ((nt & 7) > x);
    i = blockIdx.x >> 3;
  }
  CC_DEV bool more() const { return i < ntx; }
  // the tile to run now (claims the next one in the dynamic order)
  CC_DEV int begin() {
    if (ctr && threadIdx.x == 0) nxt = atomicInc(ctr + x, (unsigned)(ntx - 1));
    return x + 8 * i;
  }
  // Probe of L2 panel reuse: every workgroup of the XCD finishes its tile of wave k before
  // any starts wave k + 1, so the XCD's concurrent tiles stream their shared A / B panels at the same K position.
  // Arrivals on the XCD's word (zeroed before the launch); the wait is bounded (~2 ms) so every wave exits.
  // The caller's barrier follows.
  CC_DEV void wave_wait() {
    if (threadIdx.x != 0) return;
    const unsigned k = (unsigned)(i / nwx);
    __hip_atomic_fetch_add(wsync + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i + nwx >= ntx) return;
    const unsigned target = min((k + 1) * (unsigned)nwx, (unsigned)ntx);
    for (int it = 0; it < (1 << 16); ++it) {
      if (__hip_atomic_load(wsync + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // after the tile and pp_tile_boundary(); slot_off: the broadcast word's LDS offset (the 4-wave q4 kernels keep it
  // past their K-loop images, whose next prologue writes all of them)
  CC_DEV void advance(char* smem, int slot_off = PP_SLOT) {
    if (!ctr) {
      if (wsync) wave_wait();
      i += nwx;
      return;
    }
    int* slot = (int*)(smem + slot_off);
    if (threadIdx.x == 0) *slot = (int)nxt;
    __syncthreads();
    i = nwx + __builtin_amdgcn_readfirstlane(*slot);
  }
};

// GemmArgs::wait_ctr: thread 0 polls the producer's counter (s_sleep between reads), then one agent-scope acquire
// (drops this XCD's stale L2 lines of the producer's output) and the barrier.  Bounded: every wave exits.  Returns
// false when the bound expired: the producer's output is not complete, so the caller runs NO tile of its own (it
// must not compute on a half-updated operand) and the host-visible error word is set -- the same step's host read
// raises, and the step's clip finaliser (ClipArgs::abort, the same word) keeps every Adam launch of the step from
// applying an update.
// (smem: the broadcast word is the tile-claim slot, PP_SLOT, which no DMA writes before the first tile's prologue
// barrier)
CC_DEV bool pp_wait_ready(const GemmArgs& a, char* smem, int slot_off = PP_SLOT) {
  if (!a.wait_ctr) return true;
  int& ok = *(int*)(smem + slot_off);
  if (threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();  // (the 100 MHz constant clock: the bound does not depend on sclk)
    int ready = 1;
    while ((int)(__hip_atomic_load(a.wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.wait_target) < 0) {
      if (wall_clock64() - t0 > 100000000ull) {  // (1 s)
        if (a.wait_err) __hip_atomic_store(a.wait_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ready = 0;
        break;
      }
      // ~0.6 us between reads: every workgroup of the launch polls the one word (at 0.25 us they would put
      // ~1 G atomic reads/s on it while the producer finishes)
      __builtin_amdgcn_s_sleep(20);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ok = ready;
  }
  __syncthreads();
  // every wave takes the word into a register before anyone may write PP_SLOT again (the abort path's tile claims
  // broadcast through it at once): the waves of the workgroup all take the same branch
  const bool r = __builtin_amdgcn_readfirstlane(ok) != 0;
  __syncthreads();
  return r;
}

// The launch's prologue reduction (GemmArgs::pre: reduce_rows' two phases, the same bits as cc_reduce_rows):
// 256-thread group g of workgroup b reduces column blocks 2b + g, 2b + g + 2 * grid, ... before b's first tile.
// A few workgroups start their tiles ~2 us late (the dynamic tile order evens that out); the step saves a launch.
// (nwg: the workgroups [0, nwg) that run it)
CC_DEV void pp_prologue_reduce(const GemmArgs& a, char* smem, int nwg) {
  if (a.pre_blocks <= 0) return;
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
  float(*red)[RED_COLS] = (float(*)[RED_COLS])(smem + grp * 4 * RED_COLS * sizeof(float));
  for (int base = 2 * (int)blockIdx.x; base < a.pre_blocks; base += 2 * nwg) {  // uniform per workgroup
    const int b = base + grp;
    if (b < a.pre_blocks) reduce_rows_phase1(a.pre, b, t, red);
    __syncthreads();
    if (b < a.pre_blocks) reduce_rows_phase2<CC_F32>(a.pre, b, t, red);
    __syncthreads();
  }
}

// The forward's loss tail as prologue work of the launch (GemmArgs::tail, tail_items > 0; LossTailArgs items,
// loss_tail.h): 256-thread group g of workgroup b runs items 2b + g, 2b + g + 2 P, ... (P participating
// workgroups); the participants then count arrivals and the last one runs the loss-scalar finaliser.  That
// workgroup starts its tiles ~10 us late; the dynamic tile order evens it out.  The step saves the side
// stream's loss-tail launch and the stream fork before it.
CC_DEV void pp_prologue_loss_tail(const GemmArgs& a, char* smem) {
  if (a.tail_items <= 0) return;
  const int np = min((int)gridDim.x, (a.tail_items + 1) / 2);
  if ((int)blockIdx.x >= np) return;  // (uniform per workgroup)
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
  float(*evred)[4] = (float(*)[4])(smem + grp * 64);
  for (int base = 2 * (int)blockIdx.x; base < a.tail_items; base += 2 * np) {
    const int item = base + grp;
    loss_tail_item(a.tail, item < a.tail_items ? item : -1, t, evred);
    __syncthreads();
  }
  int* last = (int*)(smem + 256);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const bool is_last = atomicAdd(a.tail.counter, 1u) == (unsigned)(np - 1);
    if (is_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *last = is_last;
  }
  __syncthreads();
  if (*last) {
    loss_scalars_body<LOSS_THREADS>(a.tail.scal, (double(*)[6])(smem + 512));
    if (threadIdx.x == 0) atomicExch(a.tail.counter, 0u);
  }
  __syncthreads();  // (the tiles reuse the LDS)
}

template <bool AKC, bool BKC, int EPI, bool FAST = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp_kernel(const GemmArgs args) {
  __shared__ __attribute__((aligned(16))) char smem[EPI == EPI_WGDEC ? PP_LDS_W : PP_LDS];
  pp_prologue_reduce(args, smem, gridDim.x);
  pp_prologue_loss_tail(args, smem);
  if (!pp_wait_ready(args, smem)) {
    // no tile runs, but the launch still makes its claims on the per-XCD counters (each launch leaves them at 0)
    for (TileLoop L(args.nbm * args.nbn, args.tile_ctr); L.more();) {
      L.begin();
      L.advance(smem);
      __syncthreads();
    }
    return;
  }
  for (TileLoop L(args.nbm * args.nbn, args.tile_ctr); L.more();) {
    pp_tile<AKC, BKC, EPI, FAST>(args, smem, L.begin(), pp_opaque_tid());
    pp_tile_boundary();
    L.advance(smem);
  }
}

// Two independent GEMMs of one layout in one launch: tiles [0, nb0) are a0's, the rest a1's (the tile loop and
// its counters are a0's).  dW_dec and dW_enc (1152 tiles each at config 2: 4.5 waves of 256 CUs apiece) become
// 2304 tiles = 9 full waves, and one kernel boundary disappears.
template <bool AKC, bool BKC, int EPI0, int EPI1>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp_dual_kernel(const GemmArgs a0, const GemmArgs a1) {
  __shared__ __attribute__((aligned(16))) char smem[EPI0 == EPI_WGDEC || EPI1 == EPI_WGDEC ? PP_LDS_W : PP_LDS];
  const int nb0 = a0.nbm * a0.nbn;
  for (TileLoop L(2 * nb0, a0.tile_ctr, a0.wave_sync); L.more();) {
    const int t = L.begin();
    const int tid = pp_opaque_tid();
    if (t < nb0) pp_tile<AKC, BKC, EPI0>(a0, smem, t, tid);
    else pp_tile<AKC, BKC, EPI1>(a1, smem, t - nb0, tid);
    pp_tile_boundary();
    L.advance(smem);
  }
}

// G2 as ONE launch: blocks [0, nb0) are the whole-wave main tiles (a0, epilogue EPI), the rest the
// split-K units of the leftover tiles (t, as gemm_pp_splitk_kernel).  The split units are dispatched
// as the first main tiles finish, instead of after the slowest one (the two-launch form waits for
// the whole main wave to drain at the kernel boundary).
template <bool AKC, bool BKC, int EPI, bool FAST = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp_main_splitk_kernel(const GemmArgs a0, const GemmArgs t,
                                                                    int steps_per, int nk_total,
                                                                    int64_t split_stride) {
  __shared__ __attribute__((aligned(16))) char smem[PP_LDS];
  const int nb0 = a0.nbm * a0.nbn;
  if ((int)blockIdx.x < nb0) {
    pp_prologue_reduce(a0, smem, nb0);
    if (pp_wait_ready(a0, smem)) pp_tile<AKC, BKC, EPI, FAST>(a0, smem, blockIdx.x);
    return;
  }
  if (!pp_wait_ready(t, smem)) return;
  const int b = blockIdx.x - nb0;
  const int s = b / (t.nbm * t.nbn);
  const int tb = b - s * t.nbm * t.nbn;
  GemmArgs a = t;
  a.k_step0 = s * steps_per;
  a.k_steps = nk_total - a.k_step0 < steps_per ? nk_total - a.k_step0 : steps_per;
  a.out = (float*)t.out + s * split_stride;
  pp_tile<AKC, BKC, EPI_SPLIT>(a, smem, tb);
}

// Split-K pass (fp32 partial tiles, no epilogue work): block b runs contraction slice
// s = b / ntiles (steps [s * steps_per, ...)) of tile b % ntiles and stores its fp32 partial tile
// (accumulator-fragment order, EPI_SPLIT) at out + s * split_stride.  Used for the tiles left over after the whole 256-tile waves of a
// launch, so the leftover costs ~1/S of a wave instead of a full one; cc_reduce_splits sums them.
template <bool AKC, bool BKC>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp_splitk_kernel(const GemmArgs args, int steps_per, int nk_total,
                                                               int64_t split_stride) {
  __shared__ __attribute__((aligned(16))) char smem[PP_LDS];
  // split s = b / ntiles: consecutive blocks share a contraction slice (measured 64 us per block at
  // config 2, vs 80-134 us with each split pinned to one XCD: s = b % 8)
  const int s = blockIdx.x / (args.nbm * args.nbn);
  const int tb = blockIdx.x - s * args.nbm * args.nbn;
  if (!pp_wait_ready(args, smem)) return;
  GemmArgs a = args;
  a.k_step0 = s * steps_per;
  a.k_steps = nk_total - a.k_step0 < steps_per ? nk_total - a.k_step0 : steps_per;
  a.out = (float*)args.out + s * split_stride;
  pp_tile<AKC, BKC, EPI_SPLIT>(a, smem, tb);
}
