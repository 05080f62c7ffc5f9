// GEMM epilogues (included by gemm.hip inside namespace cc, after WaveGeom / V4 / EPB).
//
// Accumulator map (transposed C fragments): acc[i][j][e] = C[m0 + r0 + 16i][n0 + c0 + 16j + e]
// with r0 = wr*WTM + (lane & 15), c0 = wc*WTN + 4*(lane >> 4).
//
// The element-wise work of each epilogue is written once (epilogue_core) against an IO policy
// that supplies the tile-shaped input operand of the epilogue (the activation mask of d_acts,
// W_dec for dW_dec) and takes the dtype output, fragment by fragment:
//   RegIO -- straight from/to HBM through buffer descriptors anchored at the tile origin: a row
//            or column past the matrix edge gets an out-of-range offset (load 0, store dropped),
//            so there is no branch per fragment (a branch around each load makes the compiler
//            wait for that load by itself: one memory latency per fragment).
//   LdsIO  -- (gemm_pp.h) a swizzled LDS image of the tile, staged in and out with full-line
//            transfers.
// N % 4 == 0 (host check): a lane's 4 columns are all in range or all out.

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// descriptor over a row-major [rows][ld] matrix of element size es, anchored at (m0, n0)
CC_DEV __amdgpu_buffer_rsrc_t tile_rsrc(const void* p, int64_t ld, int m0, int n0, int M, int N, int es) {
  const char* base = (const char*)p + ((int64_t)m0 * ld + n0) * es;
  return make_rsrc(base, (uint64_t)(((int64_t)(M - m0 - 1) * ld + (N - n0)) * es));
}
// descriptor over a vector starting at element i0 with n elements
CC_DEV __amdgpu_buffer_rsrc_t vec_rsrc(const void* p, int i0, int64_t n, int es) {
  return make_rsrc((const char*)p + (int64_t)i0 * es, (uint64_t)(n - i0) * es);
}

template <int DT> CC_DEV typename V4<DT>::T bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (DT == CC_BF16) return __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
  else return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
template <int DT> CC_DEV typename V4<DT>::T pack4(const float v[4]) {
  if constexpr (DT == CC_BF16) {
    bf16x4 p;
#pragma unroll
    for (int e = 0; e < 4; ++e) p[e] = (short)f2bf(v[e]);
    return p;
  } else {
    return f32x4{v[0], v[1], v[2], v[3]};
  }
}
template <int DT> CC_DEV void bst4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float v[4]) {
  if constexpr (DT == CC_BF16)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pack4<DT>(v)), r, (int)off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pack4<DT>(v)), r, (int)off, 0, 0);
}
CC_DEV float bldf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// Fragment geometry of one wave's sub-tile: range flags and tile-relative element offsets.
template <int BNT>
struct FragGeom {
  using WG = WaveGeom<BNT>;
  int r0, c0, ldo;
  bool rv[WG::TM], cv[WG::TN];
  CC_DEV FragGeom(const GemmArgs& args, int m0, int n0, int wr, int wc, int lane) {
    r0 = wr * WG::WTM + (lane & 15);
    c0 = wc * WG::WTN + 4 * (lane >> 4);
    ldo = (int)args.ldo;
#pragma unroll
    for (int i = 0; i < WG::TM; ++i) rv[i] = m0 + r0 + 16 * i < args.M;
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) cv[j] = n0 + c0 + 16 * j < args.N;
  }
  CC_DEV bool ok(int i, int j) const { return rv[i] && cv[j]; }
  // byte offset of fragment (i, j) in a tile-anchored [.][ldo] matrix of element size es, or OOB
  CC_DEV uint32_t boff(int i, int j, int es) const {
    return ok(i, j) ? (uint32_t)(((r0 + 16 * i) * ldo + c0 + 16 * j) * es) : OOB;
  }
};

// HBM IO policy: input = mask_src (DACTS) / w_src (WGDEC), output = out, both indexed like out.
template <int DT, int BNT>
struct RegIO {
  const FragGeom<BNT>& fg;
  __amdgpu_buffer_rsrc_t rin, rout;
  static constexpr int ES = DT == CC_BF16 ? 2 : 4;
  CC_DEV RegIO(const GemmArgs& args, const FragGeom<BNT>& g, const void* in, int m0, int n0) : fg(g) {
    rout = tile_rsrc(args.out, args.ldo, m0, n0, args.M, args.N, ES);
    rin = tile_rsrc(in ? in : args.out, args.ldo, m0, n0, args.M, args.N, ES);
  }
  CC_DEV typename V4<DT>::T in4(int i, int j) const { return bld4<DT>(rin, fg.boff(i, j, ES)); }
  CC_DEV void out4(int i, int j, const float v[4]) const { bst4<DT>(rout, fg.boff(i, j, ES), v); }
  CC_DEV void out4p(int i, int j, bf16x4 p) const {  // (bf16 only) already-converted outputs
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, p), rout, (int)fg.boff(i, j, 2), 0, 0);
  }
};

// Per-fragment factor of dW_dec's L1 term: (l1_scale * sum_b acts[b, row]) * (1 / ||W_dec[row, model]||),
// 0 outside the matrix.  All 8 + 32 loads are issued before any is used (one memory latency for
// the lot; the LDS-staged epilogue issues them beside its W_dec tile DMA).
template <int BNT>
CC_DEV void wgdec_factors(const GemmArgs& args, const FragGeom<BNT>& fg, int m0, int n0,
                          float (&cw)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN]) {
  using WG = WaveGeom<BNT>;
  const __amdgpu_buffer_rsrc_t rnorm = vec_rsrc(args.norms, m0 * args.n_models, (int64_t)args.M * args.n_models, 4);
  const __amdgpu_buffer_rsrc_t rcol = vec_rsrc(args.colsum, m0, args.M, 4);
  float cs[WG::TM];
#pragma unroll
  for (int i = 0; i < WG::TM; ++i) cs[i] = bldf(rcol, fg.rv[i] ? (uint32_t)((fg.r0 + 16 * i) * 4) : OOB);
#pragma unroll
  for (int j = 0; j < WG::TN; ++j) {
    const int model = (n0 + fg.c0 + 16 * j) / args.d_model;
#pragma unroll
    for (int i = 0; i < WG::TM; ++i)
      cw[i][j] = bldf(rnorm, fg.ok(i, j) ? (uint32_t)(((fg.r0 + 16 * i) * args.n_models + model) * 4) : OOB);
  }
#pragma unroll
  for (int i = 0; i < WG::TM; ++i) {
    const float c = args.scale0 * cs[i];
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) cw[i][j] = c * cw[i][j];
  }
}

// The element-wise part of EPI_ENC / EPI_DACTS / EPI_WGDEC / EPI_WGENC over one wave's fragments.
// Per-column epilogue vectors of a wave's TN column groups (b_enc for EPI_ENC, the total decoder
// norm tn for EPI_ENC / EPI_DACTS), loaded by the caller ahead of the epilogue with no branch
// around any load (absent vectors read as 0 through out-of-range offsets): one memory latency for
// all of them, overlapped with whatever the caller waits on next.
template <int DT, int BNT>
struct EpiCols {
  typename V4<DT>::T bias[WaveGeom<BNT>::TN];
  f32x4 tn[WaveGeom<BNT>::TN];
  u32x4 bits;  // EPI_DACTS FAST: this thread's activation-mask bits (mask_bits)
  CC_DEV void load(const GemmArgs& args, const FragGeom<BNT>& fg, int n0, bool want_bias) {
    constexpr int ES = DT == CC_BF16 ? 2 : 4;
    const __amdgpu_buffer_rsrc_t rbias = vec_rsrc(want_bias ? args.bias : args.A, n0, args.N, ES);
    const __amdgpu_buffer_rsrc_t rtn = vec_rsrc(args.tn ? (const void*)args.tn : args.A, n0, args.N, 4);
#pragma unroll
    for (int j = 0; j < WaveGeom<BNT>::TN; ++j) {
      const uint32_t cvo = (uint32_t)(fg.c0 + 16 * j);
      bias[j] = bld4<DT>(rbias, want_bias ? cvo * ES : OOB);
      tn[j] = bld4<CC_F32>(rtn, args.tn ? cvo * 4 : OOB);
    }
  }
};
// 16 B of this thread's mask bits in the [tile][thread][4] u32 layout (mask_bits)
CC_DEV uint32_t* mask_bits_at(const GemmArgs& args, int tm, int tn, int tid) {
  return args.mask_bits + ((int64_t)(tm * args.nbn + tn) * 512 + tid) * 4;
}
template <int DT, int EPI, int BNT, bool FAST = false>
CC_DEV void load_epi_cols(EpiCols<DT, BNT>& c, const GemmArgs& args, const FragGeom<BNT>& fg, int n0, int tm = 0,
                          int tn = 0, int tid = 0) {
  if constexpr (EPI == EPI_ENC || EPI == EPI_DACTS) c.load(args, fg, n0, EPI == EPI_ENC && args.bias);
  if constexpr (EPI == EPI_DACTS && FAST) c.bits = *(const u32x4*)mask_bits_at(args, tm, tn, tid);
  if constexpr (EPI == EPI_DLOSS) c.load(args, fg, n0, true);  // b_dec, x_mean
}

// Tile-anatomy probe points inside the epilogue (-DCC_PP_STAMPS builds, see gemm_pp.h): s_memtime into slot k
// of the tile's 12, stored at once -- after the K loop, outside its counted waits.
#ifdef CC_PP_STAMPS
#define PP_EPI_STAMP(args, wave_slot, k)                                                       \
  do {                                                                                        \
    if ((args).stamps && threadIdx.x == 0)                                                    \
      (args).stamps[(int64_t)((wave_slot) >> 3) * 12 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define PP_EPI_STAMP(args, wave_slot, k)
#endif

// Activation-mask bit of output (i, j, e) of a lane's 32 fragments (EPI_ENC writes them, EPI_DACTS FAST reads
// them; 4 words per thread): word i / 2, bit k = 8 (i % 2) + 2j + e / 2 for the first element of the bf16 pair
// e / 2 and k + 16 for the second -- a pair's two bits are one pk_min_u16(pair, 1) shifted left by k.
CC_DEV constexpr int mask_bit_pos(int i, int j, int e) { return 8 * (i & 1) + 2 * j + (e >> 1) + 16 * (e & 1); }

// EPI_ENC, FAST, bf16 (the step's G1): per bf16 pair -- the ReLU on the rounded pair (v_pk_max_i16 against 0:
// a negative bf16 is a negative int16; max(round(t), 0) == round(max(t, 0)) bit for bit), the mask bits by one
// pk_min_u16(pair, 1) or-ed into the pair's word, the l0 count as the popcount of the bits, the column sums of
// the stored values in pairs.  The same outputs as enc_dacts_core's general arithmetic with half its VALU
// instructions.  NaN pre-activations are the exception, and their sign decides: a NaN with the sign bit clear is a
// positive int16, so it stays NaN (as torch.relu keeps every NaN) and sets its mask bit; a NaN with the sign bit set
// is a negative int16 and becomes +0 (mask bit clear), as the general form's fmaxf turns every NaN into 0.  Neither
// form matches torch for every NaN; a NaN pre-activation means the step's inputs or weights are already non-finite
// (the reference then trains on NaN too), and no fixture pins it.
template <int BNT, class IO>
CC_DEV void enc_fast_core(const GemmArgs& args, const f32x4 (&acc)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN],
                          const FragGeom<BNT>& fg, const IO& io, int tm, int n0, int wr, int lane, int wave_slot,
                          const EpiCols<CC_BF16, BNT>& cols) {
  using WG = WaveGeom<BNT>;
  static_assert(WG::TM == 8 && WG::TN == 4, "mask bits: 32 fragments");
  uint32_t bw[4] = {0u, 0u, 0u, 0u};
  const uint32_t ones = 0x00010001u;
#pragma unroll
  for (int j = 0; j < WG::TN; ++j) {
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    const f32x2 bb[2] = {{V4<CC_BF16>::get(cols.bias[j], 0), V4<CC_BF16>::get(cols.bias[j], 1)},
                         {V4<CC_BF16>::get(cols.bias[j], 2), V4<CC_BF16>::get(cols.bias[j], 3)}};
    f32x2 cs[2] = {{0.f, 0.f}, {0.f, 0.f}};  // (e 0, 1 | e 2, 3: packed adds, the per-element order unchanged)
#pragma unroll
    for (int i = 0; i < WG::TM; ++i) {
      uint32_t w[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 t = (f32x2){acc[i][j][2 * h], acc[i][j][2 * h + 1]} + bb[h];  // (packed fp32 adds)
        const float t0 = t[0], t1 = t[1];
        // (single instructions on purpose: the vector-typed forms lowered to compares and selects)
        uint32_t pr, r, pos;
        asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(pr) : "v"(t0), "v"(t1));  // RNE, as f2bf
        asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(pr));
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(pos) : "v"(r), "s"(ones));
        w[h] = r;
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(bw[i >> 1]) : "v"(pos), "i"(mask_bit_pos(i, j, 2 * h)), "v"(bw[i >> 1]));
        cs[h] += (f32x2){__uint_as_float(r << 16), __uint_as_float(r & 0xffff0000u)};
      }
      io.out4p(i, j, __builtin_bit_cast(bf16x4, (u32x2){w[0], w[1]}));
    }
    if (args.col_part) {  // reduce over the 16 lanes (rows) that share these 4 columns
      float csum[4] = {cs[0][0], cs[0][1], cs[1][0], cs[1][1]};
      row16_sum4(csum);
      if ((lane & 15) == 0 && fg.cv[j])
        st4<CC_F32>(args.col_part, (int64_t)(tm * WG::WARPS_M + wr) * args.N + n0 + fg.c0 + 16 * j, csum);
    }
  }
  PP_EPI_STAMP(args, wave_slot, 10);
  if (args.mask_bits)
    *(u32x4*)mask_bits_at(args, tm, n0 / BNT, wave_slot % 8 * 64 + lane) = u32x4{bw[0], bw[1], bw[2], bw[3]};
  if (args.wave_part1) {
    const int l0i = __builtin_popcount(bw[0]) + __builtin_popcount(bw[1]) + __builtin_popcount(bw[2]) +
                    __builtin_popcount(bw[3]);
    // (integer-valued floats below 2^24: the per-lane counts sum exactly either way)
    float t = wave_sum((float)l0i);
    if (lane == 0) args.wave_part1[wave_slot] = t;
  }
  PP_EPI_STAMP(args, wave_slot, 11);
}

// EPI_ENC / EPI_DACTS element-wise part (see epilogue_core).  FAST (bf16): every fragment in range, ReLU on.
// Activation mask (EPI_DACTS): FAST reads G1's mask bits (cols.bits, no mask tile), the general form the
// acts tile through io.in4.  EPI_ENC writes the bits (args.mask_bits, ping-pong path) for the d_acts GEMM
// of the same tile grid and wave / lane map: bit mask_bit_pos(i, j, e) of word i / 2 <-> acc[i][j][e].
template <int DT, int EPI, int BNT, bool FAST, class IO>
CC_DEV void enc_dacts_core(const GemmArgs& args, const f32x4 (&acc)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN],
                           const FragGeom<BNT>& fg, const IO& io, int tm, int n0, int wr, int lane, int wave_slot,
                           const EpiCols<DT, BNT>& cols) {
#pragma clang fp contract(off)  // (acc + tn * l1_scale: two roundings in every variant; the l1 sum fuses)
  static_assert(!(EPI == EPI_DACTS && FAST) || WaveGeom<BNT>::TM * WaveGeom<BNT>::TN == 32, "mask bits: 32 fragments");
  uint32_t bw[4] = {0u, 0u, 0u, 0u};  // EPI_ENC: the mask bits being formed
  using E = Elem<DT>;
  using WG = WaveGeom<BNT>;
  const int N = args.N;
  constexpr int JB = EPB<DT, BNT>::JB_M;
  float s_l1 = 0.f;
  int l0i = 0;  // this lane's count of positive outputs
  typename V4<DT>::T mraw[EPI == EPI_DACTS ? WG::TM : 1][JB];
#pragma unroll
  for (int j = 0; j < WG::TN; ++j) {
    if constexpr (EPI == EPI_DACTS && !FAST) {
      if (j % JB == 0) {  // the mask vectors of JB column groups, all in flight together
#pragma unroll
        for (int jj = 0; jj < JB; ++jj)
#pragma unroll
          for (int i = 0; i < WG::TM; ++i) mraw[i][jj] = io.in4(i, j + jj);
      }
    }
    float add[4], tnc[4], csum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr (EPI == EPI_ENC) {
        add[e] = V4<DT>::get(cols.bias[j], e);
        tnc[e] = cols.tn[j][e];
      } else {
        add[e] = cols.tn[j][e] * args.scale0;
        tnc[e] = 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < WG::TM; ++i) {
      const bool ok = FAST || fg.ok(i, j);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][j][e] + add[e];
        if constexpr (EPI == EPI_ENC) {
          if (FAST || args.flag) t = fmaxf(t, 0.f);
        } else if constexpr (FAST) {  // (mask_bit_pos)
          // (the bit sign-extended to an all-ones / zero mask, opaque so that it stays two VALU ops instead of
          // a compare + select per element)
          int m;
          asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(cols.bits[i >> 1]), "i"(mask_bit_pos(i, j, e)));
          t = __int_as_float(__float_as_int(t) & m);
        } else {
          t = V4<DT>::get(mraw[i][j % JB], e) > 0.f ? t : 0.f;
        }
        v[e] = FAST ? t : (ok ? E::round(t) : 0.f);
      }
      if constexpr (FAST) {
        const bf16x4 p = pack4<CC_BF16>(v);  // the bf16 rounding, once
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = V4<CC_BF16>::get(p, e);
        io.out4p(i, j, p);
      } else {
        io.out4(i, j, v);
      }
      uint32_t nib = 0u;  // EPI_ENC: this fragment's 4 mask bits (at bits 0, 16, 1, 17)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        csum[e] += v[e];
        if constexpr (EPI == EPI_ENC) {
          if constexpr (!FAST) s_l1 = __builtin_fmaf(v[e], tnc[e], s_l1);  // (FAST: no l1 partials, host)
          // v > 0 as an integer 0 / 1: med3(bits of v, 0, 1), opaque so that it is not turned back into
          // compares, whose 128 lane masks would sit in SGPRs until their later uses and spill
          int pos;
          if constexpr (FAST) asm("v_med3_i32 %0, %1, 0, 1" : "=v"(pos) : "v"(__float_as_int(v[e])));
          else pos = v[e] > 0.f;  // (the general form: its range selects need the compares anyway)
          l0i += pos;
          nib |= (uint32_t)pos << ((e >> 1) + 16 * (e & 1));  // (mask_bit_pos within the fragment)
        }
      }
      if constexpr (EPI == EPI_ENC) bw[i >> 1] |= nib << mask_bit_pos(i, j, 0);
    }
    if (args.col_part) {  // reduce over the 16 lanes (rows) that share these 4 columns
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[e] = row16_sum(csum[e]);
      if ((lane & 15) == 0 && fg.cv[j])
        st4<CC_F32>(args.col_part, (int64_t)(tm * WG::WARPS_M + wr) * N + n0 + fg.c0 + 16 * j, csum);
    }
  }
  if constexpr (EPI == EPI_ENC) {
    if constexpr (WG::TM * WG::TN == 32) {
      if (args.mask_bits)
        *(u32x4*)mask_bits_at(args, tm, n0 / BNT, wave_slot % 8 * 64 + lane) = u32x4{bw[0], bw[1], bw[2], bw[3]};
    }
    if (args.wave_part0) {
      float t = wave_sum(s_l1);
      if (lane == 0) args.wave_part0[wave_slot] = t;
    }
    if (args.wave_part1) {
      // (integer-valued floats below 2^24: the per-lane counts sum exactly either way)
      float t = wave_sum((float)l0i);
      if (lane == 0) args.wave_part1[wave_slot] = t;
    }
  }
}

// EPI_DLOSS (bf16, ping-pong LDS epilogue only): G2's reconstruction loss + its gradient on a whole-
// contraction tile (crosscoder.py:104-121 and the autograd of :104-106), the arithmetic of loss_kernel:
//   diff = (recon + b_dec) - x;  g_recon = bf16(grad_scale * diff)   (the same bits as loss_kernel)
//   row terms l2 = sum diff^2, tv = sum (x - x_mean)^2 per row and 64-column wave block
//   column sums of g_recon per 128-row wave half (the b_dec gradient's partial rows)
// io.in4 = the x tile (staged in LDS), io.out4p writes g_recon in place; cols.bias = b_dec,
// cols.tn = x_mean.  Row terms go to row_part[2][n * d/64][B] (d % 64 == 0: a wave's 64 columns lie in
// one model); rows past M are masked (FAST: every row of the launch is inside the matrix).
template <int BNT, bool FAST, class IO>
CC_DEV void dloss_core(const GemmArgs& args, const f32x4 (&acc)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN],
                       const FragGeom<BNT>& fg, const IO& io, int tm, int m0, int n0, int wr, int lane,
                       const EpiCols<CC_BF16, BNT>& cols) {
  using WG = WaveGeom<BNT>;
  const float gs = args.scale0;
  // rows outer (a row's terms complete after its 4 column groups: 2 live sums instead of 16)
  float csum[WG::TN][4];
#pragma unroll
  for (int j = 0; j < WG::TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[j][e] = 0.f;
  const int gc = n0 + fg.c0 - 4 * (lane >> 4);  // first column of this wave's 64-column block
  const int d = args.d_model, ncb = d / 64, B = args.M;
  const int m = gc / d, cb = (gc - m * d) / 64;
  float* rp = args.row_part + (int64_t)(m * ncb + cb) * B;
  const int64_t plane = (int64_t)args.n_models * ncb * B;
  const bool rows_out = lane < 16 && gc < args.N;
#pragma unroll
  for (int i = 0; i < WG::TM; ++i) {
    float l2 = 0.f, tv = 0.f;
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) {
      const bf16x4 xr = io.in4(i, j);
      float g[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xv = V4<CC_BF16>::get(xr, e);
        const float diff = (acc[i][j][e] + V4<CC_BF16>::get(cols.bias[j], e)) - xv;
        l2 += diff * diff;
        const float c = xv - cols.tn[j][e];
        tv += c * c;
        g[e] = gs * diff;
      }
      const bf16x4 p = pack4<CC_BF16>(g);  // the bf16 rounding, once
      io.out4p(i, j, p);
      if (FAST || fg.rv[i]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) csum[j][e] += V4<CC_BF16>::get(p, e);
      }
    }
    // the row's terms: sum over the 4 lane groups that hold its 64 columns
    l2 += __shfl_xor(l2, 16, 64);
    l2 += __shfl_xor(l2, 32, 64);
    tv += __shfl_xor(tv, 16, 64);
    tv += __shfl_xor(tv, 32, 64);
    const int r = m0 + fg.r0 + 16 * i;
    if (rows_out && (FAST || r < B)) {
      rp[r] = l2;
      rp[plane + r] = tv;
    }
  }
  if (args.col_part) {  // reduce over the 16 lanes (rows) that share these 4 columns
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[j][e] = row16_sum(csum[j][e]);
      if ((lane & 15) == 0 && fg.cv[j])
        st4<CC_F32>(args.col_part, (int64_t)(tm * WG::WARPS_M + wr) * args.ldo + n0 + fg.c0 + 16 * j, csum[j]);
    }
  }
}

// cols: EpiCols loaded by the caller (EPI_ENC / EPI_DACTS; otherwise unread).
// cw: dW_dec L1-term factors loaded by the caller (wgdec_factors; EPI_WGDEC with l1_scale != 0
// only, otherwise unread).  Passed by reference so they stay in registers.
// Returns the wave's squared-sum partial of a weight-gradient tile (what it stores at wave_part0[wave_slot],
// every lane), 0 for the other epilogues.
template <int DT, int EPI, int BNT, bool FAST = false, class IO>
CC_DEV float epilogue_core(const GemmArgs& args, const f32x4 (&acc)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN],
                          const FragGeom<BNT>& fg, const IO& io, int tm, int m0, int n0, int wr, int lane,
                          int wave_slot, const EpiCols<DT, BNT>& cols,
                          const float (&cw)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN]) {
  using E = Elem<DT>;
  using WG = WaveGeom<BNT>;
  if constexpr (EPI == EPI_ENC || EPI == EPI_DACTS) {
    // FAST (a kernel variant the host picks when every tile lies inside the matrix and the ReLU is on,
    // as in the step's G1 / G3): no range selects, one bf16 conversion per output, an integer l0
    // count.  Same bits as the general form.
    if constexpr (EPI == EPI_ENC && FAST && DT == CC_BF16 && BNT == 256)
      enc_fast_core<BNT>(args, acc, fg, io, tm, n0, wr, lane, wave_slot, cols);
    else
      enc_dacts_core<DT, EPI, BNT, FAST && DT == CC_BF16>(args, acc, fg, io, tm, n0, wr, lane, wave_slot, cols);
  } else if constexpr (EPI == EPI_DLOSS) {
    static_assert(DT == CC_BF16, "the fused decode + loss epilogue is bf16 only");
    dloss_core<BNT, FAST>(args, acc, fg, io, tm, m0, n0, wr, lane, cols);
  } else if constexpr (EPI == EPI_WGDEC || EPI == EPI_WGENC) {
    constexpr int JB = EPB<DT, BNT>::JB_W;
    const bool l1term = EPI == EPI_WGDEC && args.scale0 != 0.f;
    float sq = 0.f;
    float sqe[4] = {0.f, 0.f, 0.f, 0.f};  // (bf16: one partial per element position, summed at the end)
    typename V4<DT>::T wraw[EPI == EPI_WGDEC ? WG::TM : 1][JB];
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) {
      if constexpr (EPI == EPI_WGDEC) {
        if (l1term && j % JB == 0) {
#pragma unroll
          for (int jj = 0; jj < JB; ++jj)
#pragma unroll
            for (int i = 0; i < WG::TM; ++i) wraw[i][jj] = io.in4(i, j + jj);
        }
      }
#pragma unroll
      for (int i = 0; i < WG::TM; ++i) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e];
        if constexpr (EPI == EPI_WGDEC) {
          if (l1term) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += cw[i][j] * V4<DT>::get(wraw[i][j % JB], e);
          }
        }
        // out-of-range fragments are exactly 0 (zero-filled operands and inputs): no range selects
        if constexpr (DT == CC_BF16) {
          const bf16x4 p = pack4<CC_BF16>(v);  // the bf16 rounding, once (the stored bits)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = V4<CC_BF16>::get(p, e);
            sqe[e] = __builtin_fmaf(r, r, sqe[e]);
          }
          io.out4p(i, j, p);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = E::round(v[e]);
            sq += v[e] * v[e];
          }
          io.out4(i, j, v);
        }
      }
    }
    if constexpr (DT == CC_BF16) sq = (sqe[0] + sqe[1]) + (sqe[2] + sqe[3]);
    if (args.wave_part0) {
      float t = wave_sum(sq);
      if (lane == 0) args.wave_part0[wave_slot] = t;
      return t;
    }
  }
  return 0.f;
}

template <int DT, int EPI, int BNT>
CC_DEV void gemm_epilogue(const GemmArgs& args, const f32x4 (&acc)[WaveGeom<BNT>::TM][WaveGeom<BNT>::TN], int tm,
                          int m0, int n0, int wr, int wc, int lane, int wave_slot) {
  using WG = WaveGeom<BNT>;
  constexpr int ES = DT == CC_BF16 ? 2 : 4;
  const FragGeom<BNT> fg(args, m0, n0, wr, wc, lane);
  if constexpr (EPI == EPI_F32 || EPI == EPI_DEC) {
    const __amdgpu_buffer_rsrc_t ro32 = tile_rsrc(EPI == EPI_F32 ? args.out : (const void*)args.out_f32, args.ldo,
                                                  m0, n0, args.M, args.N, 4);
    const __amdgpu_buffer_rsrc_t rot = tile_rsrc(args.out, args.ldo, m0, n0, args.M, args.N, ES);
    const bool has_bias = EPI == EPI_DEC && args.bias;
    const __amdgpu_buffer_rsrc_t rbias = vec_rsrc(has_bias ? args.bias : args.A, n0, args.N, ES);
#pragma unroll
    for (int j = 0; j < WG::TN; ++j) {
      float bc[4] = {0.f, 0.f, 0.f, 0.f};
      if (has_bias) {
        const auto b = bld4<DT>(rbias, (uint32_t)((fg.c0 + 16 * j) * ES));
#pragma unroll
        for (int e = 0; e < 4; ++e) bc[e] = V4<DT>::get(b, e);
      }
#pragma unroll
      for (int i = 0; i < WG::TM; ++i) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bc[e];
        if constexpr (EPI == EPI_F32) {
          bst4<CC_F32>(ro32, fg.boff(i, j, 4), v);
        } else {
          if (args.out_f32) bst4<CC_F32>(ro32, fg.boff(i, j, 4), v);
          if (args.out) bst4<DT>(rot, fg.boff(i, j, ES), v);
        }
      }
    }
  } else {
    const void* in = EPI == EPI_DACTS ? args.mask_src : (EPI == EPI_WGDEC ? args.w_src : nullptr);
    const RegIO<DT, BNT> io(args, fg, in, m0, n0);
    float cw[WG::TM][WG::TN];
    if constexpr (EPI == EPI_WGDEC) {
      if (args.scale0 != 0.f) wgdec_factors<BNT>(args, fg, m0, n0, cw);
    }
    EpiCols<DT, BNT> cols;
    load_epi_cols<DT, EPI, BNT>(cols, args, fg, n0);
    epilogue_core<DT, EPI, BNT>(args, acc, fg, io, tm, m0, n0, wr, lane, wave_slot, cols, cw);
  }
}
