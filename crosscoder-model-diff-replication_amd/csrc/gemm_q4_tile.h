// The 4-wave GEMM (gemm_q4.h's assembly K loop) with the ping-pong's epilogues, as persistent tile-loop launches
// (included by gemm.hip after gemm_pp.h, inside namespace cc).
//
// A q4 wave (wr, wc) holds the outputs of two ping-pong waves, (wr, 2 wc) and (wr, 2 wc + 1) -- its accumulator
// columns 0-3 and 4-7 -- so every epilogue runs unchanged on each of the two halves ("virtual waves", with the
// ping-pong wave's index in every slot it writes: column-sum rows, l0 / squared-sum partials, mask-bit words), and
// the K loop accumulates in the ping-pong's order: each output, partial and bit equals the ping-pong launch's.  The
// workgroups are 256 threads; the launch-level jobs (prologue reductions, the loss tail, tile claims) are the
// ping-pong kernel's with one 256-thread group per workgroup.
#pragma once
#include "gemm_q4.h"

constexpr int Q4_SLOT = Q4_LDS;        // tile-claim / wait broadcast word: past the K-loop images, which the next
                                       // tile's prologue DMAs rewrite before its first barrier
constexpr int Q4_LDS_ALL = Q4_LDS + 64;
CC_DEV int opaque_v(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// launch-level prologue work (pp_prologue_reduce / pp_prologue_loss_tail with one 256-thread group per workgroup:
// each reduction block and loss-tail item is still one 256-thread group's, so the same bits)
CC_DEV void q4_prologue_reduce(const GemmArgs& a, char* smem) {
  if (a.pre_blocks <= 0) return;
  float(*red)[RED_COLS] = (float(*)[RED_COLS])smem;
  for (int b = blockIdx.x; b < a.pre_blocks; b += gridDim.x) {  // uniform per workgroup
    reduce_rows_phase1(a.pre, b, threadIdx.x, red);
    __syncthreads();
    reduce_rows_phase2<CC_F32>(a.pre, b, threadIdx.x, red);
    __syncthreads();
  }
}
CC_DEV void q4_prologue_loss_tail(const GemmArgs& a, char* smem) {
  if (a.tail_items <= 0) return;
  const int np = min((int)gridDim.x, a.tail_items);
  if ((int)blockIdx.x >= np) return;  // (uniform per workgroup)
  float(*evred)[4] = (float(*)[4])smem;
  for (int item = blockIdx.x; item < a.tail_items; item += np) {
    loss_tail_item(a.tail, item, threadIdx.x, evred);
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

// One output tile (whole contraction, K % 64 == 0); the epilogue's LDS image and stores as pp_epilogue_lds with 4
// waves.  wsum[h]: the squared-sum partial of virtual wave 2 wc + h (weight-gradient epilogues), else 0.
template <int EPI, bool FAST>
CC_DEV void q4_tile(const GemmArgs& args, char* smem, int bid, int tid, float (&wsum)[2]) {
  static_assert(EPI == EPI_ENC || EPI == EPI_DACTS || EPI == EPI_WGDEC || EPI == EPI_WGENC, "q4 epilogues");
  int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  tile_of_block(bid, args.nbm, args.nbn, tm, tn);
  const int m0 = tm * BM, n0 = tn * 256;
  const int M = args.M, N = args.N;
  // the epilogue's column vectors, in flight over the K loop (virtual wave v's thread index: 64 v + lane)
  EpiCols<CC_BF16, 256> ev[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    load_epi_cols<CC_BF16, EPI, 256, FAST>(ev[h], args, FragGeom<256>(args, m0, n0, wr, 2 * wc + h, lane), n0, tm, tn,
                                           (4 * wr + 2 * wc + h) * 64 + lane);
  f32x4 acc[8][8];
  q4_kloop(acc, (const char*)args.A + (int64_t)m0 * args.lda * 2, (const char*)args.B + (int64_t)n0 * args.ldb * 2,
           args.lda, (uint64_t)(M - m0) * args.lda * 2, (uint64_t)(N - n0) * args.ldb * 2, args.K / 64, smem, lane, wave);
  // (the lane index re-derived behind an opaque copy: what the epilogue computes from it is not kept live through
  // the K loop, where the fragments hold half the register file)
  lane = opaque_v(lane);
  const FragGeom<256> fg[2] = {FragGeom<256>(args, m0, n0, wr, 2 * wc, lane),
                               FragGeom<256>(args, m0, n0, wr, 2 * wc + 1, lane)};
  __syncthreads();  // every wave's last fragment reads are done: the LDS is the epilogue's
  const int rows = M - m0, cols = N - n0, ldo = (int)args.ldo;
  const int qb[4] = {0, Q4_IMG, 2 * Q4_IMG, 3 * Q4_IMG};
  // the epilogue's input tile: d_acts' activation mask (general form), dW_dec's W_dec tile (the L1 term)
  const void* in = (EPI == EPI_DACTS && !FAST) ? args.mask_src
                                               : (EPI == EPI_WGDEC && args.scale0 != 0.f ? args.w_src : nullptr);
  if (in) {
    const __amdgpu_buffer_rsrc_t rin = tile_rsrc(in, args.ldo, m0, n0, args.M, args.N, 2);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int ci = q * 4 + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void*)(smem + qb[ci >> 5] + (ci & 31) * 1024), 16,
                                               (int)piece_off(ci, lane, rows, cols, ldo), 0, 0,
                                               EPI == EPI_WGDEC ? CC_WDEC_TILE_AUX : 0);
    }
  }
  float cw[2][8][4];
  if constexpr (EPI == EPI_WGDEC) {
    if (in) {
#pragma unroll
      for (int h = 0; h < 2; ++h) wgdec_factors<256>(args, fg[h], m0, n0, cw[h]);
    }
  }
  if (in) {
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 ah[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) ah[i][j] = acc[i][4 * h + j];
    const LdsIO io(smem, qb, wr, 2 * wc + h, lane);
    wsum[h] = epilogue_core<CC_BF16, EPI, 256, FAST>(args, ah, fg[h], io, tm, m0, n0, wr, lane,
                                                     bid * 8 + 4 * wr + 2 * wc + h, ev[h], cw[h]);
  }
  __syncthreads();
  if (args.out) {
    const __amdgpu_buffer_rsrc_t rout = tile_rsrc(args.out, args.ldo, m0, n0, args.M, args.N, 2);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int ci = q * 4 + wave;
      const bf16x8 v = *(const bf16x8*)(smem + qb[ci >> 5] + (ci & 31) * 1024 + lane * 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout, (int)piece_off(ci, lane, rows, cols, ldo),
                                             0, EPI == EPI_WGDEC || EPI == EPI_WGENC ? CC_EPI_STORE_WG_AUX : CC_EPI_STORE_AUX);
    }
  }
  if (args.out_t)
    pp_store_transposed<EPI == EPI_ENC ? CC_EPI_STORE_T_AUX_ENC : CC_EPI_STORE_T_AUX, 4>(args, smem, qb, m0, n0, rows,
                                                                                       cols, lane, wave);
}

// G1 / G3 (EPI_ENC / EPI_DACTS) as a persistent q4 launch: gemm_pp_kernel's jobs and tile loop, q4 tiles.
template <int EPI, bool FAST>
CC_DEV void q4_kernel_body(const GemmArgs& args) {
  __shared__ __attribute__((aligned(16))) char smem[Q4_LDS_ALL];
  q4_prologue_reduce(args, smem);
  q4_prologue_loss_tail(args, smem);
  if (!pp_wait_ready(args, smem, Q4_SLOT)) {
    for (TileLoop L(args.nbm * args.nbn, args.tile_ctr); L.more();) {  // (the claims still drain the counters)
      L.begin();
      L.advance(smem, Q4_SLOT);
      __syncthreads();
    }
    return;
  }
  for (TileLoop L(args.nbm * args.nbn, args.tile_ctr); L.more();) {
    float w[2];
    q4_tile<EPI, FAST>(args, smem, L.begin(), pp_opaque_tid(), w);
    pp_tile_boundary();
    L.advance(smem, Q4_SLOT);
  }
}
template <int EPI, bool FAST>
__global__ __launch_bounds__(Q4_THREADS, 1) void gemm_q4_kernel(const GemmArgs args) {
  q4_kernel_body<EPI, FAST>(args);
}
// G1 runs beside the side-stream decoder-half Adam (80 VGPRs per wave): capped so that a q4 wave (this many VGPRs +
// its 256 AGPRs) leaves one Adam wave room on each SIMD, as the ping-pong's 2 x 216 registers did
#ifndef CC_Q4_ENC_VGPRS
#define CC_Q4_ENC_VGPRS 160
#endif
template <bool FAST>
__global__ __launch_bounds__(Q4_THREADS, 1) __attribute__((amdgpu_num_vgpr(CC_Q4_ENC_VGPRS))) void gemm_q4_enc_kernel(
    const GemmArgs args) {
  q4_kernel_body<EPI_ENC, FAST>(args);
}
