// HBM-bound kernels of the crosscoder training step (gfx950): input normalisation, the
// fused reconstruction loss + its gradient, decoder norms, deterministic slab reductions,
// the loss/EV finalisation, clip_grad_norm_ finalisation and the fused clip+Adam update.
// All vector accesses are 16 B per lane; every cross-block sum goes through a fixed-order
// partial slab (bit-reproducible, no float atomics).
#include "cc_common.h"

namespace cc {

#include "grad_tail.h"

constexpr int PREP_ROWS = 64;   // rows per prep block (column partial granularity)
constexpr int LOSS_ROWS = 32;   // rows per loss block
constexpr int LOSS_COLS = 512;  // columns per loss block (64 lanes x 8)

// ---------------------------------------------------------------------------------------
// Transposed copy of a block's [R rows][512 columns] bf16 output, staged in LDS: 16-B chunk c of
// row r at r * 1024 + ((c ^ (r & 7)) << 4).  ds_read_b64_tr_b16 turns 4 rows x 16 columns into
// 16 lanes x 4 rows; two of them give a lane 8 consecutive rows of one column (one 16-B store of
// out_t[col0 + c][row0 + 8k ..]).  The batch-contiguous copies feed the weight-gradient GEMMs.
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_s;
CC_DEV void tile_put8(char* lds, int r, int chunk, const float v[8]) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (short)f2bf(v[j]);
  *(bf16x8*)(lds + r * 1024 + ((chunk ^ (r & 7)) << 4)) = b;
}
// NT: non-temporal stores (prep's x^T: read once, by G5 at the step's end; kept out of the Infinity Cache it leaves
// room for what the step reads before that -- step -7 us, profiles/r04_ab_epilogue_store_policy.txt)
template <int R, bool NT = false>
CC_DEV void tile_store_transposed(const char* lds, void* out_t, int64_t ldt, int64_t col0, int ncols, int64_t row0,
                                  int nrows) {
  constexpr int RQ = R / 32;  // 32-row bands
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  for (int it = wave; it < 32 * RQ; it += 4) {
    const int cg = it / RQ, rb = (it % RQ) * 32 + g * 8;  // 16-column group, first of the lane's 8 rows
    const int ca = cg * 16 + 4 * p, c = cg * 16 + i;
    const int l0 = rb + q, l1 = rb + 4 + q;
    const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_s*)(lds + l0 * 1024 + (((ca >> 3) ^ (l0 & 7)) << 4) + (ca & 4) * 2));
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_s*)(lds + l1 * 1024 + (((ca >> 3) ^ (l1 & 7)) << 4) + (ca & 4) * 2));
    if (c < ncols && rb < nrows) {
      const bf16x8 v = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      bf16x8* dst = (bf16x8*)((bf16_t*)out_t + (col0 + c) * ldt + row0 + rb);
      if constexpr (NT) __builtin_nontemporal_store(v, dst);
      else *dst = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// x_out = dtype(x_in * factor[model]);  colsum_part[rb][k] = sum over the block's rows.
// grid: (ceil(K/512), ceil(B/64)); block 256 = 4 waves; lane -> 8 columns, wave -> 16 rows.
// TR (bf16 out): also x_t [K][B] = x_out^T through a 32-row LDS tile (two halves per block; the
// column-sum slab shares the tile's LDS, so 32 KB per block: 5 blocks per CU, one round of blocks).
template <int DIN, int DF, int DT, bool TR = false>
__global__ __launch_bounds__(256) void prep_kernel(const void* __restrict__ x_in, const void* __restrict__ factor,
                                                   void* __restrict__ x_out, float* __restrict__ colsum_part, int B,
                                                   int n, int d, void* __restrict__ x_t) {
  __shared__ __attribute__((aligned(16))) char lds[TR ? 32 * 1024 : 4 * 512 * 4];
  float(*red)[512] = (float(*)[512])lds;
  const int K = n * d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * PREP_ROWS;
  float cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float f = 1.f;
  if (factor && col < K) f = Elem<DF>::load((const typename Elem<DF>::T*)factor + col / d);
  if constexpr (TR) {
    for (int half = 0; half < 2; ++half) {
      const int base = r0 + 32 * half;
      if (base >= B) break;  // block-uniform
      if (col < K) {
        // the wave's 8 rows of this half (base + w + 4k): all loads in flight; the column sums
        // still add rows in the order r0+w, r0+w+4, ...
        float v[8][8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (base + wave + 4 * k < B) load8<DIN>(x_in, (int64_t)(base + wave + 4 * k) * K + col, v[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = base + wave + 4 * k;
          if (r >= B) break;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] = Elem<DT>::round(v[k][j] * f);
          store8<DT>(x_out, (int64_t)r * K + col, v[k]);
          tile_put8(lds, r - base, lane, v[k]);
#pragma unroll
          for (int j = 0; j < 8; ++j) cs[j] += v[k][j];
        }
      }
      __syncthreads();
      tile_store_transposed<32, true>(lds, x_t, B, (int64_t)blockIdx.x * 512, K - blockIdx.x * 512, base,
                                B - base < 32 ? B - base : 32);
      __syncthreads();
    }
  } else if (col < K) {
    // 4 rows per trip (rows rb, rb+4, rb+8, rb+12): their loads are in flight together
    for (int rb = r0 + wave; rb < r0 + PREP_ROWS && rb < B; rb += 16) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (rb + 4 * u < B) load8<DIN>(x_in, (int64_t)(rb + 4 * u) * K + col, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 4 * u;
        if (r >= B) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = Elem<DT>::round(v[u][j] * f);
        store8<DT>(x_out, (int64_t)r * K + col, v[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] += v[u][j];
      }
    }
  }
  if (!colsum_part) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = cs[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    int c = blockIdx.x * 512 + i;
    if (c < K) colsum_part[(int64_t)blockIdx.y * K + c] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
  }
}

template <int DT>
__global__ __launch_bounds__(256) void reduce_rows_kernel(const RedSeg a) {
  __shared__ float red[4][RED_COLS];
  reduce_rows_phase1(a, blockIdx.x, threadIdx.x, red);
  __syncthreads();
  reduce_rows_phase2<DT>(a, blockIdx.x, threadIdx.x, red);
}

// ---------------------------------------------------------------------------------------
// norms[h][m] = ||W_dec[h,m,:]||, total[h] = sum_m.  One wave per (h) row, all models.
// Summation order (shared with the fused W_dec^T transposition, cc_transpose_dec_norms, so both
// give the same bits): per 64-column block, each of 8 lanes sums its 8 squares in order (fma),
// the 8 lane sums combine by an xor-1/2/4 butterfly; block sums are added in ascending order.
template <int DT>
__global__ __launch_bounds__(256) void dec_norms_kernel(const void* __restrict__ W, float* __restrict__ norms,
                                                        float* __restrict__ total, float* __restrict__ inv_norms, int h,
                                                        int n, int d) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= h) return;
  float tot = 0.f;
  for (int m = 0; m < n; ++m) {
    const int64_t base = ((int64_t)row * n + m) * d;
    float s = 0.f;
    for (int c0 = 0; c0 < d; c0 += 512) {  // 8 blocks of 64 columns per pass
      const int c = c0 + lane * 8;
      float q = 0.f;
      if (c < d) {
        float v[8];
        load8<DT>(W, base + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) q = __fmaf_rn(v[j], v[j], q);
      }
      q = block8_sum(q);
#pragma unroll
      for (int g = 0; g < 8; ++g)
        if (c0 + 64 * g < d) s += __shfl(q, 8 * g, 64);
    }
    const float nr = sqrtf(s);
    if (lane == 0) {
      norms[(int64_t)row * n + m] = nr;
      if (inv_norms) inv_norms[(int64_t)row * n + m] = nr > 0.f ? 1.f / nr : 0.f;
    }
    tot += nr;
  }
  if (lane == 0) total[row] = tot;
}

// ---------------------------------------------------------------------------------------
// Reconstruction loss + gradient.  grid: (n * ncb, ceil(rows/32)); block 256 = 4 waves.
// Block covers model m = blockIdx.x / ncb, columns [m*d + cb*512, +512) ∩ model, 32 rows of the
// row range [row0, row_end) (row0 % 32 == 0).  The slabs keep the whole-batch layout, so disjoint
// row ranges can be separate launches: the latent-sharded step runs each batch slice as soon as
// its all-reduce has landed.  lane -> 8 columns; wave w -> rows r0 + w + 4i.
// TR (bf16): also g_recon_t [K][B] = g_recon^T (rows [row0, row_end)) through an LDS tile.
template <int DT, bool TR = false>
__global__ __launch_bounds__(256) void loss_kernel(const float* __restrict__ recon, const void* __restrict__ b_dec,
                                                   const void* __restrict__ x, const float* __restrict__ x_mean,
                                                   void* __restrict__ g_recon, float* __restrict__ row_part,
                                                   float* __restrict__ col_part, float grad_scale, int B, int n,
                                                   int d, int ncb, int row0, int row_end, void* __restrict__ g_t) {
  // (TR: the column-sum slab reuses the transposition tile's LDS: 32 KB per block)
  __shared__ __attribute__((aligned(16))) char tile[TR ? LOSS_ROWS * 1024 : 4 * 512 * 4];
  float(*red)[512] = (float(*)[512])tile;
  using E = Elem<DT>;
  const int K = n * d;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = blockIdx.x / ncb, cb = blockIdx.x % ncb;
  const int jc = cb * LOSS_COLS + lane * 8;  // column within model
  const bool cv = jc < d;
  const int col = m * d + jc;
  const int r0 = row0 + blockIdx.y * LOSS_ROWS;
  float bd[8], mu[8], cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bd[j] = mu[j] = cs[j] = 0.f;
  if (cv) {
    if (b_dec) load8<DT>(b_dec, col, bd);
    if (x_mean) load8f(x_mean, col, mu);
  }
  const int64_t plane = (int64_t)n * ncb * B;  // row_part [2][n*ncb][B]
  // LOSS_U rows per trip (r, r + 4, ...): their loads are in flight together (the column sums still
  // add the wave's rows in order)
  constexpr int LOSS_U = 2;
  for (int i = 0; i < LOSS_ROWS / 4; i += LOSS_U) {
    const int ra = r0 + wave + 4 * i;
    if (ra >= row_end) break;  // wave-uniform
    float rv[LOSS_U][8], xv[LOSS_U][8];
    if (cv) {
#pragma unroll
      for (int u = 0; u < LOSS_U; ++u)
        if (ra + 4 * u < row_end) {
          load8f(recon, (int64_t)(ra + 4 * u) * K + col, rv[u]);
          load8<DT>(x, (int64_t)(ra + 4 * u) * K + col, xv[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < LOSS_U; ++u) {
      const int r = ra + 4 * u;
      if (r >= row_end) break;
      float l2 = 0.f, tv = 0.f;
      if (cv) {
        float g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float diff = (rv[u][j] + bd[j]) - xv[u][j];
          l2 += diff * diff;
          float c = xv[u][j] - mu[j];
          tv += c * c;
          g[j] = E::round(grad_scale * diff);
          cs[j] += g[j];
        }
        store8<DT>(g_recon, (int64_t)r * K + col, g);
        if constexpr (TR) tile_put8(tile, r - r0, lane, g);
      }
      l2 = wave_sum(l2);
      tv = wave_sum(tv);
      if (lane == 0) {
        row_part[(int64_t)blockIdx.x * B + r] = l2;
        row_part[plane + (int64_t)blockIdx.x * B + r] = tv;
      }
    }
  }
  if constexpr (TR) {
    __syncthreads();
    const int nr = row_end - r0 < LOSS_ROWS ? row_end - r0 : LOSS_ROWS;
    tile_store_transposed<LOSS_ROWS>(tile, g_t, B, (int64_t)m * d + cb * LOSS_COLS, d - cb * LOSS_COLS, r0, nr);
    __syncthreads();  // (red reuses the tile)
  }
  if (!col_part) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = cs[j];
  __syncthreads();
  for (int i = threadIdx.x; i < LOSS_COLS; i += 256) {
    int jj = cb * LOSS_COLS + i;
    if (jj < d)
      col_part[(int64_t)(row0 / LOSS_ROWS + blockIdx.y) * K + m * d + jj] =
          ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
  }
}

#include "loss_tail.h"

__global__ __launch_bounds__(256) void ev_kernel(const EvSeg a) {
  __shared__ float red[4][4];
  ev_phase1(a, blockIdx.x, threadIdx.x, red);
  __syncthreads();
  ev_phase2(a, blockIdx.x, threadIdx.x, red);
}

__global__ __launch_bounds__(LOSS_THREADS) void loss_scalars_kernel(const ScalArgs a) {
  __shared__ double red[LOSS_THREADS / 64][6];
  loss_scalars_body<LOSS_THREADS>(a, red);
}

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(SCAL_THREADS) void clip_kernel(const ClipArgs a) {
  __shared__ double red[8][SCAL_THREADS / 64];
  __shared__ float norms[8];
  clip_body<SCAL_THREADS>(a, red, norms);
}

// ---------------------------------------------------------------------------------------
// Arrival count of a fused tail launch: every workgroup publishes what it wrote, and the last one to arrive
// (device-scope counter, reset by that workgroup for the next launch) returns true with the others' writes
// visible.  The barrier's workgroup-scope release waits for every wave's stores to reach this XCD's L2; ONE
// agent-scope release (an L2 write-back) then publishes them all before the arrival count.  Call with every
// thread of the workgroup; `last` is LDS scratch.
CC_DEV bool arrive_last(unsigned* counter, int* last) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const bool is_last = atomicAdd(counter, 1u) == gridDim.x - 1;
    if (is_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop stale lines before the reads
    *last = is_last;
  }
  __syncthreads();
  return *last;
}

// Fused grad tail: one launch of 1024-thread blocks = 4 independent 256-thread groups, each running one
// block of a column reduction (RedSeg: b_enc.grad, b_dec.grad column sums + their sq partials) -- the same
// two phases as the stand-alone kernel, so the same bits -- then the last block to finish runs clip_body
// (or the segment sums) over the partials the whole grid wrote.  Saves the finaliser's launch per step.
struct TailArgs {
  RedSeg red[2];
  int red_blocks[2];  // 256-thread groups per reduction (0: unused)
  ClipArgs clip;
  unsigned* counter;
};
template <int DT>
__global__ __launch_bounds__(SCAL_THREADS) void tail_kernel(const TailArgs a) {
  __shared__ float red[4][4][RED_COLS];
  __shared__ int last;
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255;
  int b = blockIdx.x * 4 + grp;
  // role of this group: reduction 0, reduction 1 or idle (uniform per group)
  int role = 2;
  if (b < a.red_blocks[0]) role = 0;
  else if ((b -= a.red_blocks[0]) < a.red_blocks[1]) role = 1;
  if (role < 2) reduce_rows_phase1(a.red[role], b, t, red[grp]);
  __syncthreads();
  if (role < 2) reduce_rows_phase2<DT>(a.red[role], b, t, red[grp]);
  if (!arrive_last(a.counter, &last)) return;
  __shared__ double cred[8][SCAL_THREADS / 64];
  __shared__ float cnorms[8];
  clip_body<SCAL_THREADS>(a.clip, cred, cnorms);
  if (threadIdx.x == 0) atomicExch(a.counter, 0u);
}

// Fused loss tail (crosscoder.py:106-128): the l1 partials, the per-row EV terms and the loss scalars in one
// launch of the LossTailArgs items (loss_tail.h), one 256-thread workgroup per item, whose workgroups fit beside a
// persistent GEMM workgroup (256 threads, few registers, < 0.5 KB of LDS); the last workgroup to arrive runs
// loss_scalars_body<LOSS_THREADS> (the stand-alone loss_scalars_kernel's).
__global__ __launch_bounds__(LOSS_THREADS) void loss_tail_kernel(const LossTailArgs a) {
  __shared__ float evred[4][4];
  __shared__ double sred[LOSS_THREADS / 64][6];
  __shared__ int last;
  loss_tail_item(a, blockIdx.x, threadIdx.x, evred);
  if (!arrive_last(a.counter, &last)) return;
  loss_scalars_body<LOSS_THREADS>(a.scal, sred);
  if (threadIdx.x == 0) atomicExch(a.counter, 0u);
}

// ---------------------------------------------------------------------------------------
// Fused clip-multiply + Adam (torch/optim/adam.py _single_tensor_adam, no wd/amsgrad), with the
// dtype rounding after each of torch's tensor ops:
//   g = R(g*coef); m = R(lerp(m, g, 1-b1)); v = R(R(v*b2) + (1-b2)*g*g);
//   den = R(R(R(sqrt v) / bc2s) + eps); p = R(p + (-step_size) * (m / den))
struct AdamArgs {
  void* p;
  const void* g;
  void* m;
  void* v;
  int64_t numel;
  const float* coef;
  float w1;         // 1 - beta1 (lerp weight)
  float beta2, omb2, eps;
  float bc2s;       // sqrt(1 - beta2^t)
  float neg_step;   // -lr / (1 - beta1^t)
  // clip coefficient formed in the kernel (instead of read from coef): clip_grad_norm_ over the clip_np
  // per-parameter squared sums clip_sums (e.g. all-reduced over the latent shards); block 0 writes clip_out
  // [coef, total, norms...] like cc_clip_finalize
  const float* clip_sums;
  int clip_np, clip_emulate;
  float clip_max_norm;
  float* clip_out;
  // decoder norms' per-(row, 64-column block) squared sums of the UPDATED parameters over the first
  // norm_rows x norm_ld elements (W_dec [h][K]), in cc_dec_norms' order, into norm_part[row][K / 64]
  // (adam_kernel only; nullptr: none)
  float* norm_part;
  int norm_rows, norm_ld;
  // the capped grid-stride forms: each workgroup, when its stores are done, releases them (agent scope) and adds
  // 1 here -- a reader launched on another stream (G2, cc_decode_loss's wait_ctr) waits for the count in its
  // kernel instead of for an event (nullptr: none)
  unsigned* done_ctr;
};
// Every thread of the workgroup: its stores drained, the barrier, one agent-scope release (writes the XCD's L2
// back), then the arrival count.
CC_DEV void adam_signal_done(unsigned* ctr) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// The step's clip coefficient: read (coef), formed from squared sums (clip_sums), or 1
CC_DEV float adam_coef(const AdamArgs& a) {
  if (a.clip_sums) {
    float norms[8], total;
    bool aborted = false;  // (a negative squared sum: a rank's step was aborted -- ClipArgs::sums_only writes -inf)
    for (int p = 0; p < a.clip_np; ++p) {
      aborted |= a.clip_sums[p] < 0.f;
      norms[p] = clip_param_norm((double)a.clip_sums[p], a.clip_emulate);
    }
    const float c = aborted ? CC_CLIP_ABORTED : clip_coef(norms, a.clip_np, a.clip_max_norm, a.clip_emulate, total);
    if (a.clip_out && blockIdx.x == 0 && threadIdx.x == 0) {
      a.clip_out[0] = c;
      a.clip_out[1] = total;
      for (int p = 0; p < a.clip_np; ++p) a.clip_out[2 + p] = norms[p];
    }
    return c;
  }
  return a.coef ? *a.coef : 1.f;
}
// adam_coef for the whole block: from the squared sums it is ~100 dependent VALU ops (fp64 square roots), so
// one wave forms it and the others read it from LDS -- with one 8-element chunk per thread (the bulk
// kernel) every wave forming it costs the launch ~20 us.  Call with every thread of the block.  (Not for a
// kernel meant to share CUs with the GEMMs: any LDS keeps its workgroups off a CU whose LDS a GEMM
// workgroup holds.)
CC_DEV float adam_coef_block(const AdamArgs& a) {
  if (!a.clip_sums) return a.coef ? *a.coef : 1.f;
  __shared__ float s_coef;
  if (threadIdx.x < 64) {
    const float c = adam_coef(a);
    if (threadIdx.x == 0) s_coef = c;
  }
  __syncthreads();
  return s_coef;
}
// One Adam element update with torch's rounding points (see adam_kernel).
template <int DT>
CC_DEV void adam_elem(const AdamArgs& a, float coef, float& p, float g, float& m, float& v) {
#pragma clang fp contract(off)
  using E = Elem<DT>;
  float gj = E::round(g * coef);
  float w = a.w1;
  float mj = w < 0.5f ? __builtin_fmaf(w, gj - m, m) : __builtin_fmaf(-(gj - m), 1.f - w, gj);
  mj = E::round(mj);
  float vj = E::round(v * a.beta2);
  vj = E::round(vj + a.omb2 * gj * gj);
  float den = E::round(sqrtf(vj));
  den = E::round(den / a.bc2s);
  den = E::round(den + a.eps);
  p = E::round(p + a.neg_step * (mj / den));
  m = mj;
  v = vj;
}

// cache policy of the bulk (encoder-half / whole-arena) Adam: g / m / v non-temporal, p temporal (the
// updated weights stay in the Infinity Cache for the next GEMM that reads them; measured faster than all
// temporal or all non-temporal)
constexpr int ADAM_U = 1;

// Bulk of the arena: U 8-element chunks per thread, all 4*U loads issued before any math, one
// pass over the grid (no grid-stride loop).  U = 1 measured fastest (390 us for the 151 M-element
// config-2 arena = 5.4 TB/s; U = 2: 398 us; the grid-stride loop: 431 us).
template <int DT, int U>
__global__ __launch_bounds__(256) void adam_bulk_kernel(const AdamArgs a, int64_t nchunks) {
  const int64_t c0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  float p[U][8], g[U][8], m[U][8], v[U][8];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = c0 + u * 256;
    if (c < nchunks) {
      constexpr bool PN = false, SN = true;
      ld8<DT, PN>(a.p, c * 8, p[u]); ld8<DT, SN>(a.g, c * 8, g[u]); ld8<DT, SN>(a.m, c * 8, m[u]);
      ld8<DT, SN>(a.v, c * 8, v[u]);
    }
  }
  // the coefficient after the element loads are in flight (its inputs' latency hides under theirs; formed
  // from the squared sums it also stores clip_out, which must not hold the loads back)
  const float coef = adam_coef_block(a);
  if (coef < 0.f) return;  // CC_CLIP_ABORTED: the step's update is not applied
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t c = c0 + u * 256;
    if (c < nchunks) {
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem<DT>(a, coef, p[u][j], g[u][j], m[u][j], v[u][j]);
      constexpr bool PN = false, SN = true;
      st8<DT, PN>(a.p, c * 8, p[u]); st8<DT, SN>(a.m, c * 8, m[u]); st8<DT, SN>(a.v, c * 8, v[u]);
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {
  using E = Elem<DT>;
  // (per thread, once before the grid-stride loop: no LDS, so its workgroups still fit beside a GEMM
  // workgroup that holds a CU's whole LDS -- the decoder half runs beside G1)
  const float coef = adam_coef(a);
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  // (CC_CLIP_ABORTED: the step's update is not applied -- p / m / v and the norm partials stay as they are --
  // but the done count still arrives)
  const int64_t numel = coef < 0.f ? 0 : a.numel;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < numel; i += stride) {
    float p[8], g[8], m[8], v[8];
    const bool full = i + 8 <= a.numel;
    if (full) {
      load8_nt<DT>(a.p, i, p); load8_nt<DT>(a.g, i, g); load8_nt<DT>(a.m, i, m); load8_nt<DT>(a.v, i, v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int64_t k = i + j < a.numel ? i + j : a.numel - 1;
        p[j] = E::load((const typename E::T*)a.p + k);
        g[j] = E::load((const typename E::T*)a.g + k);
        m[j] = E::load((const typename E::T*)a.m + k);
        v[j] = E::load((const typename E::T*)a.v + k);
      }
    }
    // torch's CPU/GPU kernels: lerp is an fma (Lerp.h vectorised path), every other op is a
    // separately rounded fp32 multiply/add -> no contraction here.
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma clang fp contract(off)
      float gj = E::round(g[j] * coef);
      float w = a.w1;
      float mj = w < 0.5f ? __builtin_fmaf(w, gj - m[j], m[j]) : __builtin_fmaf(-(gj - m[j]), 1.f - w, gj);
      mj = E::round(mj);
      float vj = E::round(v[j] * a.beta2);
      vj = E::round(vj + a.omb2 * gj * gj);
      float den = E::round(sqrtf(vj));
      den = E::round(den / a.bc2s);
      den = E::round(den + a.eps);
      float pj = E::round(p[j] + a.neg_step * (mj / den));
      p[j] = pj; m[j] = mj; v[j] = vj;
    }
    if (a.norm_part && i < (int64_t)a.norm_rows * a.norm_ld) {
      // the 8 lanes of an aligned group hold one 64-column block of a row (i % 64 == 8 * (lane & 7): the
      // grid stride is a multiple of 64, K % 64 == 0), all of them inside the matrix together
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) q = __fmaf_rn(p[j], p[j], q);
      q = block8_sum(q);
      if ((threadIdx.x & 7) == 0) {
        const int row = (int)(i / a.norm_ld);
        a.norm_part[(int64_t)row * (a.norm_ld >> 6) + ((int)(i - (int64_t)row * a.norm_ld) >> 6)] = q;
      }
    }
    if (full) {
      store8_nt<DT>(a.p, i, p);
      store8_nt<DT>(a.m, i, m); store8_nt<DT>(a.v, i, v);
    } else {
      for (int j = 0; j < 8 && i + j < a.numel; ++j) {
        ((typename E::T*)a.p)[i + j] = E::from_f(p[j]);
        ((typename E::T*)a.m)[i + j] = E::from_f(m[j]);
        ((typename E::T*)a.v)[i + j] = E::from_f(v[j]);
      }
    }
  }
  if (a.done_ctr) adam_signal_done(a.done_ctr);
}

// The capped-grid (side-stream) bf16 Adam with the next chunk's loads in flight during this chunk's math.
// Beside G1 its workgroups get one wave per SIMD (G1 holds 2 x 216 of the 512 registers), so it streams
// only as fast as one wave's loads in flight allow: this form keeps two chunks' loads in flight in the same
// 64 registers, the data kept packed (8 bf16 per 16 B) and unpacked one element at a time.  Same per-element
// arithmetic (adam_elem) and norm partials as adam_kernel.  numel % 8 == 0.
CC_DEV void adam_pipe_load(const AdamArgs& a, int64_t i, bf16x8& p, bf16x8& g, bf16x8& m, bf16x8& v) {
  p = __builtin_nontemporal_load((const bf16x8*)((const bf16_t*)a.p + i));
  g = __builtin_nontemporal_load((const bf16x8*)((const bf16_t*)a.g + i));
  m = __builtin_nontemporal_load((const bf16x8*)((const bf16_t*)a.m + i));
  v = __builtin_nontemporal_load((const bf16x8*)((const bf16_t*)a.v + i));
}
__global__ __launch_bounds__(256) void adam_pipe_kernel(const AdamArgs a) {
  const float coef = adam_coef(a);
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  const int64_t numel = coef < 0.f ? 0 : a.numel;  // (CC_CLIP_ABORTED: as adam_kernel)
  int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  bf16x8 p, g, m, v;
  if (i < numel) adam_pipe_load(a, i, p, g, m, v);
  for (; i < numel; i += stride) {
    const int64_t nx = i + stride;
    bf16x8 p2 = p, g2 = g, m2 = m, v2 = v;
    if (nx < numel) adam_pipe_load(a, nx, p2, g2, m2, v2);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float pj = bf2f((bf16_t)p[j]), mj = bf2f((bf16_t)m[j]), vj = bf2f((bf16_t)v[j]);
      adam_elem<CC_BF16>(a, coef, pj, bf2f((bf16_t)g[j]), mj, vj);
      p[j] = (short)f2bf(pj);
      m[j] = (short)f2bf(mj);
      v[j] = (short)f2bf(vj);
      q = __fmaf_rn(pj, pj, q);
    }
    if (a.norm_part && i < (int64_t)a.norm_rows * a.norm_ld) {  // (as adam_kernel)
      q = block8_sum(q);
      if ((threadIdx.x & 7) == 0) {
        const int row = (int)(i / a.norm_ld);
        a.norm_part[(int64_t)row * (a.norm_ld >> 6) + ((int)(i - (int64_t)row * a.norm_ld) >> 6)] = q;
      }
    }
    __builtin_nontemporal_store(p, (bf16x8*)((bf16_t*)a.p + i));
    __builtin_nontemporal_store(m, (bf16x8*)((bf16_t*)a.m + i));
    __builtin_nontemporal_store(v, (bf16x8*)((bf16_t*)a.v + i));
    p = p2; g = g2; m = m2; v = v2;
  }
  if (a.done_ctr) adam_signal_done(a.done_ctr);
}

// Decoder-half Adam over W_dec [h][K] (bf16) in 64 x 64 tiles that also emits what the next
// step needs from the updated W_dec: W_dec^T [K][h] (LDS tile read back with ds_read_b64_tr_b16)
// and the decoder norms' per-(row, 64-column block) squared sums in dec_norms_kernel's order
// (8 sequential fma per lane, xor-1/2/4 butterfly) -- one HBM pass instead of Adam + a
// transpose/norms pass.  Persistent grid over the tiles, rows fast; every element gets
// adam_elem, so p / m / v are the bits cc_adam_step produces.
// (64 VGPRs: one half-tile's 4 x 8 elements per thread at a time, so it fits beside a 2-wave-per-SIMD
// ping-pong GEMM's 208)
__global__ __launch_bounds__(256) void adam_dec_tr_kernel(const AdamArgs a, int h, int K, char* __restrict__ wt,
                                                          float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char tile[64 * 128];
  const float coef = adam_coef(a);
  if (coef < 0.f) return;  // CC_CLIP_ABORTED: the step's update is not applied
  const int nr = (h + 63) / 64, nblk = K / 64, ntiles = nr * nblk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g4 = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r0 = (t % nr) * 64, c0 = (t / nr) * 64;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int idx = threadIdx.x + 256 * k, r = idx >> 3, ch = idx & 7;
      float qs = 0.f;
      if (r0 + r < h) {
        float p[8], g[8], m[8], v[8];
        const int64_t e = (int64_t)(r0 + r) * K + c0 + 8 * ch;
        load8_nt<CC_BF16>(a.p, e, p); load8_nt<CC_BF16>(a.g, e, g);
        load8_nt<CC_BF16>(a.m, e, m); load8_nt<CC_BF16>(a.v, e, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) adam_elem<CC_BF16>(a, coef, p[j], g[j], m[j], v[j]);
        store8_nt<CC_BF16>(a.p, e, p); store8_nt<CC_BF16>(a.m, e, m); store8_nt<CC_BF16>(a.v, e, v);
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          b[j] = (short)f2bf(p[j]);
          qs = __fmaf_rn(p[j], p[j], qs);
        }
        *(bf16x8*)(tile + r * 128 + ((ch ^ (r & 7)) << 4)) = b;
      }
      qs = block8_sum(qs);
      if (ch == 0 && r0 + r < h) part[(int64_t)(r0 + r) * nblk + (c0 >> 6)] = qs;
    }
    __syncthreads();
    const int ca = 16 * w + 4 * p4, cch = ca >> 3, c = 16 * w + i;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int R = (4 * s2 + g4) * 8, l0 = R + q4, l1 = R + 4 + q4;
      const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4_s*)(tile + l0 * 128 + ((cch ^ (l0 & 7)) << 4) + (ca & 4) * 2));
      const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4_s*)(tile + l1 * 128 + ((cch ^ (l1 & 7)) << 4) + (ca & 4) * 2));
      if (r0 + R < h)
        *(bf16x8*)(wt + ((int64_t)(c0 + c) * h + r0 + R) * 2) =
            bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
    __syncthreads();
  }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace cc

using namespace cc;

#define DISPATCH_DT(dtype, KERNEL_CALL)                                   \
  do {                                                                    \
    if ((dtype) == CC_BF16) { constexpr int DT_ = CC_BF16; KERNEL_CALL; } \
    else if ((dtype) == CC_F32) { constexpr int DT_ = CC_F32; KERNEL_CALL; } \
    else return CC_ERR_DTYPE;                                             \
  } while (0)

extern "C" {

int cc_version(void) { return 100; }

const char* cc_strerror(int code) {
  switch (code) {
    case CC_OK: return "ok";
    case CC_ERR_NULL: return "crosscoder_hip: required pointer is NULL";
    case CC_ERR_DTYPE: return "crosscoder_hip: unsupported dtype (expected CC_BF16 or CC_F32)";
    case CC_ERR_SHAPE: return "crosscoder_hip: unsupported shape (d_model and dict_size must be multiples of 8)";
    case CC_ERR_ALIGN: return "crosscoder_hip: pointer or leading dimension not 16-byte aligned";
    case CC_ERR_TOO_LARGE: return "crosscoder_hip: operand panel exceeds 2 GiB buffer-descriptor range";
    default: break;
  }
  if (code >= CC_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(code - CC_ERR_HIP_BASE));
  return "crosscoder_hip: unknown error";
}

int64_t cc_prep_part_rows(int64_t B) { return (B + PREP_ROWS - 1) / PREP_ROWS; }
int64_t cc_loss_part_rows(int64_t B) { return (B + LOSS_ROWS - 1) / LOSS_ROWS; }
int64_t cc_loss_col_blocks(int64_t d) { return (d + LOSS_COLS - 1) / LOSS_COLS; }
int64_t cc_loss_scalars_len(int64_t B) { return 8 + 4 * ((B + 255) / 256); }
int64_t cc_reduce_parts(int64_t C) { return (C + RED_COLS - 1) / RED_COLS; }

int cc_prep_input_t(const void* x_in, int in_dtype, const void* factor, int factor_dtype, void* x_out, void* x_t,
                    float* colsum_part, int64_t B, int64_t n, int64_t d, int dtype, void* stream) {
  if (!x_t) return cc_prep_input(x_in, in_dtype, factor, factor_dtype, x_out, colsum_part, B, n, d, dtype, stream);
  if (!x_in || !x_out) return CC_ERR_NULL;
  if (B <= 0 || n <= 0 || d <= 0 || d % 8 || B % 8) return CC_ERR_SHAPE;
  if (dtype != CC_BF16) return CC_ERR_DTYPE;
  if (!al16(x_in) || !al16(x_out) || !al16(x_t)) return CC_ERR_ALIGN;
  if (factor && factor_dtype != CC_BF16 && factor_dtype != CC_F32) return CC_ERR_DTYPE;
  if (in_dtype != CC_BF16 && in_dtype != CC_F32) return CC_ERR_DTYPE;
  dim3 grid((unsigned)((n * d + 511) / 512), (unsigned)cc_prep_part_rows(B));
  hipStream_t st = (hipStream_t)stream;
  const bool fb = factor && factor_dtype == CC_BF16;
#define PREPT(DI, DF) \
  hipLaunchKernelGGL((prep_kernel<DI, DF, CC_BF16, true>), grid, dim3(256), 0, st, x_in, factor, x_out, colsum_part, \
                     (int)B, (int)n, (int)d, x_t)
  if (in_dtype == CC_BF16) {
    if (fb) PREPT(CC_BF16, CC_BF16); else PREPT(CC_BF16, CC_F32);
  } else {
    if (fb) PREPT(CC_F32, CC_BF16); else PREPT(CC_F32, CC_F32);
  }
#undef PREPT
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_prep_input(const void* x_in, int in_dtype, const void* factor, int factor_dtype, void* x_out,
                  float* colsum_part, int64_t B, int64_t n, int64_t d, int dtype, void* stream) {
  if (!x_in || !x_out) return CC_ERR_NULL;
  if (B <= 0 || n <= 0 || d <= 0 || d % 8) return CC_ERR_SHAPE;
  if (!al16(x_in) || !al16(x_out)) return CC_ERR_ALIGN;
  if (factor && factor_dtype != CC_BF16 && factor_dtype != CC_F32) return CC_ERR_DTYPE;
  if (in_dtype != CC_BF16 && in_dtype != CC_F32) return CC_ERR_DTYPE;
  dim3 grid((unsigned)((n * d + 511) / 512), (unsigned)cc_prep_part_rows(B));
  hipStream_t st = (hipStream_t)stream;
#define PREP(DI, DF, DO) \
  hipLaunchKernelGGL((prep_kernel<DI, DF, DO>), grid, dim3(256), 0, st, x_in, factor, x_out, colsum_part, (int)B, (int)n, (int)d, nullptr)
  int fdt = factor ? factor_dtype : CC_F32;
  if (dtype != CC_BF16 && dtype != CC_F32) return CC_ERR_DTYPE;
  if (in_dtype == CC_BF16) {
    if (fdt == CC_BF16) { if (dtype == CC_BF16) PREP(CC_BF16, CC_BF16, CC_BF16); else PREP(CC_BF16, CC_BF16, CC_F32); }
    else { if (dtype == CC_BF16) PREP(CC_BF16, CC_F32, CC_BF16); else PREP(CC_BF16, CC_F32, CC_F32); }
  } else {
    if (fdt == CC_BF16) { if (dtype == CC_BF16) PREP(CC_F32, CC_BF16, CC_BF16); else PREP(CC_F32, CC_BF16, CC_F32); }
    else { if (dtype == CC_BF16) PREP(CC_F32, CC_F32, CC_BF16); else PREP(CC_F32, CC_F32, CC_F32); }
  }
#undef PREP
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_reduce_rows(const float* part, int64_t R, int64_t C, int64_t ld, float scale, float* out_f32, void* out_t,
                   int dtype, float* sq_part, const float* dot_w, float* dot_part, void* stream) {
  if (!part) return CC_ERR_NULL;
  if (R <= 0 || C <= 0) return CC_ERR_SHAPE;
  if (sq_part && !out_t) return CC_ERR_NULL;
  if (dot_part && !dot_w) return CC_ERR_NULL;
  dim3 grid((unsigned)((C + RED_COLS - 1) / RED_COLS));
  hipStream_t st = (hipStream_t)stream;
  const RedSeg a = {part, (int)R, (int)C, ld, scale, out_f32, out_t, sq_part, dot_w, dot_part};
  if (out_t) {
    DISPATCH_DT(dtype, hipLaunchKernelGGL((reduce_rows_kernel<DT_>), grid, dim3(256), 0, st, a));
  } else {
    hipLaunchKernelGGL((reduce_rows_kernel<CC_F32>), grid, dim3(256), 0, st, a);
  }
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_dec_norms(const void* W_dec, float* norms, float* total, float* inv_norms, int64_t h, int64_t n, int64_t d,
                 int dtype, void* stream) {
  if (!W_dec || !norms || !total) return CC_ERR_NULL;
  if (h <= 0 || n <= 0 || d <= 0 || d % 8) return CC_ERR_SHAPE;
  if (!al16(W_dec)) return CC_ERR_ALIGN;
  dim3 grid((unsigned)((h + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_DT(dtype, hipLaunchKernelGGL((dec_norms_kernel<DT_>), grid, dim3(256), 0, st, W_dec, norms, total,
                                        inv_norms, (int)h, (int)n, (int)d));
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_loss_fwd_bwd_rows_t(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean,
                           void* g_recon, void* g_recon_t, float* row_part, float* col_part, float grad_scale,
                           int64_t row0, int64_t rows, int64_t B, int64_t n, int64_t d, int dtype, void* stream) {
  if (!g_recon_t)
    return cc_loss_fwd_bwd_rows(recon_f32, b_dec, x, x_mean, g_recon, row_part, col_part, grad_scale, row0, rows, B,
                                n, d, dtype, stream);
  if (!recon_f32 || !x || !g_recon || !row_part) return CC_ERR_NULL;
  if (B <= 0 || n <= 0 || d <= 0 || d % 8 || B % 8 || rows % 8) return CC_ERR_SHAPE;
  if (row0 < 0 || rows <= 0 || row0 + rows > B || row0 % LOSS_ROWS) return CC_ERR_SHAPE;
  if (dtype != CC_BF16) return CC_ERR_DTYPE;
  if (!al16(recon_f32) || !al16(x) || !al16(g_recon) || !al16(g_recon_t) || (b_dec && !al16(b_dec)) ||
      (x_mean && !al16(x_mean)))
    return CC_ERR_ALIGN;
  int ncb = (int)cc_loss_col_blocks(d);
  dim3 grid((unsigned)(n * ncb), (unsigned)cc_loss_part_rows(rows));
  hipLaunchKernelGGL((loss_kernel<CC_BF16, true>), grid, dim3(256), 0, (hipStream_t)stream, recon_f32, b_dec, x,
                     x_mean, g_recon, row_part, col_part, grad_scale, (int)B, (int)n, (int)d, ncb, (int)row0,
                     (int)(row0 + rows), g_recon_t);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_loss_fwd_bwd_rows(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean,
                         void* g_recon, float* row_part, float* col_part, float grad_scale, int64_t row0,
                         int64_t rows, int64_t B, int64_t n, int64_t d, int dtype, void* stream) {
  if (!recon_f32 || !x || !g_recon || !row_part) return CC_ERR_NULL;
  if (B <= 0 || n <= 0 || d <= 0 || d % 8) return CC_ERR_SHAPE;
  if (row0 < 0 || rows <= 0 || row0 + rows > B || row0 % LOSS_ROWS) return CC_ERR_SHAPE;
  if (!al16(recon_f32) || !al16(x) || !al16(g_recon) || (b_dec && !al16(b_dec)) || (x_mean && !al16(x_mean)))
    return CC_ERR_ALIGN;
  int ncb = (int)cc_loss_col_blocks(d);
  dim3 grid((unsigned)(n * ncb), (unsigned)cc_loss_part_rows(rows));
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_DT(dtype, hipLaunchKernelGGL((loss_kernel<DT_>), grid, dim3(256), 0, st, recon_f32, b_dec, x, x_mean,
                                        g_recon, row_part, col_part, grad_scale, (int)B, (int)n, (int)d, ncb,
                                        (int)row0, (int)(row0 + rows), nullptr));
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_loss_fwd_bwd(const float* recon_f32, const void* b_dec, const void* x, const float* x_mean, void* g_recon,
                    float* row_part, float* col_part, float grad_scale, int64_t B, int64_t n, int64_t d, int dtype,
                    void* stream) {
  return cc_loss_fwd_bwd_rows(recon_f32, b_dec, x, x_mean, g_recon, row_part, col_part, grad_scale, 0, B, B, n, d,
                              dtype, stream);
}

int cc_loss_finalize(const float* row_part, const float* l1_part, int64_t n_l1, const float* l0_part, int64_t n_l0,
                     float* ev, float* ev_a, float* ev_b, float* scalars, float* l1l0_out, int64_t B, int64_t n,
                     int64_t d, void* stream) {
  return cc_loss_finalize_mapped(row_part, l1_part, n_l1, l0_part, n_l0, ev, ev_a, ev_b, scalars, l1l0_out, nullptr,
                                 0, B, n, d, stream);
}

int cc_loss_finalize_mapped(const float* row_part, const float* l1_part, int64_t n_l1, const float* l0_part,
                            int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars, float* l1l0_out,
                            float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, void* stream) {
  return cc_loss_finalize_nb(row_part, cc_loss_col_blocks(d), l1_part, n_l1, l0_part, n_l0, ev, ev_a, ev_b, scalars,
                             l1l0_out, host_out, seq, B, n, d, stream);
}

int cc_loss_finalize_nb(const float* row_part, int64_t ncb_rows, const float* l1_part, int64_t n_l1,
                        const float* l0_part, int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars,
                        float* l1l0_out, float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, void* stream) {
  if (!row_part || !scalars) return CC_ERR_NULL;
  if (B <= 0 || n <= 0 || d <= 0 || ncb_rows <= 0) return CC_ERR_SHAPE;
  // the per-block partials of the row terms use the tail of `scalars` (cc_loss_scalars_len)
  int ncb = (int)ncb_rows;
  int nblk = (int)((B + 255) / 256);
  float* ev_part = scalars + 8;
  hipStream_t st = (hipStream_t)stream;
  const EvSeg e = {row_part, (int)B, (int)n, ncb, ev, ev_a, ev_b, ev_part, nblk};
  hipLaunchKernelGGL(ev_kernel, dim3(nblk), dim3(256), 0, st, e);
  const ScalArgs s = {ev_part, nblk, l1_part, n_l1, l0_part, n_l0, (int)B, scalars, l1l0_out, host_out, (unsigned)seq};
  hipLaunchKernelGGL(loss_scalars_kernel, dim3(1), dim3(LOSS_THREADS), 0, st, s);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_clip_finalize(const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16, float* out,
                     void* stream) {
  if (!sq || !off || !out) return CC_ERR_NULL;
  if (nparams <= 0 || nparams > 8) return CC_ERR_SHAPE;
  ClipArgs a = {};
  a.sq = sq;
  for (int i = 0; i <= nparams; ++i) a.off[i] = off[i];
  a.nparams = nparams;
  a.max_norm = max_norm;
  a.emulate_bf16 = emulate_bf16;
  a.out = out;
  hipLaunchKernelGGL(clip_kernel, dim3(1), dim3(SCAL_THREADS), 0, (hipStream_t)stream, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_segment_sums(const float* sq, const int64_t* off, int nparams, int zero_mask, float* out, void* stream) {
  if (!sq || !off || !out) return CC_ERR_NULL;
  if (nparams <= 0 || nparams > 8) return CC_ERR_SHAPE;
  ClipArgs a = {};
  a.sq = sq;
  for (int i = 0; i <= nparams; ++i) a.off[i] = off[i];
  a.nparams = nparams;
  a.out = out;
  a.sums_only = 1;
  a.zero_mask = zero_mask;
  hipLaunchKernelGGL(clip_kernel, dim3(1), dim3(SCAL_THREADS), 0, (hipStream_t)stream, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

}  // extern "C"

static AdamArgs adam_args(void* p, const void* g, void* m, void* v, int64_t numel, const float* coef, double lr,
                          double beta1, double beta2, double eps, int64_t step) {
  AdamArgs a = {};
  a.p = p; a.g = g; a.m = m; a.v = v; a.numel = numel; a.coef = coef;
  // host-side scalars in double, as torch computes them from python floats (adam.py)
  double b1 = beta1, b2 = beta2;
  a.w1 = (float)(1.0 - b1);
  a.beta2 = beta2;
  a.omb2 = (float)(1.0 - b2);
  a.eps = eps;
  double bc1 = 1.0 - pow(b1, (double)step), bc2 = 1.0 - pow(b2, (double)step);
  a.bc2s = (float)sqrt(bc2);
  a.neg_step = (float)(-((double)lr / bc1));
  return a;
}
static int adam_launch(const AdamArgs& a, int64_t max_blocks, int dtype, hipStream_t st);
static int64_t adam_capped_blocks(int64_t numel, int64_t max_blocks);

extern "C" {

int cc_adam_dec_transposed(void* p, const void* g, void* m, void* v, int64_t h, int64_t K, const float* coef,
                           double lr, double beta1, double beta2, double eps, int64_t step, int64_t max_blocks,
                           void* W_dec_t, float* part, int dtype, void* stream) {
  if (!p || !g || !m || !v || !W_dec_t || !part) return CC_ERR_NULL;
  if (dtype != CC_BF16) return CC_ERR_DTYPE;
  if (h <= 0 || K <= 0 || h % 8 || K % 64 || step <= 0 || h > (1 << 30)) return CC_ERR_SHAPE;
  if (!al16(p) || !al16(g) || !al16(m) || !al16(v) || !al16(W_dec_t)) return CC_ERR_ALIGN;
  const AdamArgs a = adam_args(p, g, m, v, h * K, coef, lr, beta1, beta2, eps, step);
  const int64_t ntiles = ((h + 63) / 64) * (K / 64);
  const int64_t blocks = max_blocks > 0 && max_blocks < ntiles ? max_blocks : ntiles;
  hipLaunchKernelGGL(adam_dec_tr_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, (int)h, (int)K,
                     (char*)W_dec_t, part);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_adam_step(void* p, const void* g, void* m, void* v, int64_t numel, const float* coef, double lr, double beta1,
                 double beta2, double eps, int64_t step, int64_t max_blocks, int dtype, void* stream) {
  if (!p || !g || !m || !v) return CC_ERR_NULL;
  if (numel <= 0 || step <= 0) return CC_ERR_SHAPE;
  if (!al16(p) || !al16(g) || !al16(m) || !al16(v)) return CC_ERR_ALIGN;
  return adam_launch(adam_args(p, g, m, v, numel, coef, lr, beta1, beta2, eps, step), max_blocks, dtype,
                     (hipStream_t)stream);
}

int cc_adam_step_clip(void* p, const void* g, void* m, void* v, int64_t numel, const float* sums, int nparams,
                      float max_norm, int emulate_bf16, float* clip_out, double lr, double beta1, double beta2,
                      double eps, int64_t step, int64_t max_blocks, int dtype, void* stream) {
  if (!p || !g || !m || !v || !sums) return CC_ERR_NULL;
  if (numel <= 0 || step <= 0 || nparams <= 0 || nparams > 6) return CC_ERR_SHAPE;
  if (!al16(p) || !al16(g) || !al16(m) || !al16(v)) return CC_ERR_ALIGN;
  AdamArgs a = adam_args(p, g, m, v, numel, nullptr, lr, beta1, beta2, eps, step);
  a.clip_sums = sums;
  a.clip_np = nparams;
  a.clip_emulate = emulate_bf16;
  a.clip_max_norm = max_norm;
  a.clip_out = clip_out;
  return adam_launch(a, max_blocks, dtype, (hipStream_t)stream);
}

int64_t cc_adam_capped_blocks(int64_t numel, int64_t max_blocks) {
  return numel > 0 && max_blocks > 0 ? adam_capped_blocks(numel, max_blocks) : 0;
}

int cc_adam_dec_norms(void* p, const void* g, void* m, void* v, int64_t numel, const float* coef, const float* sums,
                      int nparams, float max_norm, int emulate_bf16, double lr, double beta1, double beta2,
                      double eps, int64_t step, int64_t max_blocks, float* norm_part, int64_t h, int64_t K, int dtype,
                      uint32_t* done_ctr, void* stream) {
  if (!p || !g || !m || !v || !norm_part || (!coef && !sums)) return CC_ERR_NULL;
  if (done_ctr && max_blocks <= 0) return CC_ERR_SHAPE;  // (the signal is the capped grid-stride forms')
  if (numel <= 0 || step <= 0 || h <= 0 || K <= 0 || K % 64 || h * K > numel || h * K >= ((int64_t)1 << 31))
    return CC_ERR_SHAPE;
  if (sums && (nparams <= 0 || nparams > 6)) return CC_ERR_SHAPE;
  if (!al16(p) || !al16(g) || !al16(m) || !al16(v) || !al16(norm_part)) return CC_ERR_ALIGN;
  AdamArgs a = adam_args(p, g, m, v, numel, sums ? nullptr : coef, lr, beta1, beta2, eps, step);
  if (sums) {
    a.clip_sums = sums;
    a.clip_np = nparams;
    a.clip_emulate = emulate_bf16;
    a.clip_max_norm = max_norm;
  }
  a.norm_part = norm_part;
  a.norm_rows = (int)h;
  a.norm_ld = (int)K;
  a.done_ctr = done_ctr;
  // (the grid-stride form: the bulk kernel does not form the partials)
  return adam_launch(a, max_blocks > 0 ? max_blocks : 1024, dtype, (hipStream_t)stream);
}

}  // extern "C"

// workgroups of adam_launch's capped grid-stride form
static int64_t adam_capped_blocks(int64_t numel, int64_t max_blocks) {
  const int64_t blocks = ((numel + 7) / 8 + 255) / 256;
  return blocks > max_blocks ? max_blocks : blocks;
}
static int adam_launch(const AdamArgs& a, int64_t max_blocks, int dtype, hipStream_t st) {
  const int64_t numel = a.numel;
  if (max_blocks > 0) {  // capped grid-stride form: leaves most CUs to a concurrent GEMM
    const int64_t blocks = adam_capped_blocks(numel, max_blocks);
    if (dtype == CC_BF16 && numel % 8 == 0) {
      hipLaunchKernelGGL(adam_pipe_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
      CC_LAUNCH_CHECK();
      return CC_OK;
    }
    DISPATCH_DT(dtype, hipLaunchKernelGGL((adam_kernel<DT_>), dim3((unsigned)blocks), dim3(256), 0, st, a));
    CC_LAUNCH_CHECK();
    return CC_OK;
  }
  const int64_t nchunks = numel / 8;
  if (nchunks > 0) {
    const int64_t blocks = (nchunks + 256 * ADAM_U - 1) / (256 * ADAM_U);
    DISPATCH_DT(dtype, hipLaunchKernelGGL((adam_bulk_kernel<DT_, ADAM_U>), dim3((unsigned)blocks), dim3(256), 0,
                                          st, a, nchunks));
    CC_LAUNCH_CHECK();
  }
  if (numel % 8) {  // the last < 8 elements
    const int es = dtype == CC_BF16 ? 2 : 4;
    const int64_t off = nchunks * 8 * es;
    AdamArgs t = a;
    t.p = (char*)a.p + off; t.g = (const char*)a.g + off; t.m = (char*)a.m + off; t.v = (char*)a.v + off;
    t.numel = numel % 8;
    DISPATCH_DT(dtype, hipLaunchKernelGGL((adam_kernel<DT_>), dim3(1), dim3(256), 0, st, t));
    CC_LAUNCH_CHECK();
  }
  return CC_OK;
}

extern "C" {


static int grad_tail(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                     const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                     const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16,
                     int sums_only, int zero_mask, float* out, uint32_t* counter, void* stream,
                     const uint32_t* abort = nullptr) {
  if (!gpre_colpart || !g_b_enc || !sq_b_enc || !loss_colpart || !g_b_dec || !sq_b_dec || !sq || !off || !out ||
      !counter)
    return CC_ERR_NULL;
  if (R_enc <= 0 || R_dec <= 0 || h <= 0 || K <= 0) return CC_ERR_SHAPE;
  if (nparams <= 0 || nparams > 8) return CC_ERR_SHAPE;
  TailArgs a = {};
  a.red[0] = {gpre_colpart, (int)R_enc, (int)h, h, 1.f, nullptr, g_b_enc, sq_b_enc, nullptr, nullptr};
  a.red[1] = {loss_colpart, (int)R_dec, (int)K, K, 1.f, nullptr, g_b_dec, sq_b_dec, nullptr, nullptr};
  a.red_blocks[0] = (int)((h + RED_COLS - 1) / RED_COLS);
  a.red_blocks[1] = (int)((K + RED_COLS - 1) / RED_COLS);
  a.clip.sq = sq;
  for (int i = 0; i <= nparams; ++i) a.clip.off[i] = off[i];
  a.clip.nparams = nparams;
  a.clip.max_norm = max_norm;
  a.clip.emulate_bf16 = emulate_bf16;
  a.clip.out = out;
  a.clip.sums_only = sums_only;
  a.clip.zero_mask = zero_mask;
  a.clip.abort = abort;
  a.counter = counter;
  dim3 grid((unsigned)((a.red_blocks[0] + a.red_blocks[1] + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_DT(dtype, hipLaunchKernelGGL((tail_kernel<DT_>), grid, dim3(SCAL_THREADS), 0, st, a));
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_grad_tail(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                 const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                 const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16, float* clip_out,
                 uint32_t* counter, void* stream) {
  return grad_tail(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec, sq_b_dec, dtype, sq,
                   off, nparams, max_norm, emulate_bf16, 0, 0, clip_out, counter, stream);
}

// cc_grad_tail with the step's abort word (ClipArgs::abort): the fused G4G5 entry's fallback (library-internal)
int cc_grad_tail_abort(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                       const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                       const float* sq, const int64_t* off, int nparams, float max_norm, int emulate_bf16,
                       float* clip_out, uint32_t* counter, const uint32_t* abort, void* stream) {
  return grad_tail(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec, sq_b_dec, dtype, sq,
                   off, nparams, max_norm, emulate_bf16, 0, 0, clip_out, counter, stream, abort);
}

// (library-internal: cc_grad_tail_sums with the step's abort word -- the latent-sharded step's fallback form)
extern "C" int cc_grad_tail_sums_abort(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc,
                                       float* sq_b_enc, const float* loss_colpart, int64_t R_dec, int64_t K,
                                       void* g_b_dec, float* sq_b_dec, int dtype, const float* sq, const int64_t* off,
                                       int nparams, int zero_mask, float* out, uint32_t* counter,
                                       const uint32_t* abort, void* stream) {
  return grad_tail(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec, sq_b_dec, dtype, sq,
                   off, nparams, 0.f, 0, 1, zero_mask, out, counter, stream, abort);
}

int cc_grad_tail_sums(const float* gpre_colpart, int64_t R_enc, int64_t h, void* g_b_enc, float* sq_b_enc,
                      const float* loss_colpart, int64_t R_dec, int64_t K, void* g_b_dec, float* sq_b_dec, int dtype,
                      const float* sq, const int64_t* off, int nparams, int zero_mask, float* out, uint32_t* counter,
                      void* stream) {
  return grad_tail(gpre_colpart, R_enc, h, g_b_enc, sq_b_enc, loss_colpart, R_dec, K, g_b_dec, sq_b_dec, dtype, sq,
                   off, nparams, 0.f, 0, 1, zero_mask, out, counter, stream);
}

int cc_loss_tail(const float* colsum_acts, const float* tn, int64_t h, float* l1_part, const float* row_part,
                 int64_t ncb, const float* l0_part, int64_t n_l0, float* ev, float* ev_a, float* ev_b, float* scalars,
                 float* l1l0_out, float* host_out, uint32_t seq, int64_t B, int64_t n, int64_t d, uint32_t* counter,
                 void* stream) {
  if (!colsum_acts || !tn || !l1_part || !row_part || !scalars || !counter) return CC_ERR_NULL;
  if (h <= 0 || B <= 0 || n <= 0 || d <= 0 || ncb <= 0) return CC_ERR_SHAPE;
  const LossTailArgs a = make_loss_tail_args(colsum_acts, tn, h, l1_part, row_part, ncb, l0_part, n_l0, ev, ev_a, ev_b,
                                             scalars, l1l0_out, host_out, seq, B, n, counter);
  const int nblk = a.ev.nblk;
  hipLaunchKernelGGL(loss_tail_kernel, dim3((unsigned)(a.l1_wgs + nblk)), dim3(LOSS_THREADS), 0,
                     (hipStream_t)stream, a);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

}  // extern "C"
