// HBM-bound kernels around the training step: the activation buffer's shuffle
// (Buffer.refresh, buffer.py:111-113), the activation-scale fold of the demo notebook
// (fold_activation_scaling_factor, Crosscoder_model_diff.ipynb:35368-35378) and the decoder-norm
// analytics of analysis.py:9-40.  gfx950; 16 B per lane everywhere.
#include "cc_common.h"

namespace cc {

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

// dst[i] = src[perm[i]] for rows of row_bytes (a multiple of 16).  One wave per destination row,
// 16 B per lane, 4 rows per 256-thread block; the permutation entry is read once per wave.
// An index outside [0, src_rows) yields a zero row (no out-of-bounds read).
__global__ __launch_bounds__(256) void gather_rows_kernel(const char* __restrict__ src, int64_t src_rows,
                                                          const int64_t* __restrict__ perm, char* __restrict__ dst,
                                                          int64_t rows, int64_t row_bytes) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t s = perm[row];
  const bool ok = s >= 0 && s < src_rows;
  const u32x4_t* sp = (const u32x4_t*)(src + (ok ? s : 0) * row_bytes);
  u32x4_t* dp = (u32x4_t*)(dst + row * row_bytes);
  const int64_t n16 = row_bytes / 16;
  int64_t c = lane;
  for (; c + 64 < n16; c += 128) {  // two 16-B loads in flight per lane
    const u32x4_t a = __builtin_nontemporal_load(sp + c), b = __builtin_nontemporal_load(sp + c + 64);
    __builtin_nontemporal_store(ok ? a : u32x4_t{0, 0, 0, 0}, dp + c);
    __builtin_nontemporal_store(ok ? b : u32x4_t{0, 0, 0, 0}, dp + c + 64);
  }
  if (c < n16) __builtin_nontemporal_store(ok ? __builtin_nontemporal_load(sp + c) : u32x4_t{0, 0, 0, 0}, dp + c);
}

// In place: W_enc[m] *= s[m], W_dec[:, m] /= s[m], b_dec[m] /= s[m] (W_dec / b_dec optional) with the parameter dtype's
// rounding after each op (torch: dtype tensor * python float computes in fp32, rounds once).
// W_enc / W_dec are [h][n*d] (W_enc's physical h-major layout), b_dec [n*d].  Thread -> 8 columns.
template <int DT>
__global__ __launch_bounds__(256) void fold_scaling_kernel(void* __restrict__ W_enc, void* __restrict__ W_dec,
                                                           void* __restrict__ b_dec, const float* __restrict__ scale,
                                                           int64_t h, int n, int d) {
  using E = Elem<DT>;
  const int64_t K = (int64_t)n * d;
  const int64_t i8 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;  // element index in [h + 1][K]
  if (i8 >= (h + 1) * K) return;
  const int64_t row = i8 / K, col = i8 - row * K;
  const float s = scale[col / d];
  float v[8];
  if (row < h) {
    load8<DT>(W_enc, i8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = E::round(v[j] * s);
    store8<DT>(W_enc, i8, v);
    if (W_dec) {
      load8<DT>(W_dec, i8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = E::round(v[j] / s);
      store8<DT>(W_dec, i8, v);
    }
  } else if (b_dec) {  // the extra row: b_dec
    load8<DT>(b_dec, col, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = E::round(v[j] / s);
    store8<DT>(b_dec, col, v);
  }
}

// Per latent (one wave): norms[h][m] = ||W_dec[h, m]||, relative[h] = norms[h][1] / sum_m norms[h][m],
// cosine[h] = <W_dec[h,0], W_dec[h,1]> / (norms[h][0] * norms[h][1])  (analysis.py:9-12, 40).
template <int DT>
__global__ __launch_bounds__(256) void decoder_stats_kernel(const void* __restrict__ W, int64_t h, int n, int d,
                                                            float* __restrict__ norms, float* __restrict__ relative,
                                                            float* __restrict__ cosine) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= h) return;
  const int64_t base = row * n * d;
  float sq0 = 0.f, sq1 = 0.f, dot = 0.f;
  for (int c = lane * 8; c < d; c += 512) {
    float a[8], b[8];
    load8<DT>(W, base + c, a);
    if (n > 1) load8<DT>(W, base + d + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sq0 += a[j] * a[j];
      if (n > 1) {
        sq1 += b[j] * b[j];
        dot += a[j] * b[j];
      }
    }
  }
  sq0 = wave_sum(sq0);
  sq1 = wave_sum(sq1);
  dot = wave_sum(dot);
  const float n0 = sqrtf(sq0), n1 = sqrtf(sq1);
  float tot = n0 + n1;
  for (int m = 2; m < n; ++m) {  // further models: norms only
    float s = 0.f;
    for (int c = lane * 8; c < d; c += 512) {
      float a[8];
      load8<DT>(W, base + (int64_t)m * d + c, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += a[j] * a[j];
    }
    s = sqrtf(wave_sum(s));
    if (lane == 0) norms[row * n + m] = s;
    tot += s;
  }
  if (lane == 0) {
    norms[row * n] = n0;
    if (n > 1) norms[row * n + 1] = n1;
    if (relative) relative[row] = n > 1 ? n1 / tot : 0.f;
    if (cosine) cosine[row] = n > 1 ? dot / (n0 * n1) : 0.f;
  }
}

// dst[c][r] = src[r][c] for 16-bit elements (rows, cols % 8 == 0).  64 x 64 tiles: 16-B loads into
// an LDS image [64 rows][128 B] (phys chunk = chunk ^ (row & 7)), read back column-wise with
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group -> lane i holds column i); two reads
// give a lane 8 consecutive rows = one 16-B store of a transposed row.
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
// NORMS: also the squared sum of each (row, 64-column block) of the source, in dec_norms_kernel's
// order (8 sequential fma per lane, xor-1/2/4 butterfly over the 8 lanes of a block row), into
// part[row][block] -- W_dec's decoder norms come out of the same HBM pass as W_dec^T.
template <bool NORMS>
__global__ __launch_bounds__(256) void transpose_b16_kernel(const char* __restrict__ src, int rows, int cols,
                                                            int64_t ld_src, char* __restrict__ dst, int64_t ld_dst,
                                                            int rows_fast, float* __restrict__ part, int nblk) {
  __shared__ __attribute__((aligned(16))) char tile[64 * 128];
  // rows_fast: consecutive blocks walk down the source rows (= along the destination rows)
  const int r0 = (rows_fast ? blockIdx.x : blockIdx.y) * 64, c0 = (rows_fast ? blockIdx.y : blockIdx.x) * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = threadIdx.x + 256 * k, r = idx >> 3, ch = idx & 7;
    u32x4_t v = {0, 0, 0, 0};
    if (r0 + r < rows && c0 + 8 * ch < cols)
      v = __builtin_nontemporal_load((const u32x4_t*)(src + ((int64_t)(r0 + r) * ld_src + c0 + 8 * ch) * 2));
    *(u32x4_t*)(tile + r * 128 + ((ch ^ (r & 7)) << 4)) = v;
    if constexpr (NORMS) {
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = __uint_as_float((j & 1 ? v[j >> 1] >> 16 : v[j >> 1] & 0xffffu) << 16);
        q = __fmaf_rn(f, f, q);
      }
      q = block8_sum(q);
      if (ch == 0 && r0 + r < rows) part[(int64_t)(r0 + r) * nblk + (c0 >> 6)] = q;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ca = 16 * w + 4 * p, ch = ca >> 3;  // address column of this lane
  const int c = 16 * w + i;                      // column delivered to this lane
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int R = (4 * s + g) * 8;
    const int l0 = R + q, l1 = R + 4 + q;
    const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(tile + l0 * 128 + ((ch ^ (l0 & 7)) << 4) + (ca & 4) * 2));
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(tile + l1 * 128 + ((ch ^ (l1 & 7)) << 4) + (ca & 4) * 2));
    const bf16x8 v = bf16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    if (c0 + c < cols && r0 + R < rows)
      *(bf16x8*)(dst + ((int64_t)(c0 + c) * ld_dst + r0 + R) * 2) = v;
  }
}

// The decoder norms from their per-block partials (norms_finalize_row, cc_common.h): one thread per row, one
// wave per block (h/64 blocks spread over the CUs).
__global__ __launch_bounds__(64) void norms_finalize_kernel(const float* __restrict__ part, int h, int n, int bpm,
                                                            float* __restrict__ norms, float* __restrict__ total,
                                                            float* __restrict__ inv_norms) {
  const int row = blockIdx.x * 64 + threadIdx.x;
  if (row < h) norms_finalize_row(part, row, n, bpm, norms, total, inv_norms);
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace cc

using namespace cc;

extern "C" {

int cc_gather_rows(const void* src, int64_t src_rows, const int64_t* perm, void* dst, int64_t rows, int64_t row_bytes,
                   void* stream) {
  if (rows == 0) return CC_OK;  // (empty tensors may carry NULL data pointers)
  if (rows < 0 || src_rows < 0 || row_bytes <= 0 || row_bytes % 16) return CC_ERR_SHAPE;
  if (!src || !perm || !dst) return CC_ERR_NULL;
  if (!al16(src) || !al16(dst)) return CC_ERR_ALIGN;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const char*)src, src_rows, perm, (char*)dst, rows, row_bytes);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_transpose_b16(const void* src, int64_t rows, int64_t cols, int64_t ld_src, void* dst, int64_t ld_dst,
                     void* stream) {
  if (rows == 0 || cols == 0) return CC_OK;
  if (rows < 0 || cols < 0 || rows % 8 || cols % 8 || ld_src < cols || ld_dst < rows || ld_src % 8 || ld_dst % 8 ||
      rows / 64 >= 65535 || cols / 64 >= 65535)
    return CC_ERR_SHAPE;
  if (!src || !dst) return CC_ERR_NULL;
  if (!al16(src) || !al16(dst)) return CC_ERR_ALIGN;
  const unsigned nr = (unsigned)((rows + 63) / 64), nc = (unsigned)((cols + 63) / 64);
  // measured (tools/transpose_bench.py): walking the source rows first is faster when rows >= cols
  const int rf = rows >= cols;
  hipLaunchKernelGGL(transpose_b16_kernel<false>, rf ? dim3(nr, nc) : dim3(nc, nr), dim3(256), 0,
                     (hipStream_t)stream, (const char*)src, (int)rows, (int)cols, ld_src, (char*)dst, ld_dst, rf,
                     nullptr, 0);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int64_t cc_dec_norms_part_floats(int64_t h, int64_t n, int64_t d) { return d % 64 ? 0 : h * n * (d / 64); }

int cc_dec_norms_finalize(const float* part, int64_t h, int64_t n, int64_t d, float* norms, float* total,
                          float* inv_norms, void* stream) {
  if (!part || !norms || !total) return CC_ERR_NULL;
  if (h <= 0 || n <= 0 || d <= 0 || d % 64) return CC_ERR_SHAPE;
  hipLaunchKernelGGL(norms_finalize_kernel, dim3((unsigned)((h + 63) / 64)), dim3(64), 0, (hipStream_t)stream, part,
                     (int)h, (int)n, (int)(d / 64), norms, total, inv_norms);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_transpose_dec_norms(const void* W_dec, int64_t h, int64_t n, int64_t d, void* W_dec_t, float* part,
                           float* norms, float* total, float* inv_norms, void* stream) {
  if (!W_dec || !W_dec_t || !part || !norms || !total) return CC_ERR_NULL;
  const int64_t K = n * d;
  if (h <= 0 || n <= 0 || d <= 0 || d % 64 || h % 8 || h / 64 >= 65535 || K / 64 >= 65535) return CC_ERR_SHAPE;
  if (!al16(W_dec) || !al16(W_dec_t)) return CC_ERR_ALIGN;
  const unsigned nr = (unsigned)((h + 63) / 64), nc = (unsigned)(K / 64);
  const int rf = h >= K;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(transpose_b16_kernel<true>, rf ? dim3(nr, nc) : dim3(nc, nr), dim3(256), 0, st,
                     (const char*)W_dec, (int)h, (int)K, K, (char*)W_dec_t, h, rf, part, (int)(K / 64));
  hipLaunchKernelGGL(norms_finalize_kernel, dim3((unsigned)((h + 63) / 64)), dim3(64), 0, st, part, (int)h, (int)n,
                     (int)(d / 64), norms, total, inv_norms);
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_fold_scaling(void* W_enc, void* W_dec, void* b_dec, const float* scale, int64_t h, int64_t n, int64_t d,
                    int dtype, void* stream) {
  if (!W_enc || !scale) return CC_ERR_NULL;
  if (h <= 0 || n <= 0 || d <= 0 || d % 8) return CC_ERR_SHAPE;
  if (!al16(W_enc) || (W_dec && !al16(W_dec)) || (b_dec && !al16(b_dec))) return CC_ERR_ALIGN;
  const int64_t chunks = (h + 1) * n * d / 8;
  dim3 grid((unsigned)((chunks + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CC_BF16)
    hipLaunchKernelGGL((fold_scaling_kernel<CC_BF16>), grid, dim3(256), 0, st, W_enc, W_dec, b_dec, scale, h, (int)n,
                       (int)d);
  else if (dtype == CC_F32)
    hipLaunchKernelGGL((fold_scaling_kernel<CC_F32>), grid, dim3(256), 0, st, W_enc, W_dec, b_dec, scale, h, (int)n,
                       (int)d);
  else
    return CC_ERR_DTYPE;
  CC_LAUNCH_CHECK();
  return CC_OK;
}

int cc_decoder_stats(const void* W_dec, int64_t h, int64_t n, int64_t d, int dtype, float* norms, float* relative,
                     float* cosine, void* stream) {
  if (!W_dec || !norms) return CC_ERR_NULL;
  if (h <= 0 || n <= 0 || d <= 0 || d % 8) return CC_ERR_SHAPE;
  if (!al16(W_dec)) return CC_ERR_ALIGN;
  dim3 grid((unsigned)((h + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CC_BF16)
    hipLaunchKernelGGL((decoder_stats_kernel<CC_BF16>), grid, dim3(256), 0, st, W_dec, h, (int)n, (int)d, norms,
                       relative, cosine);
  else if (dtype == CC_F32)
    hipLaunchKernelGGL((decoder_stats_kernel<CC_F32>), grid, dim3(256), 0, st, W_dec, h, (int)n, (int)d, norms,
                       relative, cosine);
  else
    return CC_ERR_DTYPE;
  CC_LAUNCH_CHECK();
  return CC_OK;
}

}  // extern "C"
