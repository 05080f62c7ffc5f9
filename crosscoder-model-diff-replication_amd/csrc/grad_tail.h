// Gradient-tail building blocks shared by the stand-alone tail kernels (step_kernels.hip) and the
// weight-gradient GEMM that runs the grad tail in its own launch (gemm.hip): fixed-order column
// reductions of partial slabs and the clip_grad_norm_ finaliser.  Included inside namespace cc.
#pragma once

// ---------------------------------------------------------------------------------------
// out[j] = scale * sum_i part[i*ld + j]; optional dtype copy, squared-sum partial per block and
// dot partial per block (sum_j out[j] * dot_w[j]: the L1 loss from the activation column sums).
// Block = 64 columns x 4 waves; wave w sums rows w, w+4, ... (independent loads in flight),
// then a fixed-order combine of the 4 wave partials.  One sq / dot partial per block.
constexpr int RED_COLS = 64;
// Phase 1 (all 4 waves of a 256-thread group, t = thread in the group): column sums into red;
// phase 2 (after a barrier, wave 0 of the group): outputs + the group's sq / dot partial.  The
// stand-alone kernel and the fused tail kernels (grad_tail / loss_tail) run the same two phases.
struct RedSeg {
  const float* part;
  int R, C;
  int64_t ld;
  float scale;
  float* out_f32;
  void* out_t;
  float* sq_part;
  const float* dot_w;
  float* dot_part;
};
CC_DEV void reduce_rows_phase1(const RedSeg& a, int blk, int t, float (*red)[RED_COLS]) {
  const int lane = t & 63, wave = t >> 6;
  const int j = blk * RED_COLS + lane;
  float s = 0.f;
  if (j < a.C) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int i = wave;
    for (; i + 12 < a.R; i += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += a.part[(int64_t)(i + 4 * u) * a.ld + j];
    }
    for (; i < a.R; i += 4) v[0] += a.part[(int64_t)i * a.ld + j];
    s = (v[0] + v[1]) + (v[2] + v[3]);
  }
  red[wave][lane] = s;
}
template <int DT>
CC_DEV void reduce_rows_phase2(const RedSeg& a, int blk, int t, float (*red)[RED_COLS]) {
  if ((t >> 6) != 0) return;
  const int lane = t & 63;
  const int j = blk * RED_COLS + lane;
  float sq = 0.f, dot = 0.f;
  if (j < a.C) {
    float s = (((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]) * a.scale;
    if (a.out_f32) a.out_f32[j] = s;
    if (a.out_t) {
      typename Elem<DT>::T q = Elem<DT>::from_f(s);
      ((typename Elem<DT>::T*)a.out_t)[j] = q;
      float vq = Elem<DT>::to_f(q);
      sq = vq * vq;
    }
    if (a.dot_part) dot = s * a.dot_w[j];
  }
  if (a.sq_part) {
    sq = wave_sum(sq);
    if (lane == 0) a.sq_part[blk] = sq;
  }
  if (a.dot_part) {
    dot = wave_sum(dot);
    if (lane == 0) a.dot_part[blk] = dot;
  }
}
CC_DEV float bf16r(float f) { return bf2f(f2bf(f)); }

// clip_grad_norm_'s scalar arithmetic (torch/nn/utils/clip_grad.py): a parameter's norm from its squared sum
// (bf16-rounded as torch._foreach_norm on bf16 returns bf16), then the total norm and the coefficient
CC_DEV float clip_param_norm(double sq, int emulate_bf16) {
  const float nr = (float)sqrt(sq);
  return emulate_bf16 ? bf16r(nr) : nr;
}
CC_DEV float clip_coef(const float* norms, int nparams, float max_norm, int emulate_bf16, float& total) {
  float s = 0.f;
  for (int p = 0; p < nparams; ++p) s += norms[p] * norms[p];
  total = sqrtf(s);
  if (emulate_bf16) {
    total = bf16r(total);                       // vector_norm(stack(bf16 norms)) -> bf16
    const float den = bf16r(total + 1e-6f);     // bf16 tensor + python scalar
    return fminf(bf16r(max_norm / den), 1.f);
  }
  return fminf(max_norm / (total + 1e-6f), 1.f);
}

struct ClipArgs {
  const float* sq;
  int64_t off[9];
  int nparams;
  float max_norm;
  int emulate_bf16;
  float* out;
  int sums_only;   // cc_segment_sums: out[p] = the raw per-parameter sum (0 where zero_mask has bit p)
  int zero_mask;
  // the step's abort word (a host-mapped word an earlier launch of the step sets when it could not run, e.g. G2's
  // in-kernel wait timing out): when set, the coefficient is written as CC_CLIP_ABORTED and every Adam launch
  // that reads it leaves p / m / v untouched (nullptr: none)
  const unsigned* abort;
};
// clip_out[0] of a step that must not update the parameters: clip_grad_norm_'s coefficient min(1, max_norm /
// (total + 1e-6)) is never negative (NaN / inf norms give NaN / 0), so a negative value is free to mean it
#define CC_CLIP_ABORTED (-1.0f)
// One block of NT threads; red / norms: LDS scratch of the caller (the GEMM kernel that runs it as
// its last workgroup's tail has no LDS to spare for static arrays of its own)
template <int NT>
CC_DEV void clip_finish(const ClipArgs& a, const double* s, double (*red)[NT / 64], float* norms);
template <int NT>
CC_DEV void clip_body(const ClipArgs& a, double (*red)[NT / 64], float* norms) {
  // all parameters in one pass: each thread keeps one running sum per parameter
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    if (p < a.nparams) {
      const int64_t lo = a.off[p], hi = a.off[p + 1];
      // 4 independent loads in flight per trip (clamped index, no branch around a load)
      for (int64_t i = lo + threadIdx.x; i < hi; i += 4 * NT) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t j = i + u * NT;
          v[u] = j < hi ? a.sq[j < hi ? j : lo] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) s[p] += (double)v[u];
      }
    }
  }
  clip_finish<NT>(a, s, red, norms);
}

// The finaliser from per-thread partial sums s[p] (every thread of the block): fixed-order combine of
// the waves, per-parameter norms (bf16-rounded as torch's _foreach_norm on bf16), total, coefficient.
template <int NT>
CC_DEV void clip_finish(const ClipArgs& a, const double* s, double (*red)[NT / 64], float* norms) {
  // (the abort word may live in host memory: its load is issued first, its latency hides under the reductions)
  const unsigned aborted =
      threadIdx.x == 0 && a.abort ? __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    double t = wave_sum_d(s[p]);
    if ((threadIdx.x & 63) == 0) red[p][threadIdx.x >> 6] = t;
  }
  __syncthreads();
  if (a.sums_only) {
    if (threadIdx.x < a.nparams) {
      const int p = threadIdx.x;
      // (the step was aborted -- G2's in-kernel wait timed out, ClipArgs::abort: -inf for every parameter, so the
      // sums' all-reduce carries the abort to every rank and each Adam launch that forms its coefficient from them
      // applies nothing, adam_coef.  Each of these threads reads the word itself.)
      const bool ab = a.abort && __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
      double t = 0.0;
      for (int w = 0; w < NT / 64; ++w) t += red[p][w];
      a.out[p] = ab ? -__builtin_inff() : ((a.zero_mask >> p) & 1 ? 0.f : (float)t);
    }
    return;
  }
  if (threadIdx.x < a.nparams) {
    const int p = threadIdx.x;
    double t = 0.0;
    for (int w = 0; w < NT / 64; ++w) t += red[p][w];
    norms[p] = clip_param_norm(t, a.emulate_bf16);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float total;
    const float coef = clip_coef(norms, a.nparams, a.max_norm, a.emulate_bf16, total);
    a.out[0] = aborted ? CC_CLIP_ABORTED : coef;
    a.out[1] = total;
    for (int p = 0; p < a.nparams; ++p) a.out[2 + p] = norms[p];
  }
}

