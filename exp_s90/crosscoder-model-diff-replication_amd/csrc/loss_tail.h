// Loss-tail building blocks shared by the stand-alone kernels (step_kernels.hip) and the d_acts GEMM that
// carries the loss tail in its launch (gemm.hip): per-row explained variances + their partial sums, the l1
// partials, and the single-block loss-scalar finaliser.  Included inside namespace cc.
#pragma once

// Per-row explained variances (crosscoder.py:110-121) + per-block partial sums of the row terms.
// grid ceil(B/256), block 256. part_out[blk][4] = {sum l2_row, sum ev, sum ev_a, sum ev_b}.
struct EvSeg {
  const float* row_part;
  int B, n, ncb;
  float* ev;
  float* ev_a;
  float* ev_b;
  float* part_out;
  int nblk;  // ceil(B / 256) blocks (used by the fused tails)
};
CC_DEV void ev_phase1(const EvSeg& a, int blk, int t, float (*red)[4]) {
  const int r = blk * 256 + t;
  float v[4] = {0, 0, 0, 0};
  if (r < a.B) {
    const int B = a.B, n = a.n, ncb = a.ncb;
    const int64_t plane = (int64_t)n * ncb * B;
    const float eps = 1e-8f;
    float l2 = 0.f, tv = 0.f, l2m[2] = {0, 0}, tvm[2] = {0, 0};
    for (int m = 0; m < n; ++m) {
      float s = 0.f, u = 0.f;
      // 8 column blocks' loads in flight per trip (clamped index, no branch around a load), then the
      // in-order adds: the sequential sum's bits with one memory latency per 8 blocks
      for (int cb0 = 0; cb0 < ncb; cb0 += 8) {
        float vs[8], vu[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int cb = cb0 + q < ncb ? cb0 + q : ncb - 1;
          vs[q] = a.row_part[(int64_t)(m * ncb + cb) * B + r];
          vu[q] = a.row_part[plane + (int64_t)(m * ncb + cb) * B + r];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (cb0 + q < ncb) {
            s += vs[q];
            u += vu[q];
          }
        }
      }
      l2 += s;
      tv += u;
      if (m < 2) { l2m[m] = s; tvm[m] = u; }
    }
    float e = 1.f - l2 / (tv + eps);
    float ea = 1.f - l2m[0] / (tvm[0] + eps);
    float eb = n > 1 ? 1.f - l2m[1] / (tvm[1] + eps) : 0.f;
    if (a.ev) a.ev[r] = e;
    if (a.ev_a) a.ev_a[r] = ea;
    if (a.ev_b) a.ev_b[r] = eb;
    v[0] = l2; v[1] = e; v[2] = ea; v[3] = eb;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float s = wave_sum(v[q]);
    if ((t & 63) == 0) red[t >> 6][q] = s;
  }
}
CC_DEV void ev_phase2(const EvSeg& a, int blk, int t, float (*red)[4]) {
  if (t < 4) {
    int q = t;
    a.part_out[blk * 4 + q] = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
  }
}
// Single block: scalars = {l2, l1, l0, mean ev, mean ev_a, mean ev_b}.  NT threads: LOSS_THREADS in both the
// stand-alone finaliser and the fused loss tail (the same fp64 accumulation order, so the same bits); red: LDS
// scratch of the caller.
constexpr int SCAL_THREADS = 1024;  // (the clip finaliser's block)
constexpr int LOSS_THREADS = 256;
struct ScalArgs {
  const float* ev_part;
  int nblk;
  const float* l1_part;
  int64_t n_l1;
  const float* l0_part;
  int64_t n_wave;
  int B;
  float* scalars;
  float* l1l0_out;
  float* host_out;
  unsigned seq;
};
// (Called by every thread of a block of >= NT threads; threads from NT on take no part but the barriers.)
template <int NT>
CC_DEV void loss_scalars_body(const ScalArgs& sa, double (*red)[6]) {
  const float* __restrict__ ev_part = sa.ev_part;
  const int nblk = sa.nblk;
  const float* __restrict__ l1_part = sa.l1_part;
  const int64_t n_l1 = sa.n_l1;
  const float* __restrict__ l0_part = sa.l0_part;
  const int64_t n_wave = sa.n_wave;
  const int B = sa.B;
  float* __restrict__ scalars = sa.scalars;
  float* __restrict__ l1l0_out = sa.l1l0_out;
  float* __restrict__ host_out = sa.host_out;
  const unsigned seq = sa.seq;
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x < NT ? (int)threadIdx.x : (1 << 30);  // (no element for threads >= NT)
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int i = tid; i < nblk; i += NT) {
    acc[0] += ev_part[i * 4 + 0];
    acc[3] += ev_part[i * 4 + 1];
    acc[4] += ev_part[i * 4 + 2];
    acc[5] += ev_part[i * 4 + 3];
  }
  // 8 independent loads in flight per trip (clamped index, no branch around a load); each thread still adds
  // its elements i, i + NT, i + 2 NT, ... in order
  if (l0_part) {
    for (int64_t i = tid; i < n_wave; i += 8 * NT) {
      float b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t j = i + u * NT;
        b[u] = j < n_wave ? l0_part[j < n_wave ? j : 0] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[2] += b[u];
    }
  }
  if (l1_part)
    for (int64_t i = tid; i < n_l1; i += NT) acc[1] += l1_part[i];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    double s = wave_sum_d(acc[q]);
    if ((threadIdx.x & 63) == 0 && threadIdx.x < NT) red[threadIdx.x >> 6][q] = s;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    int q = threadIdx.x;
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += red[w][q];
    scalars[q] = (float)(s / (double)B);
    if (l1l0_out && (q == 1 || q == 2)) l1l0_out[q - 1] = (float)(s / (double)B);
    if (host_out) host_out[q] = (float)(s / (double)B);
  }
  if (threadIdx.x == 6 || threadIdx.x == 7) {
    scalars[threadIdx.x] = 0.f;
    if (host_out) host_out[threadIdx.x] = 0.f;
  }
  if (host_out) {
    // mapped pinned host memory: the 8 values reach the host before the sequence word the host
    // polls (no copy kernel, no event on the stream)
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store((unsigned*)(host_out + 8), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


// The forward's loss tail (crosscoder.py:106-128) as work items of a launch:
//   items [0, l1_wgs): 4 blocks of 64 latents, one per wave: B * l1's partial sum_j colsum[j] * tn[j] -- the dot
//     reduce_rows_phase2 forms (colsum IS that reduction of the encoder's column slab, scale 1): the same bits;
//   items [l1_wgs, l1_wgs + ev_blocks): 256 batch rows each (ev_phase1/2);
// then the last participant to arrive runs loss_scalars_body<LOSS_THREADS>.
struct LossTailArgs {
  const float* colsum;
  const float* tn;
  int h;
  float* l1_part;
  int l1_wgs;
  EvSeg ev;
  ScalArgs scal;
  unsigned* counter;
};
// One item by a 256-thread group (t = thread in the group, evred: 16 floats of the group's LDS).  The EV item
// has a barrier between its phases: every 256-thread group of the workgroup calls this the same number of times
// (item < 0: none, barriers only).
CC_DEV void loss_tail_item(const LossTailArgs& a, int item, int t, float (*evred)[4]) {
  if (item >= 0 && item < a.l1_wgs) {
    const int lane = t & 63, blk = item * 4 + (t >> 6), j = blk * 64 + lane;
    float dot = j < a.h ? a.colsum[j] * a.tn[j] : 0.f;
    dot = wave_sum(dot);
    if (lane == 0 && blk * 64 < a.h) a.l1_part[blk] = dot;
  }
  const bool ev = item >= a.l1_wgs && item < a.l1_wgs + a.ev.nblk;
  if (ev) ev_phase1(a.ev, item - a.l1_wgs, t, evred);
  __syncthreads();
  if (ev) ev_phase2(a.ev, item - a.l1_wgs, t, evred);
}

// LossTailArgs of cc_loss_tail / a cc_loss_tail_job (host side).
static inline LossTailArgs make_loss_tail_args(const float* colsum_acts, const float* tn, int64_t h, float* l1_part,
                                               const float* row_part, int64_t ncb, const float* l0_part, int64_t n_l0,
                                               float* ev, float* ev_a, float* ev_b, float* scalars, float* l1l0_out,
                                               float* host_out, uint32_t seq, int64_t B, int64_t n, uint32_t* counter) {
  LossTailArgs a = {};
  const int nred = (int)((h + 63) / 64);
  const int nblk = (int)((B + 255) / 256);
  float* ev_part = scalars + 8;  // as cc_loss_finalize (cc_loss_scalars_len)
  a.colsum = colsum_acts;
  a.tn = tn;
  a.h = (int)h;
  a.l1_part = l1_part;
  a.l1_wgs = (nred + 3) / 4;
  a.ev = {row_part, (int)B, (int)n, (int)ncb, ev, ev_a, ev_b, ev_part, nblk};
  a.scal = {ev_part, nblk, l1_part, nred, l0_part, n_l0, (int)B, scalars, l1l0_out, host_out, (unsigned)seq};
  a.counter = counter;
  return a;
}
