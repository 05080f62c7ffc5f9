// Shared device/host helpers for the crosscoder HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/crosscoder_hip.h"

#define CC_DEV __device__ __forceinline__

namespace cc {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef uint16_t bf16_t;  // raw bits

// ---- bf16 <-> f32.  f32 -> bf16 is gfx950's v_cvt_pk_bf16_f32: round-to-nearest-even like
// torch's c10::BFloat16 (NaN stays NaN, quieted); one instruction instead of the integer
// rounding sequence and its NaN branch.
CC_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
CC_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// Storage element type of params / activations: bf16 (CC_BF16) or fp32 (CC_F32).
template <int DT> struct Elem;
template <> struct Elem<CC_BF16> {
  typedef bf16_t T;
  static CC_DEV float load(const T* p) { return bf2f(*p); }
  static CC_DEV float to_f(T v) { return bf2f(v); }
  static CC_DEV T from_f(float f) { return f2bf(f); }
  static CC_DEV float round(float f) { return bf2f(f2bf(f)); }
};
template <> struct Elem<CC_F32> {
  typedef float T;
  static CC_DEV float load(const T* p) { return *p; }
  static CC_DEV float to_f(T v) { return v; }
  static CC_DEV T from_f(float f) { return f; }
  static CC_DEV float round(float f) { return f; }
};

// 8 consecutive elements as floats (16 B bf16 or 32 B fp32 vector access).
template <int DT> CC_DEV void load8(const void* base, int64_t idx, float v[8]) {
  if constexpr (DT == CC_BF16) {
    bf16x8 r = *(const bf16x8*)((const bf16_t*)base + idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)r[j]);
  } else {
    const f32x4* p = (const f32x4*)((const float*)base + idx);
    f32x4 a = p[0], b = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
}
template <int DT> CC_DEV void store8(void* base, int64_t idx, const float v[8]) {
  if constexpr (DT == CC_BF16) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[j]);
    *(bf16x8*)((bf16_t*)base + idx) = r;
  } else {
    f32x4* p = (f32x4*)((float*)base + idx);
    p[0] = f32x4{v[0], v[1], v[2], v[3]};
    p[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
}
// Non-temporal (streamed-once) variants for the HBM-bound optimizer pass.
template <int DT> CC_DEV void load8_nt(const void* base, int64_t idx, float v[8]) {
  if constexpr (DT == CC_BF16) {
    bf16x8 r = __builtin_nontemporal_load((const bf16x8*)((const bf16_t*)base + idx));
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)r[j]);
  } else {
    const f32x4* p = (const f32x4*)((const float*)base + idx);
    f32x4 a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
}
template <int DT> CC_DEV void store8_nt(void* base, int64_t idx, const float v[8]) {
  if constexpr (DT == CC_BF16) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[j]);
    __builtin_nontemporal_store(r, (bf16x8*)((bf16_t*)base + idx));
  } else {
    f32x4* p = (f32x4*)((float*)base + idx);
    __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, p);
    __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, p + 1);
  }
}
CC_DEV void load8f(const float* base, int64_t idx, float v[8]) {
  const f32x4* p = (const f32x4*)(base + idx);
  f32x4 a = p[0], b = p[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
CC_DEV void load8f_nt(const float* base, int64_t idx, float v[8]) {
  const f32x4* p = (const f32x4*)(base + idx);
  f32x4 a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
// cache policy chosen at compile time: NT = non-temporal (read / written once in the step: keep the
// Infinity Cache for operands that are read again soon)
template <int DT, bool NT> CC_DEV void ld8(const void* b, int64_t i, float v[8]) {
  if constexpr (NT) load8_nt<DT>(b, i, v); else load8<DT>(b, i, v);
}
template <int DT, bool NT> CC_DEV void st8(void* b, int64_t i, const float v[8]) {
  if constexpr (NT) store8_nt<DT>(b, i, v); else store8<DT>(b, i, v);
}

CC_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over each aligned group of 16 lanes (a DPP row), the same bits as the xor-1/2/4/8 butterfly
// (every lane gets the sum); DPP moves instead of ds_bpermute: no LDS round trips.  xor 4 / xor 8
// become row_half_mirror / row_mirror, which pair the same quads / half-rows.  EXEC must be full.
// row16_sum of 4 independent values as 16 DPP adds (the same additions in the same order: v + perm(v) per
// step).  One asm block: hipcc otherwise pairs the dpp-moved values into packed adds (a DPP move, a 64-bit move
// and half a packed add per step); interleaving the 4 values keeps every DPP read >= 2 instructions after the
// write of its source, and the leading s_nop covers the compiler's last write before the block.
CC_DEV void row16_sum4(float (&v)[4]) {
  asm volatile(
      "s_nop 1\n"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %2, %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %3, %3, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %2, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %3, %3, %3 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_add_f32_dpp %3, %3, %3 row_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
CC_DEV float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// sum over each aligned group of 8 lanes (xor-1/2/4 butterfly: every lane of the group gets the
// same bits)
CC_DEV float block8_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}
CC_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// norms[r][m] = sqrt(sum of part[r][m*bpm .. (m+1)*bpm) in ascending order), total[r] = sum_m norms, inverses
// (0 where a norm is 0): the rest of dec_norms_kernel from the per-(row, 64-column block) partials.  Each
// lane issues NORM_LOADS independent loads before adding them in order (the sum is latency-bound: one
// dependent load per add took 15 us at config 2).  Shared by the stand-alone finaliser and the G2 launch
// that carries it.
constexpr int NORM_LOADS = 12;
CC_DEV void norms_finalize_row(const float* __restrict__ part, int row, int n, int bpm, float* __restrict__ norms,
                               float* __restrict__ total, float* __restrict__ inv_norms) {
  const float* p = part + (int64_t)row * n * bpm;
  float tot = 0.f;
  for (int m = 0; m < n; ++m) {
    float s = 0.f;
    for (int b0 = 0; b0 < bpm; b0 += NORM_LOADS) {
      float v[NORM_LOADS];
#pragma unroll
      for (int u = 0; u < NORM_LOADS; ++u) v[u] = b0 + u < bpm ? p[m * bpm + b0 + u] : 0.f;
#pragma unroll
      for (int u = 0; u < NORM_LOADS; ++u)
        if (b0 + u < bpm) s += v[u];
    }
    const float nr = sqrtf(s);
    norms[(int64_t)row * n + m] = nr;
    if (inv_norms) inv_norms[(int64_t)row * n + m] = nr > 0.f ? 1.f / nr : 0.f;
    tot += nr;
  }
  total[row] = tot;
}

}  // namespace cc

#define CC_LAUNCH_CHECK()                                \
  do {                                                   \
    hipError_t e__ = hipGetLastError();                  \
    if (e__ != hipSuccess) return CC_ERR_HIP_BASE + (int)e__; \
  } while (0)
