// Experiment (tools only, never shipped): sustained MFMA throughput of the two bf16 MFMA shapes on
// register-resident random operands, every CU busy, so the package power cap sets the clock.
// Tells whether v_mfma_f32_32x32x16_bf16 does more work per joule than v_mfma_f32_16x16x32_bf16.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

__device__ inline bf16x8 rnd8(uint32_t s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s = s * 1664525u + 1013904223u;
    v[j] = (short)(0x3c00 | ((s >> 16) & 0x807f));  // bf16 in [-2, 2) with random mantissa / sign
  }
  return v;
}

// 16x16x32: 8 independent accumulators (32 VGPR), 2 A x 4 B operands
__global__ __launch_bounds__(512, 1) void mfma16(float* out, int iters, int zero) {
  const uint32_t s = (blockIdx.x * 512 + threadIdx.x) * 2654435761u;
  bf16x8 a[2], b[4];
  for (int i = 0; i < 2; ++i) a[i] = zero ? bf16x8{} : rnd8(s + i);
  for (int j = 0; j < 4; ++j) b[j] = zero ? bf16x8{} : rnd8(s + 17 * j + 5);
  f32x4 acc[2][4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
  }
  float t = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * 512 + threadIdx.x] = t;
}

// 32x32x16: 2 independent accumulators (32 VGPR) -> same accumulator footprint, same flops per loop trip
__global__ __launch_bounds__(512, 1) void mfma32(float* out, int iters, int zero) {
  const uint32_t s = (blockIdx.x * 512 + threadIdx.x) * 2654435761u;
  bf16x8 a[2], b[2];
  for (int i = 0; i < 2; ++i) a[i] = zero ? bf16x8{} : rnd8(s + i);
  for (int j = 0; j < 2; ++j) b[j] = zero ? bf16x8{} : rnd8(s + 17 * j + 5);
  f32x16 acc[2] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[k], a[i], acc[i], 0, 0, 0);
  }
  float t = 0.f;
  for (int i = 0; i < 2; ++i) t += acc[i][0] + acc[i][15];
  out[blockIdx.x * 512 + threadIdx.x] = t;
}

extern "C" int mfma_run(int kind, float* out, int blocks, int iters, int zero, void* stream) {
  if (kind == 16) hipLaunchKernelGGL(mfma16, dim3(blocks), dim3(512), 0, (hipStream_t)stream, out, iters, zero);
  else hipLaunchKernelGGL(mfma32, dim3(blocks), dim3(512), 0, (hipStream_t)stream, out, iters, zero);
  return (int)hipGetLastError();
}
