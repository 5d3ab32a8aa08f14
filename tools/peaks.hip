// Achievable-peak probes for the roofline fractions bench.py reports
// (measure the box's own peaks next to the vendor ones).
//   dr_peak_mfma: back-to-back v_mfma_f32_32x32x16_bf16 on random bf16
//     operands, four independent accumulators per wave, two waves per SIMD
//     (the score scan's occupancy). Random data matters: the clock the chip
//     holds under BF16 load is lower on random operands than on zeros
//     (MI355X_MICROARCH.md, DVFS give-back).
//   dr_peak_copy: float4 grid-stride copy, four 16-B loads in flight per lane
//     (reaches ~4.9 TB/s; the guide measures 6.29 TB/s with its own copy, and
//     bench.py uses that figure as the achievable HBM rate).
// Measurement tooling only: built into tools/_peaks/libdivrec_peaks.so,
// never linked into the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512, 1) void peak_mfma_kernel(const uint4* __restrict__ src, int iters,
                                                          float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 512 + threadIdx.x;
  bf16x8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = __builtin_bit_cast(bf16x8, src[(t * 8 + i) & 0xFFFFF]);
    b[i] = __builtin_bit_cast(bf16x8, src[(t * 8 + 4 + i) & 0xFFFFF]);
  }
  f32x16 acc[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[i], acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[t] = s;
}

// Each thread moves 4 float4 per step, all four loads issued before the
// stores (16 B x 4 in flight per lane), in a grid-stride sweep.
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void peak_copy_kernel(const f32x4* __restrict__ src,
                                                        f32x4* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const f32x4 v0 = __builtin_nontemporal_load(src + i);
    const f32x4 v1 = __builtin_nontemporal_load(src + i + stride);
    const f32x4 v2 = __builtin_nontemporal_load(src + i + 2 * stride);
    const f32x4 v3 = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(v0, dst + i);
    __builtin_nontemporal_store(v1, dst + i + stride);
    __builtin_nontemporal_store(v2, dst + i + 2 * stride);
    __builtin_nontemporal_store(v3, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// src: >= 16 MiB of random bytes; out: grid * 512 floats.
extern "C" int dr_peak_mfma(const void* src, int grid, int iters, float* out, hipStream_t s) {
  hipLaunchKernelGGL(peak_mfma_kernel, dim3(grid), dim3(512), 0, s, (const uint4*)src, iters, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dr_peak_copy(const void* src, void* dst, int64_t bytes, int grid, hipStream_t s) {
  hipLaunchKernelGGL(peak_copy_kernel, dim3(grid), dim3(256), 0, s, (const f32x4*)src,
                     (f32x4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
