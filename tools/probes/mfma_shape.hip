// MFMA shape probe (measurement tooling, not product code): back-to-back bf16
// MFMAs on random operands, 512-thread workgroups (two waves per SIMD, the
// score scan's occupancy), one workgroup per CU, for v_mfma_f32_32x32x16_bf16
// and v_mfma_f32_16x16x32_bf16 at equal flops per iteration. Under sustained
// full-chip load the clock the chip holds depends on the instruction mix
// (MI355X_MICROARCH.md reports ~1.15x the FLOP/s for the 16x16x32 loop); this
// probe measures it on this box for the scan's next-step decision.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512, 1) void mfma32_kernel(const uint4* __restrict__ src, int iters,
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

// 16x16x32: half the flops per instruction, so 8 per iteration (same flops
// per iteration as the 4 above), 8 independent accumulators.
__global__ __launch_bounds__(512, 1) void mfma16_kernel(const uint4* __restrict__ src, int iters,
                                                       float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 512 + threadIdx.x;
  bf16x8 a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = __builtin_bit_cast(bf16x8, src[(t * 16 + i) & 0xFFFFF]);
    b[i] = __builtin_bit_cast(bf16x8, src[(t * 16 + 8 + i) & 0xFFFFF]);
  }
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[i], acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[t] = s;
}

extern "C" int probe_mfma(int shape, const void* src, int grid, int iters, float* out, hipStream_t s) {
  if (shape == 32)
    hipLaunchKernelGGL(mfma32_kernel, dim3(grid), dim3(512), 0, s, (const uint4*)src, iters, out);
  else
    hipLaunchKernelGGL(mfma16_kernel, dim3(grid), dim3(512), 0, s, (const uint4*)src, iters, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
