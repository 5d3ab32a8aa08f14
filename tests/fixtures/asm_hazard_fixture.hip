// Planted inline-asm hazards for tests/test_asm_audit.py (never built into
// the library): tools/asm_audit.py must flag both kernels marked "bad" and
// pass the "good" ones.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ u32x4 ds_read(uint32_t a) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

// BAD: the fragment is read (copied into arithmetic) before the wait that
// retires its ds_read: the result is the register's stale contents.
extern "C" __global__ void planted_bad_inflight(float* out) {
  __shared__ u32x4 s[64];
  s[threadIdx.x] = u32x4{threadIdx.x, 1u, 2u, 3u};
  __syncthreads();
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) u32x4*)s) +
                     ((threadIdx.x ^ 1u) << 4);
  u32x4 v = ds_read(a);
  const float early = __uint_as_float(v.x) * 2.f;  // reads v while the load is in flight
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) : : "memory");
  out[threadIdx.x] = early + __uint_as_float(v.y);
}

// GOOD: the same, every use after the retiring wait.
extern "C" __global__ void planted_good_inflight(float* out) {
  __shared__ u32x4 s[64];
  s[threadIdx.x] = u32x4{threadIdx.x, 1u, 2u, 3u};
  __syncthreads();
  const uint32_t a = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) u32x4*)s) +
                     ((threadIdx.x ^ 1u) << 4);
  u32x4 v = ds_read(a);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) : : "memory");
  out[threadIdx.x] = __uint_as_float(v.x) * 2.f + __uint_as_float(v.y);
}

// BAD: inline asm reads an MFMA result with no wait states in between (hipcc
// inserts them only in front of its own instructions).
extern "C" __global__ void planted_bad_mfma(const u32x4* a, const u32x4* b, float* out) {
  const f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
      __builtin_bit_cast(bf16x8, a[threadIdx.x]), __builtin_bit_cast(bf16x8, b[threadIdx.x]),
      f32x16{}, 0, 0, 0);
  float m;
  asm volatile("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(acc[0]), "v"(acc[1]));
  out[threadIdx.x] = m;
}

// GOOD: the MFMA result goes through a compiler-scheduled VALU op first.
extern "C" __global__ void planted_good_mfma(const u32x4* a, const u32x4* b, float* out) {
  const f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
      __builtin_bit_cast(bf16x8, a[threadIdx.x]), __builtin_bit_cast(bf16x8, b[threadIdx.x]),
      f32x16{}, 0, 0, 0);
  const float x = acc[0] + acc[1];
  float m;
  asm volatile("v_max_f32 %0, %1, %1" : "=v"(m) : "v"(x));
  out[threadIdx.x] = m;
}
