// Measurement probe for DESIGN.md §3.8: the fold pass of
// an MMR layout whose candidate rows are NOT resident in the register file.
// Such a layout frees registers for several users per CU, but every batch of
// every user must re-read the user's C candidate rows (C x d bf16 = 256 KB at
// C = 1000, d = 128) from L2 / MALL / HBM for its MFMA fold (picks x
// candidates). This kernel runs ONLY that traffic and MFMA work: per user,
// `batches` passes over its candidates, each pass one 32x32x16 bf16 MFMA
// chain per 32-candidate tile against 32 pick rows, the per-candidate max over
// the picks folded into an LDS max term. No selection, no argmax: a LOWER
// BOUND of the alternative's time. Grid = CUs x users_per_cu workgroups of
// 256 threads, each looping over users (persistent). Measurement tooling
// only: built into tools/probes/libmmr_fold.so, never linked into the product.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kD = 128;           // row width (bf16)
constexpr int kKS = kD / 16;      // k-steps per row
constexpr int kMaxC = 1024;

__global__ __launch_bounds__(256) void mmr_fold_kernel(const uint4* __restrict__ E, int64_t n_rows,
                                                       const int32_t* __restrict__ cand, int C,
                                                       int64_t n_users, int batches,
                                                       float* __restrict__ out) {
  __shared__ float s_max[kMaxC];
  __shared__ float s_red[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 31, h = lane >> 5;
  const int ntiles = (C + 31) / 32;
  for (int64_t u = blockIdx.x; u < n_users; u += gridDim.x) {
    for (int i = threadIdx.x; i < kMaxC; i += 256) s_max[i] = 0.f;
    __syncthreads();
    for (int b = 0; b < batches; ++b) {
      // this batch's 32 pick rows (A operand): candidates b*32 .. b*32+31 of the user
      uint4 af[kKS];
      {
        const int pc = (b * 32 + col) % C;
        const int64_t prow = cand[u * C + pc];
        const uint4* src = E + prow * (kD / 8) + h;
#pragma unroll
        for (int s = 0; s < kKS; ++s) af[s] = src[2 * s];
      }
      for (int t = wave; t < ntiles; t += 4) {
        const int c = t * 32 + col;
        const int64_t row = cand[u * C + (c < C ? c : C - 1)];
        const uint4* src = E + row * (kD / 8) + h;
        uint4 bf[kKS];
#pragma unroll
        for (int s = 0; s < kKS; ++s) bf[s] = src[2 * s];
        f32x16 acc = f32x16{};
#pragma unroll
        for (int s = 0; s < kKS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[s]),
                                                        __builtin_bit_cast(bf16x8, bf[s]), acc, 0, 0, 0);
        float m = acc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, acc[r]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
        m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        if (h == 0 && c < C) s_max[c] = fmaxf(s_max[c], m);
      }
      __syncthreads();  // a batch ends with the workgroup's barrier, as in the product kernel
    }
    float v = 0.f;
    for (int i = threadIdx.x; i < C; i += 256) v += s_max[i];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if (lane == 0) s_red[wave] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[u] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    __syncthreads();
  }
  (void)n_rows;
}

extern "C" int probe_mmr_fold(const void* E, int64_t n_rows, const int32_t* cand, int C,
                              int64_t n_users, int batches, int grid, float* out, void* stream) {
  if (C < 32 || C > kMaxC || batches < 1 || grid < 1) return -1;
  hipLaunchKernelGGL(mmr_fold_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)E, n_rows, cand, C, n_users, batches, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
