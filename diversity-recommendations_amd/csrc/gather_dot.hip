// Embedding-row gather + row-wise dot: MatrixFactorization.forward
// (reference divrec/models/matrix_factorization.py:26-28) and its backward into
// dense embedding gradients (nn.Embedding sparse=False, :16-17).
//
// HBM-bound. A pair's two rows are read by a group of G lanes, 16 B per lane
// (G = row bytes / 16: d=128 fp32 -> 32 lanes, bf16 -> 16 lanes), so every
// wave-instruction reads whole contiguous row segments. Each group keeps UNR
// pairs' loads in flight before reducing, and the group reduces with
// butterfly shuffles. Algorithmic bytes per pair: 2*d*elem + 2*8 (ids) + 4 (out).
#include "common.h"

namespace {

using dr::kWave;

template <typename T>
struct Vec16;  // 16 bytes of T
template <>
struct Vec16<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float (&v)[4]) {
    float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
};
template <>
struct Vec16<__bf16> {
  static constexpr int N = 8;
  __device__ static void load(const __bf16* p, float (&v)[8]) {
    uint4 x = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = dr::bf16_bits_to_f32(w[i] & 0xffffu);
      v[2 * i + 1] = dr::bf16_bits_to_f32(w[i] >> 16);
    }
  }
};

#ifndef DR_BWD_ROWS
#define DR_BWD_ROWS 1  // backward: contiguous 32-lane row layout (0: 16-B chunks per lane)
#endif

constexpr int kUnroll = 4;
constexpr int kBlock = 256;

// G lanes per pair; each lane covers CH consecutive 16-B chunks of the row.
template <typename T, int G, int CH>
__global__ __launch_bounds__(kBlock) void gather_dot_vec(const T* __restrict__ U,
                                                         const T* __restrict__ I, int64_t d,
                                                         const int64_t* __restrict__ uid,
                                                         const int64_t* __restrict__ iid,
                                                         int64_t n, float* __restrict__ out) {
  constexpr int NV = Vec16<T>::N;
  const int gl = threadIdx.x % G;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  const int64_t ngroups = (int64_t)gridDim.x * kBlock / G;
  for (int64_t base = group; base < n; base += ngroups * kUnroll) {
    float acc[kUnroll];
    float uv[kUnroll][CH][NV], iv[kUnroll][CH][NV];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const int64_t p = base + j * ngroups;
      const int64_t pp = p < n ? p : (n - 1);
      const T* ur = U + uid[pp] * d;
      const T* ir = I + iid[pp] * d;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        Vec16<T>::load(ur + (c * G + gl) * NV, uv[j][c]);
        Vec16<T>::load(ir + (c * G + gl) * NV, iv[j][c]);
      }
    }
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int e = 0; e < NV; ++e) s = fmaf(uv[j][c][e], iv[j][c][e], s);
#pragma unroll
      for (int m = G / 2; m > 0; m >>= 1) s += __shfl_xor(s, m);
      acc[j] = s;
    }
    if (gl == 0) {
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        const int64_t p = base + j * ngroups;
        if (p < n) out[p] = acc[j];
      }
    }
  }
}

// Any d: one wave per pair, lanes stride the row.
template <typename T>
__global__ __launch_bounds__(kBlock) void gather_dot_generic(const T* __restrict__ U,
                                                             const T* __restrict__ I, int64_t d,
                                                             const int64_t* __restrict__ uid,
                                                             const int64_t* __restrict__ iid,
                                                             int64_t n, float* __restrict__ out) {
  const int lane = dr::lane_id();
  const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int64_t nw = (int64_t)gridDim.x * kBlock / kWave;
  for (int64_t p = w; p < n; p += nw) {
    const T* ur = U + uid[p] * d;
    const T* ir = I + iid[p] * d;
    float s = 0.f;
    for (int64_t e = lane; e < d; e += kWave) s = fmaf((float)ur[e], (float)ir[e], s);
    s = dr::wave_sum_f32(s);
    if (lane == 0) out[p] = s;
  }
}

template <int G, int CH>
__global__ __launch_bounds__(kBlock) void gather_dot_bwd_vec(
    const float* __restrict__ U, const float* __restrict__ I, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ gout, float* __restrict__ gU, float* __restrict__ gI) {
  const int gl = threadIdx.x % G;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  const int64_t ngroups = (int64_t)gridDim.x * kBlock / G;
  for (int64_t p = group; p < n; p += ngroups) {
    const int64_t u = uid[p], i = iid[p];
    const float g = gout[p];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t off = (int64_t)(c * G + gl) * 4;
      float uv[4], iv[4];
      Vec16<float>::load(U + u * d + off, uv);
      Vec16<float>::load(I + i * d + off, iv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (gU) atomicAdd(gU + u * d + off + e, g * iv[e]);
        if (gI) atomicAdd(gI + i * d + off + e, g * uv[e]);
      }
    }
  }
}

// Backward with the BPR kernel's contiguous row layout: a group of 32 lanes
// owns a pair and lane l handles elements l, l+32, ..., so every load and
// every atomic wave-instruction covers two contiguous 128-B row segments (the
// shape at which global_atomic_add_f32 runs at full rate; the 16-B-per-lane
// chunks of gather_dot_bwd_vec scatter each atomic instruction over 16-B
// strides). EPL = elements per lane = ceil(d / 32), any d <= 512.
template <int EPL>
__global__ __launch_bounds__(kBlock) void gather_dot_bwd_rows(
    const float* __restrict__ U, const float* __restrict__ I, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ gout, float* __restrict__ gU, float* __restrict__ gI) {
  const int gl = threadIdx.x & 31;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 5;
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / 32);
  for (int64_t p = group; p < n; p += ngroups) {
    const int64_t u = uid[p], i = iid[p];
    const float g = gout[p];
    const float* ur = U + u * d;
    const float* ir = I + i * d;
    float uv[EPL], iv[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int64_t c = gl + 32 * e;
      uv[e] = c < d ? ur[c] : 0.f;
      iv[e] = c < d ? ir[c] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int64_t c = gl + 32 * e;
      if (c < d) {
        if (gU) atomicAdd(gU + u * d + c, g * iv[e]);
        if (gI) atomicAdd(gI + i * d + c, g * uv[e]);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void gather_dot_bwd_generic(
    const float* __restrict__ U, const float* __restrict__ I, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ gout, float* __restrict__ gU, float* __restrict__ gI) {
  const int lane = dr::lane_id();
  const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int64_t nw = (int64_t)gridDim.x * kBlock / kWave;
  for (int64_t p = w; p < n; p += nw) {
    const int64_t u = uid[p], i = iid[p];
    const float g = gout[p];
    for (int64_t e = lane; e < d; e += kWave) {
      if (gU) atomicAdd(gU + u * d + e, g * I[i * d + e]);
      if (gI) atomicAdd(gI + i * d + e, g * U[u * d + e]);
    }
  }
}

int grid_for(int64_t items, int per_block) {
  int64_t g = dr::ceil_div(items, per_block);
  if (g > 256 * 8) g = 256 * 8;  // grid-stride the rest (Guideline 11)
  if (g < 1) g = 1;
  return (int)g;
}

template <typename T>
int launch_fwd(const T* U, const T* I, int64_t d, const int64_t* uid, const int64_t* iid,
               int64_t n, float* out, hipStream_t s) {
  constexpr int NV = Vec16<T>::N;
  const int64_t chunks = d % NV == 0 ? d / NV : -1;  // 16-B chunks per row
  auto go = [&](auto kern, int G) {
    const int grid = grid_for(dr::ceil_div(n, kUnroll), kBlock / G);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, U, I, d, uid, iid, n, out);
  };
  switch (chunks) {
    case 4: go(gather_dot_vec<T, 4, 1>, 4); break;
    case 8: go(gather_dot_vec<T, 8, 1>, 8); break;
    case 16: go(gather_dot_vec<T, 16, 1>, 16); break;
    case 32: go(gather_dot_vec<T, 32, 1>, 32); break;
    case 64: go(gather_dot_vec<T, 64, 1>, 64); break;
    case 128: go(gather_dot_vec<T, 64, 2>, 64); break;
    default: {
      const int grid = grid_for(n, kBlock / kWave);
      hipLaunchKernelGGL(gather_dot_generic<T>, dim3(grid), dim3(kBlock), 0, s, U, I, d, uid,
                         iid, n, out);
    }
  }
  return DR_OK;
}

}  // namespace

extern "C" int dr_gather_dot(const void* user_table, const void* item_table, int dtype,
                             int64_t d, const int64_t* user_id, const int64_t* item_id,
                             int64_t n, float* out, dr_stream_t stream) {
  DR_CHECK_ARG(d > 0, "d must be positive");
  DR_CHECK_ARG(n >= 0, "n must be >= 0");
  if (n == 0) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && item_id && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DR_F32) {
    launch_fwd((const float*)user_table, (const float*)item_table, d, user_id, item_id, n, out,
               s);
  } else if (dtype == DR_BF16) {
    launch_fwd((const __bf16*)user_table, (const __bf16*)item_table, d, user_id, item_id, n,
               out, s);
  } else {
    dr::set_error("dr_gather_dot: dtype must be DR_F32 or DR_BF16");
    return DR_EUNSUPPORTED;
  }
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_gather_dot_backward(const float* user_table, const float* item_table,
                                      int64_t d, const int64_t* user_id,
                                      const int64_t* item_id, int64_t n, const float* grad_out,
                                      float* grad_user, float* grad_item, dr_stream_t stream) {
  DR_CHECK_ARG(d > 0, "d must be positive");
  DR_CHECK_ARG(n >= 0, "n must be >= 0");
  if (n == 0 || (!grad_user && !grad_item)) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && item_id && grad_out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
#if DR_BWD_ROWS
  if (d <= 512) {
    const int grid = grid_for(n, kBlock / 32);
#define DR_BWD(EE)                                                                         \
  hipLaunchKernelGGL(gather_dot_bwd_rows<EE>, dim3(grid), dim3(kBlock), 0, s, user_table,  \
                     item_table, d, user_id, item_id, n, grad_out, grad_user, grad_item)
    switch ((int)dr::ceil_div(d, 32)) {
      case 1: DR_BWD(1); break;
      case 2: DR_BWD(2); break;
      case 3: DR_BWD(3); break;
      case 4: DR_BWD(4); break;
      case 5: case 6: DR_BWD(6); break;
      case 7: case 8: DR_BWD(8); break;
      case 9: case 10: case 11: case 12: DR_BWD(12); break;
      default: DR_BWD(16); break;
    }
#undef DR_BWD
    DR_CHECK_LAUNCH();
    return DR_OK;
  }
#endif
  const int64_t chunks = d % 4 == 0 ? d / 4 : -1;
  auto go = [&](auto kern, int G) {
    const int grid = grid_for(n, kBlock / G);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, user_table, item_table, d,
                       user_id, item_id, n, grad_out, grad_user, grad_item);
  };
  switch (chunks) {
    case 4: go(gather_dot_bwd_vec<4, 1>, 4); break;
    case 8: go(gather_dot_bwd_vec<8, 1>, 8); break;
    case 16: go(gather_dot_bwd_vec<16, 1>, 16); break;
    case 32: go(gather_dot_bwd_vec<32, 1>, 32); break;
    case 64: go(gather_dot_bwd_vec<64, 1>, 64); break;
    default: {
      const int grid = grid_for(n, kBlock / kWave);
      hipLaunchKernelGGL(gather_dot_bwd_generic, dim3(grid), dim3(kBlock), 0, s, user_table,
                         item_table, d, user_id, item_id, n, grad_out, grad_user, grad_item);
    }
  }
  DR_CHECK_LAUNCH();
  return DR_OK;
}
