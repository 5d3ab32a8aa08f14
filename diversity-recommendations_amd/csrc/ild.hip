// Intra-list diversity: IntraListDiversityScore.recommendations_loss
// (reference divrec/losses/intra_list_diversity_score.py:20-42) with
// reduction 'none':  out[u] = (sum_{p<q} D[r[u,p], r[u,q]]) / (k*(k-1)).
//
// Three ways to supply D:
//   * dense matrix (small catalogs, bit-exact parity): fp32 D is accumulated
//     sequentially in itertools.combinations order in fp32, exactly as the
//     reference's Python sum() over 0-d tensors (:40-42); integer D is summed
//     exactly. One lane per user for float D (the order is the contract),
//     one wave per user for integer D.
//   * label equality D[i,j] = (label[i] == label[j]) — the matrix built by
//     IntraListBinaryUnfairnessScore.get_distance_matrix (:60-63) — counted
//     exactly on the fly; no I x I matrix.
//   * item embeddings (any catalog size): per user the k rows are gathered
//     into MFMA fragments and the k x k Gram matrix is formed tile by tile
//     with v_mfma_f32_32x32x16_bf16; cosine / dot / euclidean distances are
//     summed over the strict upper triangle. HBM-bound at k=10 (gather of
//     k*d*2 bytes per user), MFMA-light at k=100.
#include <type_traits>

#include "common.h"

namespace {

using dr::bf16x8;
using dr::f32x16;
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename R>
__device__ __forceinline__ int64_t rec_at(const R* recs, int64_t i) {
  return (int64_t)recs[i];
}

// Id range check of one list (include/divrec_hip.h): true when every id is in
// [0, n_items). Wave-wide (every lane gets the answer); the one-lane form
// below serves the one-lane-per-user kernel.
template <typename R>
__device__ __forceinline__ bool wave_list_ok(const R* r, int k, int64_t n_items) {
  bool bad = false;
  for (int p = dr::lane_id(); p < k; p += 64) {
    const int64_t v = rec_at(r, p);
    bad |= v < 0 || v >= n_items;
  }
  return __ballot(bad) == 0ull;
}
template <typename R>
__device__ __forceinline__ bool lane_list_ok(const R* r, int k, int64_t n_items) {
  bool bad = false;
  for (int p = 0; p < k; ++p) {
    const int64_t v = rec_at(r, p);
    bad |= v < 0 || v >= n_items;
  }
  return !bad;
}

// --------------------------------------------------------------- dense, float
template <typename R, typename T, typename ACC>
__global__ __launch_bounds__(256) void ild_dense_seq(const R* __restrict__ recs, int64_t n_users,
                                                     int k, const T* __restrict__ D,
                                                     int64_t n_items, float* __restrict__ out,
                                                     double* __restrict__ raw,
                                                     int32_t* __restrict__ err) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= n_users) return;
  const R* r = recs + u * k;
  if (!lane_list_ok(r, k, n_items)) {
    if (raw) raw[u] = __builtin_nan("");
    else out[u] = __builtin_nanf("");
    if (err) atomicAdd(err, 1);
    return;
  }
  ACC acc = 0;
  for (int p = 0; p < k; ++p) {
    const T* row = D + rec_at(r, p) * n_items;
    for (int q = p + 1; q < k; ++q) acc += row[rec_at(r, q)];
  }
  if (raw) raw[u] = (double)acc;  // the pair sum in D's precision (user_ild)
  else out[u] = (float)acc / (float)(k * (k - 1));
}

// --------------------------------------------------------------- dense, integer
template <typename R, typename T>
__global__ __launch_bounds__(256) void ild_dense_int(const R* __restrict__ recs, int64_t n_users,
                                                     int k, const T* __restrict__ D,
                                                     int64_t n_items, float* __restrict__ out,
                                                     double* __restrict__ raw,
                                                     int32_t* __restrict__ err) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      if (raw) raw[u] = __builtin_nan("");
      else out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  long long acc = 0;
  for (int p = 0; p < k; ++p) {
    const T* row = D + rec_at(r, p) * n_items;
    for (int q = p + 1 + lane; q < k; q += 64) acc += (long long)row[rec_at(r, q)];
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
  if (lane == 0) {
    if (raw) raw[u] = (double)acc;  // exact while |sum| < 2^53
    else out[u] = (float)acc / (float)(k * (k - 1));
  }
}

// --------------------------------------------------------------- labels
constexpr int kLabelMaxK = 1024;
template <typename R>
__global__ __launch_bounds__(256) void ild_labels_kernel(const R* __restrict__ recs,
                                                         int64_t n_users, int k,
                                                         const int64_t* __restrict__ labels,
                                                         int64_t n_items, float* __restrict__ out,
                                                         int32_t* __restrict__ err) {
  __shared__ int64_t s_lab[4][kLabelMaxK];
  const int lane = dr::lane_id();
  const int wave = threadIdx.x >> 6;
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform; no block barrier below
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  int64_t* lab = s_lab[wave];
  for (int p = lane; p < k; p += 64) lab[p] = labels[rec_at(r, p)];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  long long cnt = 0;
  for (int p = lane; p < k; p += 64) {
    const int64_t lp = lab[p];
    for (int q = p + 1; q < k; ++q) cnt += (lab[q] == lp);
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) cnt += __shfl_xor(cnt, m);
  if (lane == 0) out[u] = (float)cnt / (float)(k * (k - 1));
}

// Lists longer than the LDS staging area (the reference's user_ild takes any
// length, intra_list_diversity_score.py:36-42): the same exact count with the
// labels read through the cache; one wave per user.
template <typename R>
__global__ __launch_bounds__(256) void ild_labels_long_kernel(const R* __restrict__ recs,
                                                              int64_t n_users, int k,
                                                              const int64_t* __restrict__ labels,
                                                              int64_t n_items,
                                                              float* __restrict__ out,
                                                              int32_t* __restrict__ err) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  long long cnt = 0;
  for (int p = lane; p < k; p += 64) {
    const int64_t lp = labels[rec_at(r, p)];
    for (int q = p + 1; q < k; ++q) cnt += (labels[rec_at(r, q)] == lp);
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) cnt += __shfl_xor(cnt, m);
  if (lane == 0) out[u] = (float)cnt / (float)((long long)k * (k - 1));  // as the short kernel
}

// --------------------------------------------------------------- embeddings
// One wave per user. Tile t holds rows [32t, 32t+32) of the user's list as
// MFMA fragments: lane l -> row (l & 31), k-slice 8*(l >> 5) + 16*s. The same
// fragment serves as A (rows) and B (columns) operand of X * X^T.
template <int D>
__device__ __forceinline__ void load_tile(const __bf16* __restrict__ E, const int64_t* rows,
                                          int t, int k, bf16x8 (&f)[D / 16]) {
  const int lane = dr::lane_id();
  const int p = 32 * t + (lane & 31);
  const int64_t row = rows[p < k ? p : 0];
  const uint4* src = reinterpret_cast<const uint4*>(E + row * D + 8 * (lane >> 5));
#pragma unroll
  for (int s = 0; s < D / 16; ++s) f[s] = __builtin_bit_cast(bf16x8, src[2 * s]);
}

template <int D>
__device__ __forceinline__ f32x16 gram_tile(const bf16x8 (&x)[D / 16], const bf16x8 (&y)[D / 16]) {
  f32x16 acc = f32x16{};
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[s], y[s], acc, 0, 0, 0);
  return acc;
}

// Same, but the zero accumulator is threaded through an empty asm that reads
// `after`: the tile's MFMAs cannot be hoisted above the work that produced
// `after`, so only one tile's accumulators are live at a time (hipcc otherwise
// hoists all ten Gram tiles of a 128-row list: 400+ registers, one wave/SIMD).
template <int D>
__device__ __forceinline__ f32x16 gram_tile_after(const bf16x8 (&x)[D / 16],
                                                  const bf16x8 (&y)[D / 16], float after) {
  f32x16 acc = f32x16{};
  asm volatile("" : "+v"(acc) : "v"(after));
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[s], y[s], acc, 0, 0, 0);
  return acc;
}

constexpr int kEmbMaxK = 128;

template <typename R, int D>
__global__ __launch_bounds__(256) void ild_embedding_kernel(const R* __restrict__ recs,
                                                            int64_t n_users, int k,
                                                            const __bf16* __restrict__ E,
                                                            int64_t n_items, int kind,
                                                            float* __restrict__ out,
                                                            int32_t* __restrict__ err) {
  __shared__ int64_t s_rows[4][kEmbMaxK];
  __shared__ float s_nsq[4][kEmbMaxK];
  const int lane = dr::lane_id();
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5, col = lane & 31;
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  int64_t* rows = s_rows[wave];
  float* nsq = s_nsq[wave];
  for (int p = lane; p < k; p += 64) rows[p] = rec_at(r, p);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nt = (k + 31) / 32;

  // Squared norms from the diagonal tiles: element (row == col) sits in the
  // lane with col = j and register r = (j & 3) + 4 * (j >> 3) when (j >> 2) & 1 == h.
  for (int t = 0; t < nt; ++t) {
    bf16x8 x[D / 16];
    load_tile<D>(E, rows, t, k, x);
    const f32x16 g = gram_tile<D>(x, x);
    const int ri = (col & 3) + 4 * (col >> 3);
    float v = g[0];
#pragma unroll
    for (int q = 1; q < 16; ++q) v = (ri == q) ? g[q] : v;
    if (((col >> 2) & 1) == h) nsq[32 * t + col] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  float sum = 0.f;
  for (int ti = 0; ti < nt; ++ti) {
    bf16x8 x[D / 16];
    load_tile<D>(E, rows, ti, k, x);
    for (int tj = ti; tj < nt; ++tj) {
      bf16x8 y[D / 16];
      load_tile<D>(E, rows, tj, k, y);
      const f32x16 g = gram_tile<D>(x, y);  // g[r] = <e_i, e_j>, i = row, j = col
      const int j = 32 * tj + col;
      const float nj = j < k ? nsq[j] : 1.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (i < j && j < k) {
          const float ni = nsq[i];
          float dist;
          if (kind == DR_ILD_COSINE) dist = 1.f - g[q] / (sqrtf(ni) * sqrtf(nj));
          else if (kind == DR_ILD_DOT) dist = g[q];
          else dist = sqrtf(fmaxf(ni + nj - 2.f * g[q], 0.f));
          sum += dist;
        }
      }
    }
  }
  sum = dr::wave_sum_f32(sum);
  if (lane == 0) out[u] = sum / (float)(k * (k - 1));
}

// Long lists (k > 128, any width; the reference's user_ild takes any
// length): one wave per workgroup streams the list's row tiles from the
// cache; the per-row terms of all k rows sit in LDS (4 B each), every
// upper-triangle Gram tile is one MFMA pass over two gathered tiles, and the
// pair distances are summed in double (a k = 4096 list has 8.4M pairs).
constexpr int kEmbLongMaxK = 16384;

template <typename R, int D, int KIND>
__global__ __launch_bounds__(64) void ild_embedding_long(const R* __restrict__ recs,
                                                         int64_t n_users, int k,
                                                         const __bf16* __restrict__ E,
                                                         int64_t n_items,
                                                         float* __restrict__ out,
                                                         int32_t* __restrict__ err) {
  constexpr int KS = D / 16;
  // per row: 1/|e| (cosine) or |e|^2 (euclidean); sized by the launch to k
  // floats (none for dot products), so a list of 129 rows keeps the CU's LDS
  // for other workgroups
  extern __shared__ float s_w[];
  const int lane = dr::lane_id();
  const int h = lane >> 5, col = lane & 31;
  const int64_t u = blockIdx.x;
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  const int nt = (k + 31) / 32;
  auto load = [&](int t, bf16x8 (&f)[KS]) {
    const int p = 32 * t + col;
    const int64_t row = rec_at(r, p < k ? p : 0);
    const uint4* src = reinterpret_cast<const uint4*>(E + row * D + 8 * h);
#pragma unroll
    for (int s = 0; s < KS; ++s) f[s] = __builtin_bit_cast(bf16x8, src[2 * s]);
  };
  if constexpr (KIND != DR_ILD_DOT) {
    for (int t = 0; t < nt; ++t) {
      bf16x8 x[KS];
      load(t, x);
      const f32x16 g = gram_tile<D>(x, x);
      const int ri = (col & 3) + 4 * (col >> 3);
      float v = g[0];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = (ri == q) ? g[q] : v;
      if (KIND == DR_ILD_COSINE) v = 1.f / sqrtf(v);
      if (((col >> 2) & 1) == h && 32 * t + col < k) s_w[32 * t + col] = v;
    }
    __syncthreads();
  }
  double sum = 0.0;
  for (int ti = 0; ti < nt; ++ti) {
    bf16x8 x[KS];
    load(ti, x);
    float wi[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h;
      wi[q] = (KIND != DR_ILD_DOT && i < k) ? s_w[i] : 0.f;
    }
    for (int tj = ti; tj < nt; ++tj) {
      bf16x8 y[KS];
      load(tj, y);
      const f32x16 g = gram_tile<D>(x, y);  // g[q] = <e_i, e_j>, i = row, j = col
      const int j = 32 * tj + col;
      const bool jv = j < k;
      const float wj = (KIND != DR_ILD_DOT && jv) ? s_w[j] : 0.f;
      float part = 0.f;  // <= 16 terms in fp32, the tile sums in double
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h;
        const bool ok = jv && (ti < tj || i < j);
        float dist;
        if constexpr (KIND == DR_ILD_COSINE) dist = fmaf(-g[q], wi[q] * wj, 1.f);
        else if constexpr (KIND == DR_ILD_DOT) dist = g[q];
        else dist = sqrtf(fmaxf(wi[q] + wj - 2.f * g[q], 0.f));
        part += ok ? dist : 0.f;
      }
      sum += (double)part;
    }
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) sum += __shfl_xor(sum, m);
  if (lane == 0) out[u] = (float)(sum / ((double)k * (double)(k - 1)));
}

template <typename R, int D>
void launch_long(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni, int kind,
                 float* out, int32_t* err, hipStream_t s) {
  const dim3 grid((unsigned)n_users);
  const size_t lds = (size_t)k * sizeof(float);  // k <= kEmbLongMaxK: at most 64 KB
  if (kind == DR_ILD_COSINE)
    hipLaunchKernelGGL((ild_embedding_long<R, D, DR_ILD_COSINE>), grid, 64, lds, s, recs, n_users, k, E, ni, out, err);
  else if (kind == DR_ILD_DOT)
    hipLaunchKernelGGL((ild_embedding_long<R, D, DR_ILD_DOT>), grid, 64, 0, s, recs, n_users, k, E, ni, out, err);
  else
    hipLaunchKernelGGL((ild_embedding_long<R, D, DR_ILD_EUCLIDEAN>), grid, 64, lds, s, recs, n_users, k, E, ni, out, err);
}

// Register-resident variant for nt = NT row tiles: every row of the list is
// gathered into MFMA fragments up front (all loads in flight together), then
// the norms and the upper-triangle Gram tiles are formed from registers. The
// per-row terms (|e|^2, and 1/|e| for cosine) are computed once per row, so a
// pair costs one fma (cosine), nothing (dot) or one sqrt (euclidean); the
// pair mask is structural (off-diagonal tiles need only j < k). Fragments:
// NT * D/16 * 4 VGPRs (128 at NT=4, D=128).
template <typename R, int D, int NT, int KIND>
// Two waves per SIMD: with the Gram tiles serialised (gram_tile_after) even
// the 128-row list fits in 256 registers, so one wave's row gathers overlap
// the other's MFMAs (profiles/r01_ild_ab_*.json).
__global__ __launch_bounds__(256, 2) void ild_embedding_regs(const R* __restrict__ recs,
                                                          int64_t n_users, int k,
                                                          const __bf16* __restrict__ E,
                                                          int64_t n_items,
                                                          float* __restrict__ out,
                                                          int32_t* __restrict__ err) {
  constexpr int KS = D / 16;
  __shared__ float s_w[4][NT * 32];  // per row: 1/|e| (cosine) or |e|^2 (euclidean)
  const int lane = dr::lane_id();
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5, col = lane & 31;
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const R* r = recs + u * k;
  if (!wave_list_ok(r, k, n_items)) {  // wave-uniform
    if (lane == 0) {
      out[u] = __builtin_nanf("");
      if (err) atomicAdd(err, 1);
    }
    return;
  }
  float* w = s_w[wave];
  bf16x8 x[NT][KS];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int p = 32 * t + col;
    const int64_t row = rec_at(r, p < k ? p : 0);
    const uint4* src = reinterpret_cast<const uint4*>(E + row * D + 8 * h);
#pragma unroll
    for (int s = 0; s < KS; ++s) x[t][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
  }
  if constexpr (KIND != DR_ILD_DOT) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x16 g = gram_tile<D>(x[t], x[t]);
      const int ri = (col & 3) + 4 * (col >> 3);
      float v = g[0];
#pragma unroll
      for (int q = 1; q < 16; ++q) v = (ri == q) ? g[q] : v;
      if (KIND == DR_ILD_COSINE) v = 1.f / sqrtf(v);
      if (((col >> 2) & 1) == h) w[32 * t + col] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  float sum = 0.f;
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) {
    float wi[16];
    if constexpr (KIND != DR_ILD_DOT) {
#pragma unroll
      for (int q = 0; q < 16; ++q) wi[q] = w[32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h];
    }
#pragma unroll
    for (int tj = ti; tj < NT; ++tj) {
      f32x16 g;
      if constexpr (NT >= 3) g = gram_tile_after<D>(x[ti], x[tj], sum);  // registers are the limit
      else g = gram_tile<D>(x[ti], x[tj]);  // short lists: let the scheduler overlap tiles
      const int j = 32 * tj + col;
      const bool jv = j < k;
      const float wj = (KIND != DR_ILD_DOT && jv) ? w[j] : 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h;
        const bool ok = jv && (ti < tj || i < j);
        float dist;
        if constexpr (KIND == DR_ILD_COSINE) dist = fmaf(-g[q], wi[q] * wj, 1.f);
        else if constexpr (KIND == DR_ILD_DOT) dist = g[q];
        else dist = sqrtf(fmaxf(wi[q] + wj - 2.f * g[q], 0.f));
        sum += ok ? dist : 0.f;
      }
    }
  }
  sum = dr::wave_sum_f32(sum);
  if (lane == 0) out[u] = sum / (float)(k * (k - 1));
}

template <typename R, int D, int KIND>
void launch_regs_kind(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni,
                      float* out, int32_t* err, hipStream_t s, int grid) {
  switch ((k + 31) / 32) {
    case 1: hipLaunchKernelGGL((ild_embedding_regs<R, D, 1, KIND>), grid, 256, 0, s, recs, n_users, k, E, ni, out, err); break;
    case 2: hipLaunchKernelGGL((ild_embedding_regs<R, D, 2, KIND>), grid, 256, 0, s, recs, n_users, k, E, ni, out, err); break;
    case 3: hipLaunchKernelGGL((ild_embedding_regs<R, D, 3, KIND>), grid, 256, 0, s, recs, n_users, k, E, ni, out, err); break;
    default: hipLaunchKernelGGL((ild_embedding_regs<R, D, 4, KIND>), grid, 256, 0, s, recs, n_users, k, E, ni, out, err); break;
  }
}

template <typename R, int D>
void launch_regs(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni, int kind,
                 float* out, int32_t* err, hipStream_t s, int grid) {
  if (kind == DR_ILD_COSINE) launch_regs_kind<R, D, DR_ILD_COSINE>(recs, n_users, k, E, ni, out, err, s, grid);
  else if (kind == DR_ILD_DOT) launch_regs_kind<R, D, DR_ILD_DOT>(recs, n_users, k, E, ni, out, err, s, grid);
  else launch_regs_kind<R, D, DR_ILD_EUCLIDEAN>(recs, n_users, k, E, ni, out, err, s, grid);
}

// ------------------------------------------------------ embeddings, streamed
// k <= 128 at d in {32, 64, 128}: the ILD of the headline metric (config 4,
// and config 5 after MMR). The one-wave-per-user kernel above issues the id
// load, the range check and the row gather as dependent round trips with
// nothing else in flight, and its per-pair epilogue is ~2000 VALU per user
// (5.8 ms = 57 % of HBM for 1M users, k = 100, d = 128). Here a persistent
// grid of 4-wave workgroups (one wave per SIMD, up to 512 VGPRs) runs every
// wave as a pipeline over its own users u = w, w + W, ... (W = waves in the
// grid):
//   * a user's rows reach a per-wave LDS buffer by LDS-DMA
//     (global_load_lds_dwordx4: a 1-KB piece is 4 / 8 / 16 whole rows of
//     256 / 128 / 64 B) NB users ahead of the one being computed; the image
//     is XOR-swizzled through the source chunk like the score scan's, so the
//     A-fragment ds_read_b128s are conflict-free; its ids arrive the same
//     way (dword DMA) NB users before its rows;
//   * nothing else of the wave touches VMEM (the result store is counted
//     asm), so each wait is an exact s_waitcnt vmcnt(N) that leaves the next
//     users' pieces in flight;
//   * an iteration reads the user's fragments into registers, refills the
//     buffer with the next user's pieces at once, and forms the Gram tiles;
//     the epilogue is one FMA per Gram element (below).
// Row buffers per wave (NB) as many as fit the 160-KB LDS, at most 16:
// k = 100, d = 128 keeps one user per wave in flight (4 x 25 KB per CU),
// k = 10 nine.
#ifdef DR_ILD_DIAG
// per-wave s_memtime cycles of each phase (diag builds only): wait, LDS
// reads, issue + compute, tail, total, users
__device__ uint64_t g_ild_diag[8192][8];
#define ILD_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ILD_ADD(slot, t0) dg[slot] += __builtin_amdgcn_s_memtime() - (t0)
#else
#define ILD_T0(v) ((void)0)
#define ILD_ADD(slot, t0) ((void)0)
#endif
constexpr int kStreamWaves = 4;
constexpr int kStreamMinK = 40;  // shorter lists take the one-wave-per-user kernel
constexpr int kStreamMaxBufs = 16;
constexpr int kStreamLds = 163840;
constexpr int kStreamHead = kStreamWaves * (128 * 4 + kStreamMaxBufs * 4);  // per-row terms, bad flags

struct StreamShape {
  int ni;   // row pieces (1 KB) per user
  int nid;  // id DMA instructions (64 dwords) per user
  int nb;   // row buffers per wave
  __host__ __device__ uint32_t wave_bytes(int b) const {
    return (uint32_t)b * ni * 1024u + (uint32_t)(b + 1) * nid * 256u;
  }
};
inline StreamShape stream_shape(int k, int d, int rec_bytes) {
  StreamShape sh;
  const int rpi = 64 / (d / 8);
  sh.ni = (k + rpi - 1) / rpi;
  sh.nid = (k * (rec_bytes / 4) + 63) / 64;
  sh.nb = kStreamMaxBufs;
  // LDS, and the exact vmcnt wait of the pipeline (at most 63 younger ops)
  while (sh.nb > 1 && (kStreamHead + kStreamWaves * sh.wave_bytes(sh.nb) > (uint32_t)kStreamLds ||
                       1 + (sh.nb - 1) * (sh.ni + sh.nid + 1) > 63))
    --sh.nb;
  double v;
  if (dr::plan_knob(DR_KNOB_ILD_BUFS, &v) && (int)v < sh.nb) sh.nb = (int)v;  // A/B knob
  return sh;
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [LO, HI] (an immediate: binary
// search over the encodings, six scalar branches)
template <int LO, int HI>
__device__ __forceinline__ void wait_vm_exact(int n) {
  if constexpr (LO == HI) {
    asm volatile("s_waitcnt vmcnt(%c0)" : : "i"(LO) : "memory");
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) wait_vm_exact<LO, MID>(n);
    else wait_vm_exact<MID + 1, HI>(n);
  }
}

// Sum over the wave in VALU only (the __shfl_xor form is six dependent LDS
// round trips, ds_bpermute): quad and row rotations by DPP, then the 16- and
// 32-lane halves by v_permlane16/32_swap. Every lane gets the sum.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  auto dpp = [](float x, auto CTRL) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(CTRL)::value,
                                                      0xf, 0xf, false));
  };
  v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
  v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
  v += dpp(v, std::integral_constant<int, 0x124>{});  // row_ror:4
  v += dpp(v, std::integral_constant<int, 0x128>{});  // row_ror:8
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

template <typename R, int D, int NT, int KIND>
__global__ __launch_bounds__(kStreamWaves * 64, 1) void ild_embedding_stream(
    const R* __restrict__ recs, int64_t n_users, int k, const __bf16* __restrict__ E,
    int64_t n_items, float* __restrict__ out, int32_t* __restrict__ err, StreamShape sh) {
  constexpr int KS = D / 16;
  constexpr int CPR = D / 8;                               // 16-B chunks per row
  constexpr int RPI = 64 / CPR;                            // rows per 1-KB piece
  constexpr int RPB = (2 * D >= 256) ? 1 : 256 / (2 * D);  // rows per 256-B bank row
  constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  __shared__ __attribute__((aligned(16))) char smem[kStreamLds];
  const int lane = dr::lane_id();
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int h = lane >> 5, col = lane & 31, gq = lane / CPR;
  const int64_t gw = (int64_t)blockIdx.x * kStreamWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kStreamWaves;
  if (gw >= n_users) return;  // wave-uniform; the kernel has no workgroup barrier
  const int nmine = (int)((n_users - 1 - gw) / nw + 1);
  const int ni = sh.ni, nid = sh.nid, nb = sh.nb;
  const int ndw = k * (int)sizeof(R) / 4;  // id dwords per user
  const uint32_t buf_bytes = (uint32_t)ni * 1024u, ids_bytes = (uint32_t)nid * 256u;
  const uint32_t wave_off = kStreamHead + (uint32_t)wave * sh.wave_bytes(nb);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  float* w = reinterpret_cast<float*>(smem) + wave * 128;  // per-row terms of the current user
  int* badf = reinterpret_cast<int*>(smem + kStreamWaves * 512) + wave * kStreamMaxBufs;
  const char* Eb = reinterpret_cast<const char*>(E);
  // past the wave's last user the pipeline keeps issuing (that user again),
  // so every iteration issues the same VMEM count and the waits stay exact
  auto user_of = [&](int m) -> int64_t { return gw + (int64_t)(m < nmine ? m : nmine - 1) * nw; };
  auto buf_off = [&](int m) -> uint32_t { return wave_off + (uint32_t)(m % nb) * buf_bytes; };
  auto ids_off = [&](int m) -> uint32_t {
    return wave_off + (uint32_t)nb * buf_bytes + (uint32_t)(m % (nb + 1)) * ids_bytes;
  };
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  // the list of user m: nid dword DMAs (entries past the list repeat its last dword)
  auto issue_ids = [&](int m) {
    const char* src = reinterpret_cast<const char*>(recs + user_of(m) * k);
    const uint32_t dst = lds0 + ids_off(m);
    for (int j = 0; j < nid; ++j) {
      const int e = 64 * j + lane < ndw ? 64 * j + lane : ndw - 1;
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(dst + 256u * (uint32_t)j);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                   : : "v"(src + 4 * e), "s"(m0) : "memory", "m0");
    }
  };
  // The rows of user m (its list landed): piece j, lane l fills image row
  // r = j RPI + l / CPR, physical chunk l % CPR, with the logical chunk
  // (l % CPR) ^ swz(r); rows past the list repeat its last row. The list is
  // range-checked first: an out-of-range id reads row 0 and marks the user
  // bad (NaN, *err). The pieces' ids are read 8 at a time (one wait per
  // batch of LDS reads, not a dependent round trip per piece).
  auto issue_rows = [&](int m) {
    const R* ids = reinterpret_cast<const R*>(smem + ids_off(m));
    const int64_t v0 = (int64_t)ids[lane < k ? lane : k - 1];
    const int64_t v1 = (int64_t)ids[lane + 64 < k ? lane + 64 : k - 1];
    const bool bad = v0 < 0 || v0 >= n_items || v1 < 0 || v1 >= n_items;
    const bool anybad = __ballot(bad) != 0ull;
    if (lane == 0) badf[m % nb] = anybad ? 1 : 0;
    const uint32_t dst = lds0 + buf_off(m);
    for (int j0 = 0; j0 < ni; j0 += 8) {
      int64_t idv[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int r = (j0 + jj) * RPI + gq;
        idv[jj] = (int64_t)ids[r < k ? r : k - 1];
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = j0 + jj;
        if (j >= ni) break;
        const uint64_t id = (idv[jj] >= 0 && idv[jj] < n_items) ? (uint64_t)idv[jj] : 0ull;
        const int lc = (lane % CPR) ^ (((j * RPI + gq) / RPB) & SWM);
        const char* src = Eb + id * (uint64_t)(2 * D) + lc * 16;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(dst + 1024u * (uint32_t)j);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     : : "v"(src), "s"(m0) : "memory", "m0");
      }
    }
  };

  // per-lane constants of the Gram epilogue: register q of a 32x32 tile holds
  // row i(q) = (q & 3) + 8 (q >> 2) + 4 h of column col
  f2 onehot[8], upper[8];  // q == the diagonal's register; i(q) < col
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int q0 = 2 * q, q1 = 2 * q + 1;
    const int ri = (col & 3) + 4 * (col >> 3);
    onehot[q] = f2{ri == q0 ? 1.f : 0.f, ri == q1 ? 1.f : 0.f};
    upper[q] = f2{(q0 & 3) + 8 * (q0 >> 2) + 4 * h < col ? 1.f : 0.f,
                  (q1 & 3) + 8 * (q1 >> 2) + 4 * h < col ? 1.f : 0.f};
  }
  // prologue: the lists of users 0..nb-1, then (in the loop's issue order)
  // list(m + nb) + rows(m) for m < nb
  for (int m = 0; m < nb; ++m) issue_ids(m);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int m = 0; m < nb; ++m) {
    issue_ids(m + nb);
    issue_rows(m);
  }
  const int per = ni + nid + 1;  // VMEM ops of one iteration: a list, the rows, the result
  int nbad = 0;
#ifdef DR_ILD_DIAG
  uint64_t dg[8] = {};
  ILD_T0(t_all);
#endif
  for (int n = 0; n < nmine; ++n) {
    // rows(n) (issued in iteration n - nb, or prologue step n, after the list
    // of user n + nb) have landed; only younger ops may be pending
    const int vm = n < nb ? (nb - 1 - n) * (per - 1) + n * per : 1 + (nb - 1) * per;
    ILD_T0(t_w);
    wait_vm_exact<0, 63>(vm);
    ILD_ADD(0, t_w);
    ILD_T0(t_f);
    // one batch of LDS reads: the user's fragments, the next user's piece ids
    const char* img = smem + buf_off(n);
    bf16x8 x[NT][KS];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int rr = 32 * t + col < k ? 32 * t + col : k - 1;
      const char* row = img + rr * (2 * D);
      const int sw = (rr / RPB) & SWM;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        x[t][s] = *reinterpret_cast<const bf16x8*>(row + (((2 * s + h) ^ sw) << 4));
    }
    const bool bad = badf[n % nb] != 0;
    // the fragments are in registers before the buffer is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ILD_ADD(1, t_f);
    ILD_T0(t_c);
    issue_ids(n + 2 * nb);
    issue_rows(n + nb);
    // Diagonal Gram tiles first: |e_i|^2 of their rows (lane (col, h) with
    // h = (col >> 2) & 1 holds G[col][col] in register ri), reused for their
    // own pairs; off-diagonal tiles (ti < tj) as the epilogue reaches them.
    // (Issuing all tiles before the epilogue, and the next user's pieces
    // between them, measured no better: the wave issues in order, so neither
    // overlaps the pieces' issue stalls.)
    f32x16 gd[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) gd[t] = gram_tile<D>(x[t], x[t]);
    // per-row term (rows >= k: 0): cosine 1/|e|, dot 1, euclidean |e|^2
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // the diagonal element by a one-hot dot product (packed FMAs; a select
      // chain needs 16 lane masks in SGPRs, which spill)
      f2 dv = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q) dv = __builtin_elementwise_fma(onehot[q], f2{gd[t][2 * q], gd[t][2 * q + 1]}, dv);
      float v = dv.x + dv.y;
      if constexpr (KIND == DR_ILD_COSINE) v = __builtin_amdgcn_rsqf(v);  // <= 1 ulp
      else if constexpr (KIND == DR_ILD_DOT) v = 1.f;
      if (((col >> 2) & 1) == h) w[32 * t + col] = 32 * t + col < k ? v : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the 16 rows of a lane's accumulator: i = (q & 3) + 8 (q >> 2) + 4 h, so
    // rows 8m + 4h .. +3 are registers 4m .. 4m + 3 (one ds_read_b128 each)
    auto row_terms = [&](int t, float (&wi)[16]) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float4 v4 = *reinterpret_cast<const float4*>(w + 32 * t + 8 * m + 4 * h);
        wi[4 * m] = v4.x, wi[4 * m + 1] = v4.y, wi[4 * m + 2] = v4.z, wi[4 * m + 3] = v4.w;
      }
    };
    auto tile_of = [&](int ti, int tj) -> f32x16 {
      return ti == tj ? gd[ti] : gram_tile<D>(x[ti], x[tj]);
    };
    float sum = 0.f;
    if constexpr (KIND != DR_ILD_EUCLIDEAN) {
      // cosine: sum_{i<j} (1 - w_i w_j G_ij) = k(k-1)/2 - sum_j w_j sum_{i<j} w_i G_ij;
      // dot: sum_j w_j sum_{i<j} w_i G_ij with w = 1. A lane's part is one
      // FMA per Gram element: its column's weighted sum over its 16 rows,
      // the strict upper triangle of a diagonal tile by zeroed row weights
      // (rows >= k carry weight 0, as i and as j).
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
        float wi[16];
        row_terms(ti, wi);
#pragma unroll
        for (int tj = ti; tj < NT; ++tj) {
          const f32x16 g = tile_of(ti, tj);
          const float wj = w[32 * tj + col];
          f2 c = {0.f, 0.f};  // packed FMAs, two chains
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            f2 wq = {wi[2 * q], wi[2 * q + 1]};
            if (tj == ti) wq = wq * upper[q];  // i < j: 0/1 per lane
            c = __builtin_elementwise_fma(wq, f2{g[2 * q], g[2 * q + 1]}, c);
          }
          sum = fmaf(wj, c.x + c.y, sum);
        }
      }
      sum = wave_sum_dpp(sum);
      if constexpr (KIND == DR_ILD_COSINE) sum = (float)(k * (k - 1) / 2) - sum;
    } else {
      // |e_i - e_j| = sqrt(|e_i|^2 + |e_j|^2 - 2 G_ij): one sqrt per pair
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
        float wi[16];
        row_terms(ti, wi);
#pragma unroll
        for (int tj = ti; tj < NT; ++tj) {
          const f32x16 g = tile_of(ti, tj);
          const int j = 32 * tj + col;
          const bool jv = j < k;
          const float wj = w[j];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int i = 32 * ti + (q & 3) + 8 * (q >> 2) + 4 * h;
            const bool ok = jv && (ti < tj || i < j);
            const float dist = sqrtf(fmaxf(wi[q] + wj - 2.f * g[q], 0.f));
            sum += ok ? dist : 0.f;
          }
        }
      }
      sum = wave_sum_dpp(sum);
    }
    float res = sum / (float)(k * (k - 1));
#ifdef DR_ILD_DIAG
    asm volatile("" : "+v"(res));
#endif
    ILD_ADD(2, t_c);
    ILD_T0(t_t);
    if (bad) {
      res = __builtin_nanf("");
      ++nbad;
    }
    // w is rewritten by the next user's norms only after every lane read it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0)
      asm volatile("global_store_dword %0, %1, off" : : "v"(out + user_of(n)), "v"(res) : "memory");
    ILD_ADD(3, t_t);
  }
#ifdef DR_ILD_DIAG
  ILD_ADD(5, t_all);
  dg[6] = nmine;
  if (lane == 0 && gw < 8192)
    for (int i = 0; i < 8; ++i) g_ild_diag[gw][i] = dg[i];
#endif
#pragma clang diagnostic pop
  // no LDS-DMA may be outstanding when the wave ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nbad && err && lane == 0) atomicAdd(err, nbad);
}

template <typename R, int D, int KIND>
void launch_stream_kind(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni,
                        float* out, int32_t* err, hipStream_t s, const StreamShape& sh, int grid) {
  switch ((k + 31) / 32) {
    case 1: hipLaunchKernelGGL((ild_embedding_stream<R, D, 1, KIND>), grid, kStreamWaves * 64, 0, s, recs, n_users, k, E, ni, out, err, sh); break;
    case 2: hipLaunchKernelGGL((ild_embedding_stream<R, D, 2, KIND>), grid, kStreamWaves * 64, 0, s, recs, n_users, k, E, ni, out, err, sh); break;
    case 3: hipLaunchKernelGGL((ild_embedding_stream<R, D, 3, KIND>), grid, kStreamWaves * 64, 0, s, recs, n_users, k, E, ni, out, err, sh); break;
    default: hipLaunchKernelGGL((ild_embedding_stream<R, D, 4, KIND>), grid, kStreamWaves * 64, 0, s, recs, n_users, k, E, ni, out, err, sh); break;
  }
}

template <typename R, int D>
void launch_stream(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni, int kind,
                   float* out, int32_t* err, hipStream_t s) {
  const StreamShape sh = stream_shape(k, D, (int)sizeof(R));
  const int64_t need = dr::ceil_div(n_users, kStreamWaves);  // a wave per user at most
  const int cus = dr::device_cus();
  const int grid = (int)(need < cus ? need : cus);
  if (kind == DR_ILD_COSINE) launch_stream_kind<R, D, DR_ILD_COSINE>(recs, n_users, k, E, ni, out, err, s, sh, grid);
  else if (kind == DR_ILD_DOT) launch_stream_kind<R, D, DR_ILD_DOT>(recs, n_users, k, E, ni, out, err, s, sh, grid);
  else launch_stream_kind<R, D, DR_ILD_EUCLIDEAN>(recs, n_users, k, E, ni, out, err, s, sh, grid);
}

template <typename R>
int launch_embedding(const R* recs, int64_t n_users, int k, const __bf16* E, int64_t ni, int d,
                     int kind, float* out, int32_t* err, hipStream_t s) {
  const int grid = (int)dr::ceil_div(n_users, 4);
  if (k > kEmbMaxK) {  // long lists: the streaming kernel, any width
    switch (d) {
      case 32: launch_long<R, 32>(recs, n_users, k, E, ni, kind, out, err, s); return DR_OK;
      case 64: launch_long<R, 64>(recs, n_users, k, E, ni, kind, out, err, s); return DR_OK;
      case 128: launch_long<R, 128>(recs, n_users, k, E, ni, kind, out, err, s); return DR_OK;
      case 256: launch_long<R, 256>(recs, n_users, k, E, ni, kind, out, err, s); return DR_OK;
      default:
        dr::set_error("dr_ild_embedding: d must be one of 32, 64, 128, 256");
        return DR_EUNSUPPORTED;
    }
  }
  // the whole list fits in registers for d <= 128 (k <= 128 = 4 tiles).
  // Streamed where it wins (profiles/r06/ild_ab/, 1M users over 10M rows):
  // d = 128 cosine / dot lists longer than kStreamMinK (k = 100 4.4-4.8
  // against 4.7-5.7 ms, k = 64 2.78 against 2.82-3.04). One wave per user
  // elsewhere: short lists, where the stream's per-user pipeline overhead
  // dominates (k = 10 0.72 against 1.14-1.2 ms, k = 40 2.25-2.41 against
  // 2.32-2.44), d = 64 (2.82-2.96 against 3.07-3.54 ms: half the bytes per
  // user for the same pipeline), and euclidean (8.6 against 12.0 ms: the
  // per-pair sqrt on one wave per SIMD). DR_KNOB_ILD_STREAM forces either.
  double sv;
  const bool stream = dr::plan_knob(DR_KNOB_ILD_STREAM, &sv)
                          ? sv != 0.0
                          : d == 128 && kind != DR_ILD_EUCLIDEAN && k > kStreamMinK;
  if (stream && (d == 32 || d == 64 || d == 128)) {
    if (d == 32) launch_stream<R, 32>(recs, n_users, k, E, ni, kind, out, err, s);
    else if (d == 64) launch_stream<R, 64>(recs, n_users, k, E, ni, kind, out, err, s);
    else launch_stream<R, 128>(recs, n_users, k, E, ni, kind, out, err, s);
    return DR_OK;
  }
  if (d == 32 || d == 64 || d == 128) {
    if (d == 32) launch_regs<R, 32>(recs, n_users, k, E, ni, kind, out, err, s, grid);
    else if (d == 64) launch_regs<R, 64>(recs, n_users, k, E, ni, kind, out, err, s, grid);
    else launch_regs<R, 128>(recs, n_users, k, E, ni, kind, out, err, s, grid);
    return DR_OK;
  }
  switch (d) {
    case 256: hipLaunchKernelGGL((ild_embedding_kernel<R, 256>), grid, 256, 0, s, recs, n_users, k, E, ni, kind, out, err); break;
    default:
      dr::set_error("dr_ild_embedding: d must be one of 32, 64, 128, 256");
      return DR_EUNSUPPORTED;
  }
  return DR_OK;
}

template <typename R>
int launch_dense(const R* recs, int64_t n_users, int k, const void* D, int dd, int64_t n_items,
                 float* out, double* raw, int32_t* err, hipStream_t s) {
  switch (dd) {
    case DR_F32: {
      const int grid = (int)dr::ceil_div(n_users, 256);
      hipLaunchKernelGGL((ild_dense_seq<R, float, float>), grid, 256, 0, s, recs, n_users, k,
                         (const float*)D, n_items, out, raw, err);
      break;
    }
    case DR_F64: {
      const int grid = (int)dr::ceil_div(n_users, 256);
      hipLaunchKernelGGL((ild_dense_seq<R, double, double>), grid, 256, 0, s, recs, n_users, k,
                         (const double*)D, n_items, out, raw, err);
      break;
    }
    case DR_I32: {
      const int grid = (int)dr::ceil_div(n_users, 4);
      hipLaunchKernelGGL((ild_dense_int<R, int32_t>), grid, 256, 0, s, recs, n_users, k,
                         (const int32_t*)D, n_items, out, raw, err);
      break;
    }
    case DR_I64: {
      const int grid = (int)dr::ceil_div(n_users, 4);
      hipLaunchKernelGGL((ild_dense_int<R, int64_t>), grid, 256, 0, s, recs, n_users, k,
                         (const int64_t*)D, n_items, out, raw, err);
      break;
    }
    default:
      dr::set_error("dr_ild_dense: dist dtype must be DR_F32, DR_F64, DR_I32 or DR_I64");
      return DR_EUNSUPPORTED;
  }
  return DR_OK;
}

}  // namespace

extern "C" int dr_ild_dense(const void* recs, int rec_dtype, int64_t n_users, int k,
                            const void* dist, int dist_dtype, int64_t n_items, float* out,
                            int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(k >= 1, "k must be >= 1");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "rec_dtype must be DR_I32/DR_I64");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && dist && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  int rc = rec_dtype == DR_I32
               ? launch_dense((const int32_t*)recs, n_users, k, dist, dist_dtype, n_items, out,
                              nullptr, err, s)
               : launch_dense((const int64_t*)recs, n_users, k, dist, dist_dtype, n_items, out,
                              nullptr, err, s);
  if (rc != DR_OK) return rc;
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_ild_dense_pair_sum(const void* recs, int rec_dtype, int64_t n_users, int k,
                                     const void* dist, int dist_dtype, int64_t n_items,
                                     double* out, int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(k >= 1, "k must be >= 1");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "rec_dtype must be DR_I32/DR_I64");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && dist && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  int rc = rec_dtype == DR_I32
               ? launch_dense((const int32_t*)recs, n_users, k, dist, dist_dtype, n_items, nullptr,
                              out, err, s)
               : launch_dense((const int64_t*)recs, n_users, k, dist, dist_dtype, n_items, nullptr,
                              out, err, s);
  if (rc != DR_OK) return rc;
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_ild_labels(const void* recs, int rec_dtype, int64_t n_users, int k,
                             const int64_t* labels, int64_t n_items, float* out, int32_t* err,
                             dr_stream_t stream) {
  DR_CHECK_ARG(k >= 1, "k must be >= 1");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "rec_dtype must be DR_I32/DR_I64");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && labels && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)dr::ceil_div(n_users, 4);
#define DR_LAB(KERN, RT)                                                                   \
  hipLaunchKernelGGL((KERN<RT>), grid, 256, 0, s, (const RT*)recs, n_users, k, labels, \
                     n_items, out, err)
  if (k <= kLabelMaxK) {  // the list's labels staged in LDS
    if (rec_dtype == DR_I32) DR_LAB(ild_labels_kernel, int32_t);
    else DR_LAB(ild_labels_kernel, int64_t);
  } else {
    if (rec_dtype == DR_I32) DR_LAB(ild_labels_long_kernel, int32_t);
    else DR_LAB(ild_labels_long_kernel, int64_t);
  }
#undef DR_LAB
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_ild_embedding(const void* recs, int rec_dtype, int64_t n_users, int k,
                                const void* item_table, int64_t n_items, int d, int kind,
                                float* out, int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(k >= 1 && k <= kEmbLongMaxK, "k must be in [1, 16384]");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "rec_dtype must be DR_I32/DR_I64");
  DR_CHECK_ARG(kind == DR_ILD_COSINE || kind == DR_ILD_DOT || kind == DR_ILD_EUCLIDEAN,
               "unknown distance kind");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && item_table && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  int rc = rec_dtype == DR_I32
               ? launch_embedding((const int32_t*)recs, n_users, k, (const __bf16*)item_table,
                                  n_items, d, kind, out, err, s)
               : launch_embedding((const int64_t*)recs, n_users, k, (const __bf16*)item_table,
                                  n_items, d, kind, out, err, s);
  if (rc != DR_OK) return rc;
  DR_CHECK_LAUNCH();
  return DR_OK;
}

#ifdef DR_ILD_DIAG
// Diag builds only: copy the per-wave phase counters of the last streamed ILD
// launch (8192 waves x 8 u64) to host memory.
extern "C" int dr_ild_diag_read(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ild_diag), sizeof(g_ild_diag)) == hipSuccess ? 0 : -1;
}
#endif
