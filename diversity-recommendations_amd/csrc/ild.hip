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
#include "common.h"

namespace {

using dr::bf16x8;
using dr::f32x16;

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
  // the whole list fits in registers for d <= 128 (k <= 128 = 4 tiles)
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
