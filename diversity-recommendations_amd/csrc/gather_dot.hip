// Embedding-row gather + row-wise dot: MatrixFactorization.forward
// (reference divrec/models/matrix_factorization.py:26-28) and its backward into
// dense embedding gradients (nn.Embedding sparse=False, :16-17).
//
// HBM-bound. A pair's two rows are read by a group of G lanes, 16 B per lane
// (G = the row's 16-B chunks rounded up to a power of two: d=128 fp32 -> 32
// lanes, bf16 -> 16), so every wave-instruction reads whole contiguous row
// segments. Each group walks a CONTIGUOUS span of pairs with UNR pairs in
// flight, and a row equal to the previous pair's row of the same table is
// taken from that pair's registers instead of being read again: the
// reference's own call patterns are runs — RankingDataset yields
// (torch.full((n,), u), candidates) (base_datasets.py:165-171), PairWiseDataset
// the m x m product of one user with a positive repeated m times
// (base_datasets.py:94-107). Algorithmic bytes per pair: 2 * 8 (ids) + 4 (out)
// + d * elem for every row that differs from the previous pair's.
//
// Ids are range-checked against the table row counts (nn.Embedding raises
// IndexError): an invalid pair reads no row of its own, writes NaN (forward)
// or adds nothing (backward), and is counted in *err when err is not NULL.
// Row ids are int32 after the check (tables of up to 2^31 rows).
#include "common.h"

namespace {

using dr::kWave;

template <typename T>
struct Vec16;  // 16 bytes of T; dot(a, b) of two such raw chunks in fp32
template <>
struct Vec16<float> {
  static constexpr int N = 4;
  __device__ static float dot(const uint4& a, const uint4& b, float s) {
    s = fmaf(__uint_as_float(a.x), __uint_as_float(b.x), s);
    s = fmaf(__uint_as_float(a.y), __uint_as_float(b.y), s);
    s = fmaf(__uint_as_float(a.z), __uint_as_float(b.z), s);
    return fmaf(__uint_as_float(a.w), __uint_as_float(b.w), s);
  }
};
template <>
struct Vec16<__bf16> {
  static constexpr int N = 8;
  __device__ static float dot(const uint4& a, const uint4& b, float s) {
    const uint32_t wa[4] = {a.x, a.y, a.z, a.w}, wb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s = fmaf(dr::bf16_bits_to_f32(wa[i] & 0xffffu), dr::bf16_bits_to_f32(wb[i] & 0xffffu), s);
      s = fmaf(dr::bf16_bits_to_f32(wa[i] >> 16), dr::bf16_bits_to_f32(wb[i] >> 16), s);
    }
    return s;
  }
};

constexpr int kUnroll = 4;
constexpr int kGatherUW = 8;  // pairs in flight per lane group when a lane holds one 16-B row chunk
constexpr int kBlock = 256;

__device__ __forceinline__ bool in_rows(int64_t r, int64_t n) { return r >= 0 && r < n; }

// G lanes per pair; lane gl covers 16-B chunks gl, gl + G, ... (CH of them)
// of the row's `chunks`. The pairs are cut into blocks of G consecutive
// pairs, dealt to the groups cyclically (neighbouring groups stream
// neighbouring rows of a sequential pattern: contiguous per-group spans put
// the groups' concurrent reads a power-of-two stride apart, onto the same HBM
// channels, and measured 20 % slower there); UNR pairs in flight:
//   * lane gl loads (and range-checks) the ids of pair base + gl: two
//     coalesced loads per G pairs instead of one broadcast load per pair and
//     id; they reach the group by ds_bpermute;
//   * a row equal to the previous pair's row of the same table is taken from
//     that pair's registers (runs: the reference's call patterns);
//   * the UNR partial dot products of a step are reduced over the group by
//     log2(UNR) transpose-halving exchanges and log2(G / UNR) butterfly steps
//     (UNR - 1 + log2(G / UNR) shuffles per UNR pairs instead of log2(G) per
//     pair), after which lanes gl = j * G / UNR hold pair j's sum and store it.
//   UNR = 8 pairs in flight per group when a lane holds one 16-B chunk of a
//   row, else 4 (registers).
template <typename T, int G, int CH, bool MASK, int UNR>
__global__ __launch_bounds__(kBlock) void gather_dot_runs(
    const T* __restrict__ U, int64_t nu, const T* __restrict__ I, int64_t ni, int64_t d,
    int chunks, const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    float* __restrict__ out, int32_t* __restrict__ err) {
  constexpr int NV = Vec16<T>::N;
  static_assert(G % UNR == 0 && (UNR & (UNR - 1)) == 0, "UNR pairs per step, a power of two <= G");
  constexpr int Q = G / UNR;  // lanes per pair after the halving steps
  const int lane = dr::lane_id();
  const int gl = lane % G;
  const int gbase = lane - gl;  // first lane of this group in the wave
  const int jj = gl / Q;        // the pair of a step this lane ends up holding
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / G);
  const int64_t p_end = n;
  uint4 uv[UNR][CH], iv[UNR][CH];  // raw 16-B row chunks (4 registers each)
  int cu = -2, ci = -2;  // ids (-1 = invalid) of the rows in uv / iv[UNR - 1]
  int bad = 0;
  auto load_row = [&](const T* tab, int r, uint4 (&v)[CH]) {
    const T* row = tab + (int64_t)(r < 0 ? 0 : r) * d;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = c * G + gl;
      if (!MASK || ch < chunks)  // MASK: the row has fewer than G * CH chunks
        v[c] = *reinterpret_cast<const uint4*>(row + ch * NV);
      else
        v[c] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto copy_row = [&](uint4 (&dst)[CH], const uint4 (&src)[CH]) {
#pragma unroll
    for (int c = 0; c < CH; ++c) dst[c] = src[c];
  };
  for (int64_t base = group * G; base < p_end; base += ngroups * G) {
    // ids of this lane's pair, range-checked: -1 = out of range (row 0 is
    // read, the pair's output is NaN); past the end: the last pair again
    const int64_t mp = base + gl < p_end ? base + gl : p_end - 1;
    const int64_t u64 = uid[mp], i64 = iid[mp];
    const int my_u = in_rows(u64, nu) ? (int)u64 : -1;
    const int my_i = in_rows(i64, ni) ? (int)i64 : -1;
#pragma unroll 1
    for (int j0 = 0; j0 < G; j0 += UNR) {
      int u[UNR], it[UNR];
#pragma unroll
      for (int j = 0; j < UNR; ++j) {
        u[j] = __shfl(my_u, gbase + j0 + j);
        it[j] = __shfl(my_i, gbase + j0 + j);
      }
#pragma unroll
      for (int j = 0; j < UNR; ++j) {
        const int pu = j ? u[j - 1] : cu, pi = j ? it[j - 1] : ci;
        if (u[j] != pu) load_row(U, u[j], uv[j]);
        else copy_row(uv[j], uv[j ? j - 1 : UNR - 1]);
        if (it[j] != pi) load_row(I, it[j], iv[j]);
        else copy_row(iv[j], iv[j ? j - 1 : UNR - 1]);
      }
      cu = u[UNR - 1];
      ci = it[UNR - 1];
      float sm[UNR];
#pragma unroll
      for (int j = 0; j < UNR; ++j) {
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c) sum = Vec16<T>::dot(uv[j][c], iv[j][c], sum);
        sm[j] = sum;
      }
      // halving steps: at partner distance w the lane keeps the half of its
      // values whose pair index bit matches its lane bit w, adding the
      // partner's copy of that half
#pragma unroll
      for (int v = UNR, w = G / 2; v > 1; v >>= 1, w >>= 1) {
        const bool up = (gl & w) != 0;
#pragma unroll
        for (int t = 0; t < v / 2; ++t) {
          const float send = up ? sm[t] : sm[t + v / 2];
          const float keep = up ? sm[t + v / 2] : sm[t];
          sm[t] = keep + __shfl_xor(send, w);
        }
      }
#pragma unroll
      for (int w = Q / 2; w >= 1; w >>= 1) sm[0] += __shfl_xor(sm[0], w);
      const int64_t p = base + j0 + jj;
      if (gl % Q == 0 && p < p_end) {
        const int su = dr::select_reg<UNR>(u, jj), si = dr::select_reg<UNR>(it, jj);
        const bool ok = su >= 0 && si >= 0;
        out[p] = ok ? sm[0] : __builtin_nanf("");
        bad += ok ? 0 : 1;
      }
    }
  }
  if (bad && err) atomicAdd(err, bad);
}

// Any d: one wave per pair, lanes stride the row.
template <typename T>
__global__ __launch_bounds__(kBlock) void gather_dot_generic(
    const T* __restrict__ U, int64_t nu, const T* __restrict__ I, int64_t ni, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    float* __restrict__ out, int32_t* __restrict__ err) {
  const int lane = dr::lane_id();
  const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int64_t nw = (int64_t)gridDim.x * kBlock / kWave;
  for (int64_t p = w; p < n; p += nw) {
    const int64_t u = uid[p], i = iid[p];
    if (!in_rows(u, nu) || !in_rows(i, ni)) {  // wave-uniform
      if (lane == 0) {
        out[p] = __builtin_nanf("");
        if (err) atomicAdd(err, 1);
      }
      continue;
    }
    const T* ur = U + u * d;
    const T* ir = I + i * d;
    float s = 0.f;
    for (int64_t e = lane; e < d; e += kWave) s = fmaf((float)ur[e], (float)ir[e], s);
    s = dr::wave_sum_f32(s);
    if (lane == 0) out[p] = s;
  }
}

// Backward with the BPR kernel's contiguous row layout: a group of 32 lanes
// owns a pair and lane l handles elements l, l+32, ..., so every load and
// every atomic wave-instruction covers two contiguous 128-B row segments (the
// shape at which global_atomic_add_f32 runs at full rate; 16-B-per-lane
// chunks scatter each atomic instruction over 16-B strides and measured 3.9x
// slower). EPL = elements per lane = ceil(d / 32), any d <= 512.
template <int EPL>
__global__ __launch_bounds__(kBlock) void gather_dot_bwd_rows(
    const float* __restrict__ U, int64_t nu, const float* __restrict__ I, int64_t ni, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ gout, float* __restrict__ gU, float* __restrict__ gI,
    int32_t* __restrict__ err) {
  const int gl = threadIdx.x & 31;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 5;
  const int64_t ngroups = (int64_t)gridDim.x * (kBlock / 32);
  int bad = 0;
  for (int64_t p = group; p < n; p += ngroups) {
    const int64_t u = uid[p], i = iid[p];
    if (!in_rows(u, nu) || !in_rows(i, ni)) {  // uniform in the 32-lane group
      bad += gl == 0 ? 1 : 0;
      continue;
    }
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
  if (bad && err) atomicAdd(err, bad);
}

__global__ __launch_bounds__(kBlock) void gather_dot_bwd_generic(
    const float* __restrict__ U, int64_t nu, const float* __restrict__ I, int64_t ni, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ iid, int64_t n,
    const float* __restrict__ gout, float* __restrict__ gU, float* __restrict__ gI,
    int32_t* __restrict__ err) {
  const int lane = dr::lane_id();
  const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int64_t nw = (int64_t)gridDim.x * kBlock / kWave;
  for (int64_t p = w; p < n; p += nw) {
    const int64_t u = uid[p], i = iid[p];
    if (!in_rows(u, nu) || !in_rows(i, ni)) {  // wave-uniform
      if (lane == 0 && err) atomicAdd(err, 1);
      continue;
    }
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
int launch_fwd(const T* U, int64_t nu, const T* I, int64_t ni, int64_t d, const int64_t* uid,
               const int64_t* iid, int64_t n, float* out, int32_t* err, hipStream_t s) {
  constexpr int NV = Vec16<T>::N;
  const int64_t chunks = d % NV == 0 ? d / NV : -1;  // 16-B chunks per row
  auto go = [&](auto kern, int G) {
    // blocks of G pairs dealt cyclically, up to 8 workgroups per CU
    const int grid = grid_for(dr::ceil_div(dr::ceil_div(n, G), kBlock / G), 1);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, U, nu, I, ni, d, (int)chunks, uid,
                       iid, n, out, err);
  };
  constexpr int UW = kGatherUW;  // pairs in flight per group (rows held raw: 4 registers per chunk)
#define DR_RUNS(GG, CC)                                                                       \
  (chunks == GG * CC                                                                           \
       ? go(gather_dot_runs<T, GG, CC, false, (GG >= UW && CC == 1) ? UW : 4>, GG)             \
       : go(gather_dot_runs<T, GG, CC, true, (GG >= UW && CC == 1) ? UW : 4>, GG))
  if (chunks > 0 && chunks <= 4) DR_RUNS(4, 1);
  else if (chunks > 0 && chunks <= 8) DR_RUNS(8, 1);
  else if (chunks > 0 && chunks <= 16) DR_RUNS(16, 1);
  else if (chunks > 0 && chunks <= 32) DR_RUNS(32, 1);
  else if (chunks > 0 && chunks <= 64) DR_RUNS(64, 1);
  else if (chunks > 0 && chunks <= 128) DR_RUNS(64, 2);
#undef DR_RUNS
  else {
    const int grid = grid_for(n, kBlock / kWave);
    hipLaunchKernelGGL(gather_dot_generic<T>, dim3(grid), dim3(kBlock), 0, s, U, nu, I, ni, d,
                       uid, iid, n, out, err);
  }
  return DR_OK;
}

}  // namespace

extern "C" int dr_gather_dot(const void* user_table, int64_t n_user_rows, const void* item_table,
                             int64_t n_item_rows, int dtype, int64_t d, const int64_t* user_id,
                             const int64_t* item_id, int64_t n, float* out, int32_t* err,
                             dr_stream_t stream) {
  DR_CHECK_ARG(d > 0, "d must be positive");
  DR_CHECK_ARG(n >= 0 && n_user_rows >= 0 && n_item_rows >= 0, "sizes must be >= 0");
  DR_CHECK_ARG(n_user_rows < 0x7fffffffLL && n_item_rows < 0x7fffffffLL,
               "tables must have fewer than 2^31 rows");
  if (n == 0) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && item_id && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DR_F32) {
    launch_fwd((const float*)user_table, n_user_rows, (const float*)item_table, n_item_rows, d,
               user_id, item_id, n, out, err, s);
  } else if (dtype == DR_BF16) {
    launch_fwd((const __bf16*)user_table, n_user_rows, (const __bf16*)item_table, n_item_rows, d,
               user_id, item_id, n, out, err, s);
  } else {
    dr::set_error("dr_gather_dot: dtype must be DR_F32 or DR_BF16");
    return DR_EUNSUPPORTED;
  }
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_gather_dot_backward(const float* user_table, int64_t n_user_rows,
                                      const float* item_table, int64_t n_item_rows, int64_t d,
                                      const int64_t* user_id, const int64_t* item_id, int64_t n,
                                      const float* grad_out, float* grad_user, float* grad_item,
                                      int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(d > 0, "d must be positive");
  DR_CHECK_ARG(n >= 0 && n_user_rows >= 0 && n_item_rows >= 0, "sizes must be >= 0");
  if (n == 0 || (!grad_user && !grad_item)) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && item_id && grad_out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (d <= 512) {
    const int grid = grid_for(n, kBlock / 32);
#define DR_BWD(EE)                                                                          \
  hipLaunchKernelGGL(gather_dot_bwd_rows<EE>, dim3(grid), dim3(kBlock), 0, s, user_table,   \
                     n_user_rows, item_table, n_item_rows, d, user_id, item_id, n, grad_out, \
                     grad_user, grad_item, err)
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
  } else {
    const int grid = grid_for(n, kBlock / kWave);
    hipLaunchKernelGGL(gather_dot_bwd_generic, dim3(grid), dim3(kBlock), 0, s, user_table,
                       n_user_rows, item_table, n_item_rows, d, user_id, item_id, n, grad_out,
                       grad_user, grad_item, err);
  }
  DR_CHECK_LAUNCH();
  return DR_OK;
}
