// Device-side pairwise sampling: the per-user sampling of PairWiseDataset.__iter__
// (reference divrec/datasets/base_datasets.py:70-107), SURVEY.md §8f rank 4.
//
// Per user u (in the given order):
//   positives = random.choices(unique positives of u, k=m)            (:74-79, :89)
//   negatives = random.choices(items - positives - frozen, k=m)       (:81-90)
//   yield the m x m Cartesian product, positive-major                 (:92-107)
// The reference draws from Python's Mersenne Twister; that stream is not
// reproducible here, so parity is distributional: every positive is one of
// u's positives (uniform over the unique list), every negative is uniform over
// the allowed set (rejection sampling against the sorted positive and frozen
// lists), and the output layout is the reference's. Draws come from a
// counter-based hash of (seed, user id, draw, try): deterministic for a
// given seed, independent of the launch geometry and of how users are chunked.
//
// Kernels: draw_kernel — one thread per (user, draw): m positive and m negative
// draws, int32 [n, m] each; expand_kernel — one thread per triple, int64 ids.
// Both are latency/HBM-bound byte work (a few binary searches per draw).
#include "common.h"

namespace {

constexpr int kBlock = 256;
constexpr int kMaxTries = 4096;  // rejection tries per negative draw

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t draw_bits(uint64_t seed, int64_t pos, int64_t draw,
                                              int64_t attempt) {
  uint64_t z = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(pos + 1));
  z = mix64(z ^ (0xd1b54a32d192ed03ull * (uint64_t)(draw + 1)));
  return mix64(z + 0x8cb92ba72f3d8dd7ull * (uint64_t)(attempt + 1));
}

__device__ __forceinline__ bool contains(const int32_t* __restrict__ list, int64_t n,
                                         int32_t item) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (list[mid] < item) lo = mid + 1; else hi = mid;
  }
  return lo < n && list[lo] == item;
}

// u = users[b]; threads [0, m) of a user draw positives, [m, 2m) negatives.
__global__ __launch_bounds__(kBlock) void draw_kernel(
    const int64_t* __restrict__ users, int64_t n, const int64_t* __restrict__ pos_rowptr,
    const int32_t* __restrict__ pos_items, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, int64_t n_items, int m, uint64_t seed,
    int32_t* __restrict__ pos_out, int32_t* __restrict__ neg_out, int32_t* __restrict__ err) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= n * 2 * m) return;
  const int64_t b = t / (2 * m);
  const int j = (int)(t - b * 2 * m);
  const int64_t u = users[b];
  const int64_t p0 = pos_rowptr[u], np = pos_rowptr[u + 1] - p0;
  if (j < m) {
    if (np == 0) {  // reference: random.choices([]) raises IndexError
      pos_out[b * m + j] = -1;
      atomicAdd(err, 1);
      return;
    }
    const uint64_t r = draw_bits(seed, u, j, 0);
    pos_out[b * m + j] = pos_items[p0 + (int64_t)(r % (uint64_t)np)];
    return;
  }
  const int32_t* ex = nullptr;
  int64_t nx = 0;
  if (excl_rowptr) {
    ex = excl_items + excl_rowptr[u];
    nx = excl_rowptr[u + 1] - excl_rowptr[u];
  }
  int32_t pick = -1;
  for (int a = 0; a < kMaxTries; ++a) {
    const int32_t c = (int32_t)(draw_bits(seed, u, j, a) % (uint64_t)n_items);
    if (!contains(pos_items + p0, np, c) && !(nx && contains(ex, nx, c))) {
      pick = c;
      break;
    }
  }
  if (pick < 0) atomicAdd(err, 1);  // allowed set empty (or vanishingly small)
  neg_out[b * m + (j - m)] = pick;
}

// triple e = (b * m + i) * m + jn: user b, positive i, negative jn (pos-major).
__global__ __launch_bounds__(kBlock) void expand_kernel(
    const int64_t* __restrict__ users, int64_t n, int m, const int32_t* __restrict__ pos_out,
    const int32_t* __restrict__ neg_out, int64_t* __restrict__ uid, int64_t* __restrict__ pid,
    int64_t* __restrict__ nid) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t mm = (int64_t)m * m;
  if (e >= n * mm) return;
  const int64_t b = e / mm;
  const int64_t r = e - b * mm;
  const int64_t i = r / m, jn = r - i * m;
  uid[e] = users[b];
  pid[e] = pos_out[b * m + i];
  nid[e] = neg_out[b * m + jn];
}

}  // namespace

extern "C" int dr_sample_pairwise(const int64_t* users, int64_t n_users,
                                  const int64_t* pos_rowptr, const int32_t* pos_items,
                                  const int64_t* excl_rowptr, const int32_t* excl_items,
                                  int64_t n_items, int m, uint64_t seed, int32_t* pos_out,
                                  int32_t* neg_out, int64_t* uid, int64_t* pid, int64_t* nid,
                                  int32_t* err_count, dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_items >= 1 && n_items < 0x7fffffffLL,
               "n_users >= 0 and 1 <= n_items < 2^31 required");
  DR_CHECK_ARG(m >= 1 && m <= 65536, "m (max_sampled) must be in [1, 65536]");
  DR_CHECK_ARG((excl_rowptr == nullptr) == (excl_items == nullptr),
               "excl_rowptr and excl_items must both be set or both be NULL");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(users && pos_rowptr && pos_items && pos_out && neg_out && err_count,
               "null pointer");
  DR_CHECK_ARG((uid == nullptr) == (pid == nullptr) && (pid == nullptr) == (nid == nullptr),
               "uid, pid and nid must all be set (expand) or all be NULL");
  hipStream_t s = (hipStream_t)stream;
  const int64_t draws = n_users * 2 * m;
  hipLaunchKernelGGL(draw_kernel, dim3((unsigned)dr::ceil_div(draws, kBlock)), dim3(kBlock), 0,
                     s, users, n_users, pos_rowptr, pos_items, excl_rowptr, excl_items, n_items,
                     m, seed, pos_out, neg_out, err_count);
  DR_CHECK_LAUNCH();
  if (uid) {
    const int64_t triples = n_users * (int64_t)m * m;
    hipLaunchKernelGGL(expand_kernel, dim3((unsigned)dr::ceil_div(triples, kBlock)),
                       dim3(kBlock), 0, s, users, n_users, m, pos_out, neg_out, uid, pid, nid);
    DR_CHECK_LAUNCH();
  }
  return DR_OK;
}
