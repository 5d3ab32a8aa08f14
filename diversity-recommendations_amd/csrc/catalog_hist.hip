// Catalog histogram of a batch of recommendation lists,
// the counting step of the two catalog-diversity metrics:
//   counts[i]  = occurrences of item i over all lists — EntropyDiversityScore
//                takes them from torch.unique(recommendations, return_counts)
//                (reference divrec/metrics/entropy_diversity_score.py:19-26);
//   pos_sum[i] = sum of the 0-based positions of those occurrences — PRI's
//                avg_rank (popularity_rank_correlation_for_items.py:28-39)
//                builds the same sums in a Python dict, one item at a time.
// Integer atomics, so the sums are exact in any order. One lane per list
// entry; no-return atomics (the values are not needed by the kernel).
// HBM-bound: U*k id reads (4 or 8 B) plus two scattered atomics per entry.
#include "common.h"

namespace {

template <typename R>
__global__ __launch_bounds__(256) void catalog_hist_kernel(const R* __restrict__ recs, int64_t n,
                                                           int k, int64_t n_items,
                                                           int32_t* __restrict__ counts,
                                                           unsigned long long* __restrict__ pos_sum) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
    const int64_t item = (int64_t)recs[e];
    if (item < 0 || item >= n_items) continue;  // empty slots (-1) are not items
    atomicAdd(&counts[item], 1);
    if (pos_sum) atomicAdd(&pos_sum[item], (unsigned long long)(e % k));
  }
}

}  // namespace

extern "C" int dr_catalog_histogram(const void* recs, int rec_dtype, int64_t n_users, int k,
                                    int64_t n_items, int32_t* counts, uint64_t* pos_sum,
                                    dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && k >= 1 && n_items >= 1, "bad sizes");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "recs must be int32 or int64");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && counts, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = n_users * (int64_t)k;
  const int64_t blocks = dr::ceil_div(n, 256);
  const dim3 grid((unsigned)(blocks < 65536 ? blocks : 65536));
  auto* ps = reinterpret_cast<unsigned long long*>(pos_sum);
  if (rec_dtype == DR_I32)
    hipLaunchKernelGGL(catalog_hist_kernel<int32_t>, grid, dim3(256), 0, s,
                       (const int32_t*)recs, n, k, n_items, counts, ps);
  else
    hipLaunchKernelGGL(catalog_hist_kernel<int64_t>, grid, dim3(256), 0, s,
                       (const int64_t*)recs, n, k, n_items, counts, ps);
  DR_CHECK_LAUNCH();
  return DR_OK;
}
