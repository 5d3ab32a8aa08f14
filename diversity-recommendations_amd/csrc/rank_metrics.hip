// Accuracy metrics of a top-k list against each user's test interactions, one
// pass over the recommendations:
//   precision@k  = hits / k                        (metrics/precision_at_k.py:6-22)
//   recall@k     = hits / |positives|              (metrics/recall_at_k.py:6-22)
//   AP@k         = sum_p cumhits(p) / (p+1) / k    (metrics/average_precision_at_k.py:6-24,
//                  over ALL positions, the reference's own formula)
//   NDCG@k       = sum_p rel(p) / log2(p+2) / sum_p 1/log2(p+2)
//                                                  (metrics/normalized_discounted_cumulative_gain.py:6-23)
// The reference does one O(N) interaction mask per user; here positives come
// as a CSR (sorted item ids per user) and membership is a binary search. One
// wave per user; positions are split over lanes and the per-position terms are
// combined with a wave-wide inclusive scan of the hit flags.
#include "common.h"

namespace {

__device__ __forceinline__ bool contains_sorted(const int32_t* __restrict__ list, int n,
                                                int64_t item) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)list[mid] < item) lo = mid + 1; else hi = mid;
  }
  return lo < n && (int64_t)list[lo] == item;
}

template <typename R>
__global__ __launch_bounds__(256) void rank_metrics_kernel(
    const R* __restrict__ recs, int64_t n_users, int k, const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ items, float* __restrict__ prec, float* __restrict__ rec,
    float* __restrict__ ap, float* __restrict__ ndcg) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const int64_t p0 = rowptr[u];
  const int npos = (int)(rowptr[u + 1] - p0);
  const int32_t* pos = items + p0;
  int carry = 0;  // hits in earlier 64-position blocks
  float ap_sum = 0.f, dcg = 0.f, idcg = 0.f;
  for (int b0 = 0; b0 < k; b0 += 64) {
    const int p = b0 + lane;
    const bool in = p < k && contains_sorted(pos, npos, (int64_t)recs[u * k + p]);
    const uint64_t bal = __ballot(in);
    // inclusive prefix count of hits up to position p
    const int pre = carry + (int)__builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u)) +
                    (in ? 1 : 0);
    if (p < k) {
      ap_sum += (float)pre / (float)(p + 1);
      const float disc = log2f((float)(p + 2));
      dcg += (in ? 1.f : 0.f) / disc;
      idcg += 1.f / disc;
    }
    carry += __popcll(bal);
  }
  ap_sum = dr::wave_sum_f32(ap_sum);
  dcg = dr::wave_sum_f32(dcg);
  idcg = dr::wave_sum_f32(idcg);
  if (lane == 0) {
    if (prec) prec[u] = (float)carry / (float)k;
    if (rec) rec[u] = npos > 0 ? (float)((double)carry / (double)npos) : __builtin_nanf("");
    if (ap) ap[u] = ap_sum / (float)k;
    if (ndcg) ndcg[u] = dcg / idcg;
  }
}

}  // namespace

extern "C" int dr_rank_metrics(const void* recs, int rec_dtype, int64_t n_users, int k,
                               const int64_t* pos_rowptr, const int32_t* pos_items,
                               float* precision, float* recall, float* avg_precision,
                               float* ndcg, dr_stream_t stream) {
  DR_CHECK_ARG(k >= 1, "k must be >= 1");
  DR_CHECK_ARG(rec_dtype == DR_I32 || rec_dtype == DR_I64, "rec_dtype must be DR_I32/DR_I64");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(recs && pos_rowptr && pos_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)dr::ceil_div(n_users, 4);
  if (rec_dtype == DR_I32)
    hipLaunchKernelGGL((rank_metrics_kernel<int32_t>), grid, 256, 0, s, (const int32_t*)recs,
                       n_users, k, pos_rowptr, pos_items, precision, recall, avg_precision, ndcg);
  else
    hipLaunchKernelGGL((rank_metrics_kernel<int64_t>), grid, 256, 0, s, (const int64_t*)recs,
                       n_users, k, pos_rowptr, pos_items, precision, recall, avg_precision, ndcg);
  DR_CHECK_LAUNCH();
  return DR_OK;
}
