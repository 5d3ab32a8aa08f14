// Full-catalog user x item scoring with a fused top-K: the MI355X form of
// get_model_recommendations (reference divrec/train/utils.py:53-77), whose
// per-user loop scores every RankingDataset candidate (base_datasets.py:136-171)
// with MatrixFactorization.forward (matrix_factorization.py:26-28) and keeps
// candidates[argsort(scores, descending=True)][:k].
//
// Kernels:
// score_scan_kernel (score_scan.h; instantiated per table dtype in
//   score_scan_bf16.hip and score_scan_f32.hip) — the streaming MFMA scan with
//   the fused threshold top-k into per-user candidate buffers.
// topk_threshold_kernel — one wave per user: ks-th best key of the sample scan.
// topk_finalize_kernel — one wave per user: gather the candidates of all
//   chunks, drop excluded items, bitonic sort, write the k best.
// topk_merge_kernel / topk_merge_stream_kernel — merge sorted partial lists
//   (the exchange step of the item-sharded multi-GPU top-k).
//
// Keys encode (score desc, item asc) as one 64-bit unsigned order, so the
// result is a deterministic total order and any item partition (chunks,
// GPUs) gives bit-identical top-k lists.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "score_scan.h"

namespace {

using namespace dr_topk;

// ------------------------------------------------------------------ per-user gather
// Where a user's candidate buffers live (Plan / TopkArgs): every user has its
// chunk-0 buffer at row = its position; a user of a split tail block has
// chunks - 1 more at rows n_users_pad + (j - 1) * tail_pad + (u - head_users).
constexpr int kMaxChunks = 16;  // = kMaxTailChunks (the plan's bound)

struct BufMap {
  int64_t n_users_pad;
  int64_t head_users;  // positions below this have one buffer
  int64_t tail_pad;    // users of the split tail blocks
  int chunks;          // buffers of a tail user
  __device__ int64_t row(int64_t u, int j) const {
    return j == 0 ? u : n_users_pad + (int64_t)(j - 1) * tail_pad + (u - head_users);
  }
  __device__ int n(int64_t u) const { return u < head_users ? 1 : chunks; }
};

BufMap buf_map(const Plan& p) {
  return BufMap{p.n_users_pad, p.head_users(), (p.n_ublocks - p.n_head) * p.users_per_wg,
                p.tail_chunks};
}

// One user's candidate keys of every buffer into registers (element e =
// lane*P + i), excluded items dropped; 0 = empty. The plan bounds the count
// by 64*P.
template <int P>
__device__ __forceinline__ void gather_candidates(const uint64_t* __restrict__ cand,
                                                  const int32_t* __restrict__ cnt, const BufMap m,
                                                  int cap, int64_t u,
                                                  const int64_t* __restrict__ excl_rowptr,
                                                  const int32_t* __restrict__ excl_items,
                                                  int64_t er, uint64_t (&key)[P]) {
  const int lane = dr::lane_id();
#pragma unroll
  for (int i = 0; i < P; ++i) key[i] = 0ull;
  const int nc = m.n(u);
  int off = 0;
  // chunk loop unrolled to its static bound so key[] stays in registers
#pragma unroll
  for (int c = 0; c < kMaxChunks; ++c) {
    if (c < nc) {
      const int64_t r = m.row(u, c);
      const int n = cnt[r];
      const uint64_t* src = cand + (size_t)r * cap;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int e = lane * P + i;
        if (e >= off && e < off + n) key[i] = src[e - off];
      }
      off += n;
    }
  }
  if (excl_rowptr) {  // er: the user's exclusion row
    const int64_t e0 = excl_rowptr[er], e1 = excl_rowptr[er + 1];
    const int n = (int)(e1 - e0);
    const int32_t* list = excl_items + e0;
    if (n > 0) {
      // lower_bound of every key's item by binary lifting: one runtime loop
      // over the (uniform) steps around the unrolled per-key work, so key[]
      // keeps static indices (P independent searches, each a loop of its
      // own, left key[] in scratch at P >= 16)
      int lo[P];
#pragma unroll
      for (int i = 0; i < P; ++i) lo[i] = 0;
      int step = 1;
      while (2 * step <= n) step *= 2;
      for (; step > 0; step >>= 1) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const int c = lo[i] + step;
          if (c <= n && list[c - 1] < (int32_t)dr::key_item(key[i])) lo[i] = c;
        }
      }
#pragma unroll
      for (int i = 0; i < P; ++i)
        if (key[i] != 0ull && lo[i] < n && list[lo[i]] == (int32_t)dr::key_item(key[i]))
          key[i] = 0ull;
    }
  }
}

// ------------------------------------------------------------------ finalize
// One wave per user of [u0, n_users): all its candidate buffers -> drop
// excluded items -> wave-wide register bitonic sort -> k best, decoded.
//   * Guessed-threshold scans (fail_cnt != NULL): a user left with fewer than
//     k keys may have lost items to a threshold guessed too high; it is
//     appended to the fail list (its user row and position) for the rescan.
//   * The rescan's finalize (pos_map != NULL): list entry u is written to the
//     caller's position pos_map[u]; the count comes from the device.
template <int P>
__global__ __launch_bounds__(256) void topk_finalize_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, const BufMap m, int cap,
    int64_t u0, int64_t n_users, int k, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, float* __restrict__ out_s,
    int32_t* __restrict__ out_i, const int64_t* __restrict__ pos_map,
    const int32_t* __restrict__ n_users_dev, const int64_t* __restrict__ user_ids,
    int32_t* __restrict__ fail_cnt, int64_t* __restrict__ fail_rows,
    int64_t* __restrict__ fail_pos, const float* __restrict__ fail_thr_src,
    float* __restrict__ fail_thr) {
  const int lane = dr::lane_id();
  const int64_t u = u0 + (((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6);
  if (n_users_dev) {
    const int64_t n = *n_users_dev;
    n_users = n < n_users ? n : n_users;
  }
  if (u >= n_users) return;  // wave-uniform
  const int64_t op = pos_map ? pos_map[u] : u;  // output and exclusion row
  uint64_t key[P];
  gather_candidates<P>(cand, cnt, m, cap, u, excl_rowptr, excl_items, op, key);
  dr::wave_sort_desc<P>(key);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    if (e < k) {
      const bool empty = key[i] == 0ull;
      out_s[op * k + e] = empty ? -INFINITY : dr::key_score(key[i]);
      out_i[op * k + e] = empty ? -1 : (int32_t)dr::key_item(key[i]);
    }
  }
  if (fail_cnt && lane == (k - 1) / P && dr::select_key<P>(key, (k - 1) % P) == 0ull) {
    const int32_t f = atomicAdd(fail_cnt, 1);
    fail_rows[f] = user_ids ? user_ids[u] : u;
    fail_pos[f] = op;
    if (fail_thr) fail_thr[f] = fail_thr_src[u];  // the user's second-tier threshold
  }
}

// Drop the keys of excluded items (sorted exclusion list of n items): binary
// lifting in one uniform loop over the steps, so key[] keeps static indices.
template <int P>
__device__ __forceinline__ void drop_excluded(uint64_t (&key)[P], const int32_t* __restrict__ list,
                                              int n) {
  if (n <= 0) return;
  int lo[P];
#pragma unroll
  for (int i = 0; i < P; ++i) lo[i] = 0;
  int step = 1;
  while (2 * step <= n) step *= 2;
  for (; step > 0; step >>= 1) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int c = lo[i] + step;
      if (c <= n && list[c - 1] < (int32_t)dr::key_item(key[i])) lo[i] = c;
    }
  }
#pragma unroll
  for (int i = 0; i < P; ++i)
    if (key[i] != 0ull && lo[i] < n && list[lo[i]] == (int32_t)dr::key_item(key[i])) key[i] = 0ull;
}

// ------------------------------------------------------------------ second-tier finalize
// Users of a second-tier rescan (dev_split chunk plan, device count): one
// wave per user streams the keys of all its chunk buffers, any number of
// them, through a 2048-key register sort that keeps the running best 1024
// (elements [0, 1024)); new keys enter elements [1024, 2048). Excluded items
// are dropped, the k best written to the caller's position pos_map[u]; a user
// left with fewer than k keys (its second-tier threshold was still too high)
// goes to the third-tier list.
struct DevSplitArgs {
  int upwg, grid, max_c;
  int64_t buf_blocks, n_items, stage_items;
};

__global__ __launch_bounds__(256) void topk_finalize_stream_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, const DevSplitArgs dsa,
    int cap, int64_t n_users_max, int k, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, float* __restrict__ out_s, int32_t* __restrict__ out_i,
    const int64_t* __restrict__ pos_map, const int32_t* __restrict__ n_users_dev,
    const int64_t* __restrict__ user_ids, int32_t* __restrict__ fail_cnt,
    int64_t* __restrict__ fail_rows, int64_t* __restrict__ fail_pos) {
  constexpr int P = 32;
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  int64_t n = *n_users_dev;
  n = n < n_users_max ? n : n_users_max;
  if (u >= n) return;  // wave-uniform
  const int64_t nb = (n + dsa.upwg - 1) / dsa.upwg;
  const DevSplit ds = dev_split_plan(nb, dsa.grid, dsa.max_c, dsa.buf_blocks, dsa.n_items,
                                     dsa.stage_items);
  const int64_t rows_per_chunk = nb * dsa.upwg;  // chunk j of user u: row j * rows_per_chunk + u
  int64_t total = 0;
  for (int j = 0; j < ds.chunks; ++j) total += cnt[j * rows_per_chunk + u];
  const int64_t op = pos_map[u];
  const int32_t* ex = nullptr;
  int exn = 0;
  if (excl_rowptr) {
    ex = excl_items + excl_rowptr[op];
    exn = (int)(excl_rowptr[op + 1] - excl_rowptr[op]);
  }
  // keys at flat positions [x0, x0 + 64 * P) of the concatenated buffers into
  // elements e = lane * P + i with lane >= lane0
  uint64_t key[P];
#pragma unroll
  for (int i = 0; i < P; ++i) key[i] = 0ull;
  auto load = [&](int64_t x0, int lane0) {
    if (lane < lane0) return;
    uint64_t nk[P];
#pragma unroll
    for (int i = 0; i < P; ++i) nk[i] = 0ull;
    int64_t off = 0;
    for (int j = 0; j < ds.chunks; ++j) {
      const int64_t r = j * rows_per_chunk + u;
      const int64_t nj = cnt[r];
      const uint64_t* src = cand + (size_t)r * cap;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int64_t x = x0 + (int64_t)(lane - lane0) * P + i;
        if (x >= off && x < off + nj) nk[i] = src[x - off];
      }
      off += nj;
    }
    drop_excluded<P>(nk, ex, exn);
#pragma unroll
    for (int i = 0; i < P; ++i) key[i] = nk[i];
  };
  load(0, 0);
  dr::wave_sort_desc<P>(key);
  for (int64_t next = 64 * P; next < total; next += 32 * P) {
    load(next, 32);
    dr::wave_sort_desc<P>(key);
  }
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    if (e < k) {
      const bool empty = key[i] == 0ull;
      out_s[op * k + e] = empty ? -INFINITY : dr::key_score(key[i]);
      out_i[op * k + e] = empty ? -1 : (int32_t)dr::key_item(key[i]);
    }
  }
  if (lane == (k - 1) / P && dr::select_key<P>(key, (k - 1) % P) == 0ull) {
    const int32_t f = atomicAdd(fail_cnt, 1);
    fail_rows[f] = user_ids[u];
    fail_pos[f] = op;
  }
}

// ------------------------------------------------------------------ threshold
// One wave per user position of [u0, u1) of the sample scan: the starting
// threshold of the main scan, strictly below the user's k-th best
// (non-excluded) sample score, so every score >= it passes the scan's
// `score > thr` test. -inf when the sample holds fewer than k candidates;
// +inf for padding positions (no user).
// thr[u] is taken at sample rank k1 (the first tier: the main scan's
// threshold), thr2[u] at rank k (the safe rank: a second-tier rescan's, for
// users whose first-tier guess fails); thr2 may be NULL.
template <int P>
__global__ __launch_bounds__(256) void topk_threshold_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, const BufMap m, int cap,
    int64_t u0, int64_t u1, int64_t n_users, int k, int k1, float* __restrict__ thr,
    float* __restrict__ thr2) {
  const int lane = dr::lane_id();
  const int64_t u = u0 + (((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6);
  if (u >= u1) return;  // wave-uniform
  if (u >= n_users) {
    if (lane == 0) {
      thr[u] = INFINITY;
      if (thr2) thr2[u] = INFINITY;
    }
    return;
  }
  uint64_t key[P];
  gather_candidates<P>(cand, cnt, m, cap, u, nullptr, nullptr, u, key);
  dr::wave_sort_desc<P>(key);
  auto below_key = [](uint64_t kk) {
    float t = -INFINITY;
    if (kk != 0ull) {
      const float s = dr::key_score(kk);
      const float below = s - fmaxf(fabsf(s) * 0x1p-20f, 0x1p-100f);
      t = below < s ? below : -INFINITY;  // NaN / inf scores: no pruning
    }
    return t;
  };
  if (lane == (k1 - 1) / P) thr[u] = below_key(dr::select_key<P>(key, (k1 - 1) % P));
  if (thr2 && lane == (k - 1) / P) thr2[u] = below_key(dr::select_key<P>(key, (k - 1) % P));
}

// The same thresholds from the dense tile maxima of a gmax == 2 sample scan
// (TopkArgs::tmax): one THREAD per user position of [0, n_pad) streams its
// column ([user / 32][tile][user % 32]: a wave reads two 128-B lines per tile,
// 8 tiles in flight) into a descending register array of its KS best maxima.
// A maximum above the lane's cut (its KS-th best at the last merge) is
// appended to the lane's LDS list (kDenseBuf slots); when some lane's list
// could overflow, every lane merges its list through a branch-free insertion
// network, new[j] = max(old[j], min(old[j-1], v)) (2 VALU per entry), and
// raises its cut. Appends cost ~3 VALU per tile; merges run ~KS (1 + ln(T /
// KS)) / kDenseBuf times per wave instead of once per tile (the wave's lanes
// insert at different tiles: a per-tile network ran on nearly every tile).
// Values at or below the cut cannot change the KS-th order statistic. The
// k-th best tile maximum equals the k-th best key of the compaction path's
// buffer (same maxima, same rank), so the thresholds are bit-identical to it.
// NaN maxima (a tile whose 32 scores are all NaN) rank nothing: a lower bound
// either way. KS >= k >= k1.
constexpr int kDenseMaxKs = 72;
constexpr int kDenseBuf = 24;
constexpr double kDenseMaxGiB = 16.0;

__device__ __forceinline__ float below_score(float s) {
  const float b = s - fmaxf(fabsf(s) * 0x1p-20f, 0x1p-100f);
  return b < s ? b : -INFINITY;  // -inf / +inf: no pruning
}

template <int KS>
__global__ __launch_bounds__(256) void topk_threshold_dense_kernel(
    const float* __restrict__ tmax, int64_t T, int64_t n_pad, int64_t n_users, int k, int k1,
    float* __restrict__ thr, float* __restrict__ thr2) {
  constexpr int kIn = 8;
  static_assert(kDenseBuf >= kIn, "a merge leaves room for one batch");
  __shared__ float lst[4][kDenseBuf][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (__builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * 256 + (threadIdx.x & ~63)) >= n_pad)))
    return;  // whole wave past the end
  const bool live = u < n_users;
  const float* src = tmax + (size_t)((live ? u : 0) >> 5) * (size_t)T * 32 + (u & 31);
  float best[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) best[j] = -INFINITY;
  float cut = -INFINITY;
  int n = 0;
  auto merge = [&]() {
    for (int i = 0; __builtin_amdgcn_ballot_w64(i < n) != 0ull; ++i) {
      const float v = i < n ? lst[wave][i][lane] : -INFINITY;
#pragma unroll
      for (int j = KS - 1; j > 0; --j) best[j] = fmaxf(best[j], fminf(best[j - 1], v));
      best[0] = fmaxf(best[0], v);
    }
    n = 0;
    cut = best[KS - 1];
  };
  auto add = [&](float v) {
    v = v == v ? v : -INFINITY;
    if (v > cut) lst[wave][n++][lane] = v;
  };
  int64_t t = 0;
  if (live) {
    for (; t + kIn <= T; t += kIn) {
      float v[kIn];
#pragma unroll
      for (int i = 0; i < kIn; ++i) v[i] = src[(size_t)(t + i) * 32];
#pragma unroll
      for (int i = 0; i < kIn; ++i) add(v[i]);
      if (__builtin_amdgcn_ballot_w64(n > kDenseBuf - kIn) != 0ull) merge();
    }
    for (; t < T; ++t) {
      add(src[(size_t)t * 32]);
      if (__builtin_amdgcn_ballot_w64(n >= kDenseBuf) != 0ull) merge();
    }
  }
  merge();
  if (u >= n_pad) return;
  if (!live) {
    thr[u] = INFINITY;
    if (thr2) thr2[u] = INFINITY;
    return;
  }
  float v1 = -INFINITY, v2 = -INFINITY;
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    if (j == k1 - 1) v1 = best[j];
    if (j == k - 1) v2 = best[j];
  }
  thr[u] = below_score(v1);
  if (thr2) thr2[u] = below_score(v2);
}

// Launch topk_threshold_dense_kernel for ranks (k1, k) over positions [0, n_pad).
bool launch_threshold_dense(const float* tmax, int64_t T, int64_t n_pad, int64_t n_users, int k,
                            int k1, float* thr, float* thr2, hipStream_t s) {
  const dim3 grid((unsigned)dr::ceil_div(n_pad, 256));
#define DR_TD(KK) \
  hipLaunchKernelGGL((topk_threshold_dense_kernel<KK>), grid, dim3(256), 0, s, tmax, T, n_pad, \
                     n_users, k, k1, thr, thr2)
  if (k <= 8) DR_TD(8);
  else if (k <= 16) DR_TD(16);
  else if (k <= 24) DR_TD(24);
  else if (k <= 32) DR_TD(32);
  else if (k <= 48) DR_TD(48);
  else if (k <= 72) DR_TD(72);
  else return false;
#undef DR_TD
  return true;
}

// ------------------------------------------------------------------ merge
// One wave per user: gather parts*k_in (score, item) pairs, sort, keep k_out.
template <int P>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ in_s,
                                                         const int32_t* __restrict__ in_i,
                                                         int parts, int64_t n_users, int k_in,
                                                         int k_out, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const int total = parts * k_in;
  uint64_t key[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    uint64_t kk = 0ull;
    if (e < total) {
      const int p = e / k_in, j = e % k_in;
      const size_t o = ((size_t)p * n_users + u) * k_in + j;
      const int32_t it = in_i[o];
      kk = it < 0 ? 0ull : dr::make_key(in_s[o], (uint32_t)it);
    }
    key[i] = kk;
  }
  dr::wave_sort_desc<P>(key);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    if (e < k_out) {
      const bool empty = key[i] == 0ull;
      out_s[u * k_out + e] = empty ? -INFINITY : dr::key_score(key[i]);
      out_i[u * k_out + e] = empty ? -1 : (int32_t)dr::key_item(key[i]);
    }
  }
}

int p_for(int total) {
  for (int p = 2; p <= 32; p <<= 1)
    if (total <= 64 * p) return p;
  return -1;
}

// ------------------------------------------------------------------ planning
// Plans take w, the row width in bf16 units (d for bf16 tables, 2d for fp32).
// Workgroup slots = CUs (one 512-thread workgroup per CU). DR_KNOB_SCAN_SLOTS
// overrides the count so that tests can reach the split-tail plans with
// small inputs; the result is identical for any plan.
int knob_int(int id, int fallback) {
  double v;
  return dr::plan_knob(id, &v) ? (int)v : fallback;
}

int device_cus() {
  const int slots = knob_int(DR_KNOB_SCAN_SLOTS, 0);
  if (slots > 0) return slots;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return cus > 0 ? cus : 256;
}

int64_t stage_items_for(int w, int cap) {
  return (int64_t)(stage_bytes_for(w, cap) / (kTileItems * w * 2)) * kTileItems;
}

// Smallest candidate capacity that leaves at least 32 keys of headroom above
// k + kSlack once a stage's worth of new keys (the margin) is reserved.
int cap_for(int w, int k) {
  for (int cap = 512; cap <= 2048; cap <<= 1)
    if (k + kSlack + 32 <= cap - (int)stage_items_for(w, cap)) return cap;
  return -1;
}

constexpr int kMaxTailChunks = 16;
constexpr bool kLongFlush = true;  // long lists flush at CAP - margin, not k + kSlack + kFlushGap
// Compaction slack and flush gap of the sample scan (ks <= ~70 keys per user).
constexpr int kSampleSlackDefault = 32;
constexpr int kSampleGapDefault = 96;
constexpr int kSampleGmax = 1;  // sample scans keep tile maxima (TopkArgs::gmax)
constexpr int kSampleSlack = kSampleSlackDefault;
constexpr int kSampleGap = kSampleGapDefault;
// The finalize of a split-tail user sorts every chunk's end-compacted keys
// (<= k + kSlack each) in one wave; at most 1024 of them keeps its sort at
// P = 16 (a 2048-key sort costs ~6x the 512-key one of a whole-catalog user).
constexpr int kMaxTailKeys = 1024;
constexpr bool kHeadKeep = true;  // long lists: whole-catalog units end compacted to 1024 keys

// Grid tail: U users make B = ceil(U / UPWG) user blocks for `slots`
// workgroups. Whole-catalog units run in ceil(B / slots) rounds, the last one
// with B % slots of the CUs busy (1M users at d = 128: 977 blocks, the 4th
// round on 209 of 256 CUs, 4.6 % of the scan idle). The plan keeps
// H = floor(B / slots) * slots "head" blocks whole and splits each of the T
// tail blocks into c catalog chunks, c chosen to minimise
// H / slots + ceil(T c / slots) / c (in whole-unit times); the chunks'
// buffers are merged by the finalize. With B < slots, H = 0 and the chunks
// fill the idle CUs instead.
//
// Measured (tools/variant_bench.py, 1M users, d = 128, k = 100, lists
// identical; profiles/r02_scan/ab_split_*.json): the split gains less than the
// idle-CU count suggests, because the chip clocks up while a last round runs on
// fewer CUs: +0.7 % at 1.25M items (an 8-way shard), and at 10M items +1.5 %
// together with the seeding it needs (a chunk scanned from -inf pays its own
// survivor stream), which alone costs 1.1 % there at the 1/32 sample stride
// and breaks even at 1/128. So a head/tail split is planned only for
// catalogs the guess can seed (seedable); a grid smaller than the CU count
// (H = 0) is chunked in any case, as before.
// Small catalogs (round 6): with at most kKeepAllItems rows the candidate
// buffer is sized to hold every row (CAP >= n_items, at most 2048: the finalize
// sort's bound), so the scan never compacts (TopkArgs::keep_all) and the
// finalize sorts all keys. Config 1's 943 users x 1682 rows ran ONE
// workgroup whose waves compacted each user's buffer several times from -inf.
// Measured against the compacting plan (lists identical,
// profiles/r06/keep_all/): 943 x 1682 d = 32 3.40 -> 1.55 ms, d = 64 2.07 ->
// 1.56, 10K x 2000 k = 100 4.18 -> 2.07; config 1's whole evaluation step
// 9.09 -> 5.23 ms. The 2048-key finalize per user grows with the users
// (60K x 2048 k = 10: 2.35 -> 3.30 ms, break-even near 20K), so the rule
// takes calls of at most kKeepAllUsers users. Such calls have few user
// blocks, so their catalog is split into stage-long chunks over more CUs (no
// chunk compacts; the finalize gathers every chunk's keys): 943 x 1682 d = 64
// 1.55 -> 0.86 ms, 10K x 2000 k = 100 2.05 -> 1.10, config 1's step 3.17 ->
// 2.43 ms. Unseeded main scans only (the caller says so: allow_keep_all).
constexpr bool kKeepAll = true;
constexpr int64_t kKeepAllItems = 2048;
constexpr int64_t kKeepAllUsers = 16384;

Plan make_plan(int64_t n_users, int64_t n_items, int w, int k, bool seedable,
               bool allow_keep_all = false) {
  Plan p{};
  p.cap = cap_for(w, k);
  if (kKeepAll && allow_keep_all && !seedable && p.cap > 0 && n_items <= kKeepAllItems &&
      n_users <= kKeepAllUsers && w <= 256) {  // CAP-2048 instances exist for w <= 256
    p.keep_all = 1;
    p.all_keys = n_items;
    while (p.cap < n_items) p.cap <<= 1;
  }
  p.users_per_wg = nut_for(w) * 32 * waves_for(w);
  p.n_ublocks = dr::ceil_div(n_users, p.users_per_wg);
  p.n_users_pad = p.n_ublocks * p.users_per_wg;
  const int64_t slots = device_cus();
  const int64_t stage_items = stage_items_for(w, p.cap);
  int max_c_override = 0;
  const int64_t B = p.n_ublocks;
  const int64_t H = (B / slots) * slots;
  // each chunk stays long enough to amortise its start (B fragments, ring
  // fill) and its end compaction; a grid smaller than the CU count (H = 0)
  // may split down to 8192-row chunks: a catalog shorter than 2^17 rows
  // otherwise ran on one CU (1000 users x 100K items: 12.85 -> 4.24 ms).
  // Shorter chunks lose: every chunk compacts each of its users once at its
  // end (~0.9 ms per workgroup), which config 1's 1682-row catalog split in 3
  // paid (5.1 -> 6.0 ms).
  // keep-all plans (small catalogs, no compaction) split down to one stage
  // per chunk: no chunk pays an end compaction, and the few user blocks of
  // such a call would otherwise scan on as many CUs
  const int64_t min_chunk = p.keep_all ? stage_items
                          : H > 0 ? 65536 : std::max<int64_t>(stage_items, 8192);
  if (H > 0 && !seedable) max_c_override = 1;
  const int64_t T = B - H;
  int best_c = 1;
  double best = (double)H / slots + (double)dr::ceil_div(T, slots);
  int max_c = max_c_override > 0 ? max_c_override : kMaxTailChunks;
  if (const int c = knob_int(DR_KNOB_SCAN_SPLIT, 0); c != 0) max_c = c > 0 ? c : 1;  // A/B knob
  // a head user's finalize already sorts 2048 keys when its flush bound
  // passes 1024 (k >= ~800): the tail may then gather as many
  const int head_flush = std::min(k + kSlack + kFlushGap, p.cap - (int)stage_items);
  int max_keys = head_flush > kMaxTailKeys ? 2048 : kMaxTailKeys;
  if (const int m = knob_int(DR_KNOB_TAIL_KEYS, 0); m > 0) max_keys = m;  // A/B knob
  for (int c = 2; c <= max_c && T > 0; ++c) {
    if (n_items / c < min_chunk) break;
    if (!p.keep_all && c * k > max_keys) break;  // each chunk keeps at least k keys
    const double t = (double)H / slots + (double)dr::ceil_div(T * c, slots) / c;
    if (t < best * 0.99) {  // a smaller split unless a larger one gains > 1 %
      best = t;
      best_c = c;
    }
  }
  p.n_head = best_c > 1 ? H : B;
  p.tail_chunks = best_c;
  p.chunk_items = best_c > 1
      ? dr::ceil_div(dr::ceil_div(n_items, best_c), stage_items) * stage_items : n_items;
  p.slack = kSlack;
  // Long lists: once k + kSlack + kFlushGap passes 1024 keys the head finalize
  // sorts 2048 keys anyway, so a buffer may fill to CAP - margin before its
  // first compaction at no finalize cost. A seeded k = 1000 scan admits ~1.5 k
  // survivors (the guess's rank): with the flush at k + 128 = 1128 every user
  // compacted a ~1.1K-key buffer 3-4 times in the last third of the catalog;
  // at CAP - margin = 1792 most users never compact.
  p.gap = head_flush > kMaxTailKeys && kLongFlush ? p.cap - (int)stage_items - k - kSlack
                                                     : kFlushGap;
  // a tail chunk ends with at most end_keep >= k keys, so c of them fit the
  // finalize's max_keys
  p.end_keep = best_c > 1 && !p.keep_all ? std::min(k + kSlack, max_keys / best_c) : 0;
  // Long lists (the flush bound above 1024 keys): every whole-catalog unit ends
  // with a compaction to at most kMaxTailKeys keys (slack kMaxTailKeys - k), so
  // the finalize sorts 1024 keys per user instead of 2048 (k = 1000: the
  // 2048-key sort cost ~24 ms per 1M users).
  p.head_keep = kHeadKeep && head_flush > kMaxTailKeys && k + 8 <= kMaxTailKeys ? kMaxTailKeys : 0;
  p.buf_rows = p.n_users_pad + (int64_t)(best_c - 1) * (B - p.n_head) * p.users_per_wg;
  const int64_t units = p.n_head + (B - p.n_head) * best_c;
  p.grid = (int)(units < slots ? units : slots);
  p.cand_bytes = (size_t)p.buf_rows * p.cap * sizeof(uint64_t);
  p.cnt_bytes = ((size_t)p.buf_rows * sizeof(int32_t) + 255) & ~(size_t)255;
  return p;
}

// Largest candidate count the finalize of a head / split-tail user gathers.
// A whole-catalog buffer ends with at most flush_at keys (the scan compacts
// every buffer above flush_at = min(k + kSlack + kFlushGap, CAP - margin) at
// each stage end, the last included), so k = 100 sorts 256 keys, not CAP = 512
// (the sort instances start at 256 keys).
int flush_keys(const Plan& p, int w, int k) {
  // never compacted: every row's key (and rank k reached: every output slot written)
  if (p.keep_all) return (int)std::max<int64_t>(p.all_keys, k);
  const int f = k + p.slack + p.gap;
  const int m = p.cap - (int)stage_items_for(w, p.cap);
  return f < m ? f : m;
}
int head_keys(const Plan& p, int w, int k) {
  const int n = p.head_keep > 0 ? p.head_keep : flush_keys(p, w, k);
  return n > 256 ? n : 256;
}
int tail_keys(const Plan& p, int w, int k) {
  if (p.tail_chunks <= 1) return head_keys(p, w, k);
  // keep-all chunks are never compacted (not even to head_keep): all their
  // keys, at most n_items <= 2048 over the chunks
  if (p.keep_all) return std::max(256, flush_keys(p, w, k));
  const int n = p.tail_chunks * p.end_keep;
  return n > 256 ? n : 256;
}

// Guessed thresholds (kGuess). A scan that starts at -inf stores every
// running top-k record of a user: ~k * (1 + ln(I / k)) keys, the survivor
// stream that dominates short catalogs (47 % of wave time at d=64 over 1M
// items). Instead a first scan over a strided sample of S = I / kGuessStride
// rows keeps each user's ks best, and the main scan starts from just below the
// ks-th best sample score. ks is the mean number of the user's true top k
// inside the sample plus kGuessSigma standard deviations (+3), so for
// exchangeable catalogs the guess is below the true k-th best score for all
// but ~1e-8 of users. The guess is verified, not trusted: the finalize
// appends every user left with fewer than k keys to a fail list, and those
// users are rescanned from -inf (device-side count, no host sync). Results are
// bit-identical to the plain scan in every case; a catalog whose sampled rows
// are unrepresentative only pays the rescan (one extra unit scan per 1024
// failing users). Used up to kGuessMaxItems rows (measured, 6-sigma margin:
// +14 % at d=64 over 1M items, +6 % at d=128 over 1.25M, +1.7 % over 5M,
// -0.3 to -0.8 % over 10M).
struct Guess {
  int64_t S = 0;       // sample rows (0 = plain scan)
  int64_t stride = 0;  // sample row i is slice row i * stride
  int ks = 0;          // safe rank of the guessed threshold in the sample (second tier)
  int ks1 = 0;         // first-tier rank (<= ks): the main scan's threshold
};

constexpr bool kGuess = true;  // guessed thresholds for catalogs of >= 2^18 rows
constexpr double kGuessSigma = 6.0;
constexpr int kGuessStrideDefault = 32;
// Two-tier guess (round 3): the main scan starts from the sample's
// ks1-th best score; the users it fails are rescanned from their safe
// (6-sigma) threshold by a second-tier scan spread over every CU, and the
// rare users that fail that too by the whole-catalog rescan from -inf.
// ks1 (round 5) is the smallest rank whose Poisson(mu) tail P(X >= ks1) is at
// most kGuessTail = 0.5 % (the share of users expected to fail it); the
// round-3 rule mu + 3 sigma + 1 had tails of 0.12-0.15 %. Measured with the
// z knob giving the same ranks (profiles/r05/ab19/, ab20/, lists identical):
// config 2 (ks1 10 -> 9) -1.05 %, d = 32 -2.7 %, an 8-way shard's 1.25M rows
// -0.8 %, k = 1000 (50 -> 48) -0.2 %; the headline keeps 5 (the 0.84 % tail
// of 4 measured +0.1 %).
int poisson_tail_rank(double mu, double tail) {
  double pmf = std::exp(-mu), cdf = 0.0;
  for (int j = 1; j < 4096; ++j) {
    cdf += pmf;                         // P(X <= j - 1)
    if (1.0 - cdf <= tail) return j;    // P(X >= j)
    pmf *= mu / (double)j;
  }
  return 4096;
}
constexpr double kGuessTail = 0.005;
// catalog chunks per user block of a second-tier rescan: 128 lets the usual
// one or two failing blocks fill the grid (round 6, 64 -> 128: the headline's
// rescan 6.8 -> ~3.9 ms, call -2.9 ms; k = 1000 -1.9 ms; lists identical,
// profiles/r06/rescan_chunks/)
constexpr int kMaxRescanChunks = 128;
constexpr int64_t kGuessStride = kGuessStrideDefault;
constexpr int64_t kGuessMinItems = 1 << 18;
constexpr int kGuessMaxLog2 = 23;  // measured: +1.7 % at 5M rows, -0.3 % at 10M
constexpr int64_t kGuessMaxItems = 1ll << kGuessMaxLog2;
// Long lists pay a survivor stream of ~k (1 + ln(I / k)) keys per user from
// -inf (10K keys at k = 1000 over 10M items: 3.5x the k = 100 scan), which the
// guess removes at any catalog length.
constexpr int kGuessLongK = 256;

// A plan with a split tail is always seeded (from kGuessMinItems rows): an
// unseeded chunk pays the survivor stream of its own catalog part from -inf,
// ~c times the keys of one whole-catalog pass for its users.
Guess guess_for(int64_t n_items, int k, bool split_tail) {
  Guess g;
  if (!kGuess || n_items < kGuessMinItems) return g;
  const int force = knob_int(DR_KNOB_SCAN_SEED, -1);  // A/B knob: 0 never, 1 always
  if (force == 0) return g;
  if (n_items > kGuessMaxItems && k < kGuessLongK && !split_tail && force != 1) return g;
  // Long catalogs sample more sparsely: the sample scan starts from -inf and
  // is survivor-dense (~1.5x the per-row cost of the seeded scan), so about
  // 2^16 sample rows are kept (stride 32 up to 2^22 rows, 64 from 4.2M,
  // 128 from 8.4M). Measured with the split tail at 1M x 10M, d = 128:
  // stride 32 / 64 / 128 / 256 = 1912 / 1879 / 1873 / 1880 ms
  // (profiles/r02_scan/ab_stride_10m.json). Long lists too since round 6
  // (k = 1000 at 1M x 10M, lists identical, profiles/r06/k1000_stride/:
  // stride 32 / 64 / 128 = 1990.8 / 1971.8 / 1963.9 ms; 128 also puts the
  // sample on the dense tile-max path, 9.8 GB instead of 39 GB at 32).
  g.stride = kGuessStride;
  while (g.stride < 128 && n_items / (2 * g.stride) >= 65536) g.stride *= 2;
  if (const int st = knob_int(DR_KNOB_GUESS_STRIDE, 0); st > 1) g.stride = st;  // A/B knob
  // a whole number of 32-row tiles: the sample is stored tile-transposed
  // (sample_rows_kernel), and rows left out only lower the sample's order
  // statistics, so the guess stays a lower bound
  g.S = n_items / g.stride / kTileItems * kTileItems;
  const double mu = (double)k * (double)g.S / (double)n_items;
  int ks = (int)ceil(mu + kGuessSigma * sqrt(mu) + 3.0);
  g.ks = ks < k ? ks : k;
  int ks1 = poisson_tail_rank(mu, kGuessTail);
  double z1 = 3.0, c1 = 1.0;
  const bool zk = dr::plan_knob(DR_KNOB_GUESS_Z1, &z1);  // A/B knobs: the round-3 form
  const bool ck = dr::plan_knob(DR_KNOB_GUESS_C1, &c1);
  if (zk || ck) ks1 = (int)ceil(mu + z1 * sqrt(mu) + c1);
  if (ks1 < 1) ks1 = 1;
  if (knob_int(DR_KNOB_GUESS_TIGHT, 1) == 0) ks1 = g.ks;  // A/B knob: one tier (ks1 = ks)
  g.ks1 = ks1 < g.ks ? ks1 : g.ks;
  return g;
}

size_t diag_bytes() {
#ifdef DR_TOPK_DIAG
  return (size_t)device_cus() * kMaxWaves * kDgSlots * sizeof(uint64_t);
#else
  return 0;
#endif
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout, 256-B aligned pieces:
//   [cand | cnt | thr (tier 1, tier 2) | sample rows | fail rows | fail positions |
//    fail thresholds | tier-2 fail rows | tier-2 fail positions | fail counts | diag].
// The sample scan, the main scan and the rescans run one after the other on
// the stream and share the candidate region.
// The sample scan keeps dense tile maxima (TopkArgs::gmax == 2) when its rank
// fits the dense threshold kernel and the [users][tiles] float matrix fits
// kDenseMaxGiB (it shares the candidate region: the main scan starts after
// the thresholds are read); else the compaction path (gmax == 1).
// DR_KNOB_SAMPLE_DENSE = 0 forces the compaction path (A/B and the
// bit-identity test of the two); a value > 1 is the budget in GiB.
bool sample_dense(int ks, int64_t n_users_pad, int64_t S) {
  double gib = kDenseMaxGiB;
  if (dr::plan_knob(DR_KNOB_SAMPLE_DENSE, &gib) && gib <= 0.0) return false;
  if (gib <= 1.0) gib = kDenseMaxGiB;  // 1: on, default budget
  return ks <= kDenseMaxKs && (double)n_users_pad * (double)(S / kTileItems) * 4.0 <= gib * 1073741824.0;
}
size_t dense_bytes(int64_t n_users_pad, int64_t S) {
  return (size_t)n_users_pad * (size_t)(S / kTileItems) * 4;
}

struct Layout {
  Plan main, sample;
  Guess g;
  bool dense = false;  // the sample scan keeps dense tile maxima
  size_t cand = 0, cnt = 0, thr = 0, samp = 0, frows = 0, fpos = 0, fthr = 0, fcnt = 0, diag = 0;
  size_t off_thr() const { return cand + cnt; }
  size_t off_samp() const { return off_thr() + 2 * thr; }
  size_t off_frows() const { return off_samp() + samp; }
  size_t off_fpos() const { return off_frows() + frows; }
  size_t off_fthr() const { return off_fpos() + fpos; }
  size_t off_frows2() const { return off_fthr() + fthr; }
  size_t off_fpos2() const { return off_frows2() + frows; }
  size_t off_fcnt() const { return off_fpos2() + fpos; }
  size_t off_diag() const { return off_fcnt() + fcnt; }
  size_t total() const { return off_diag() + diag; }
};

Layout make_layout(int64_t n_users, int64_t n_items, int w, int k) {
  Layout L{};
  L.main = make_plan(n_users, n_items, w, k, kGuess && n_items >= kGuessMinItems, true);
  L.g = guess_for(n_items, k, L.main.tail_chunks > 1);
  L.cand = L.main.cand_bytes;
  L.cnt = L.main.cnt_bytes;
  if (L.g.S > 0) {
    L.sample = make_plan(n_users, L.g.S, w, L.g.ks, false);
    // the sample keeps only ks keys per user: compact it tighter
    L.sample.slack = kSampleSlack;
    L.sample.gap = kSampleGap;
    L.dense = sample_dense(L.g.ks, L.sample.n_users_pad, L.g.S);
    const size_t sb = L.dense ? al256(dense_bytes(L.sample.n_users_pad, L.g.S)) : L.sample.cand_bytes;
    L.cand = L.cand > sb ? L.cand : sb;
    L.cnt = L.cnt > L.sample.cnt_bytes ? L.cnt : L.sample.cnt_bytes;
    L.thr = al256((size_t)L.main.n_users_pad * sizeof(float));
    L.samp = al256((size_t)L.g.S * w * 2);
    L.frows = al256((size_t)n_users * sizeof(int64_t));
    L.fpos = al256((size_t)n_users * sizeof(int64_t));
    L.fthr = al256((size_t)n_users * sizeof(float));
    L.fcnt = 256;
  }
  L.diag = diag_bytes();
  return L;
}

// Sample rows, tile-transposed: the S = 32 T sample rows j * stride (j < S)
// are stored so that sample j = q T + r sits in row q of tile r, i.e. output
// row p = 32 r + q. A tile (the GMAX sample scan keeps one max per user and
// tile) then holds samples T apart — catalog rows T * stride apart — so items
// that cluster by id (e.g. ids ordered by popularity) fall into different
// tiles. 16 B per thread.
__global__ __launch_bounds__(256) void sample_rows_kernel(const uint4* __restrict__ I,
                                                          int64_t stride, int64_t S, int cpr,
                                                          uint4* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= S * cpr) return;
  const int64_t p = t / cpr, c = t % cpr;
  const int64_t T = S / kTileItems;
  const int64_t j = (p % kTileItems) * T + p / kTileItems;
  out[t] = I[j * stride * cpr + c];
}


// Row width in bf16 units for a table dtype and embedding width, or -1 when
// no scan is instantiated for it (the host pads other widths with zero
// columns, which change no dot product).
int width_for(int dtype, int d) {
  if (dtype == DR_BF16 && (d == 32 || d == 64 || d == 128 || d == 256 || d == 512)) return d;
  if (dtype == DR_F32 && (d == 32 || d == 64 || d == 128 || d == 256)) return 2 * d;
  return -1;
}

bool launch_scan(const Plan& p, const TopkArgs& a, int dtype, int w, bool seeded, hipStream_t s) {
  return dtype == DR_F32 ? launch_scan_f32(p, a, w, seeded, s)
                         : launch_scan_bf16(p, a, w, seeded, s);
}

// ------------------------------------------------------------------ streaming merge
// Merge of more than 2048 partial entries per user (e.g. 8 shards x top-1000):
// one wave per user keeps the running best keys in elements [0, 1024) of a
// 2048-key register array; every round loads the next <= 1024 input entries
// into elements [1024, 2048) and re-sorts. Needs k_out <= 1024.
__global__ __launch_bounds__(256) void topk_merge_stream_kernel(
    const float* __restrict__ in_s, const int32_t* __restrict__ in_i, int parts, int64_t n_users,
    int k_in, int k_out, float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  constexpr int P = 32;
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  const int64_t total = (int64_t)parts * k_in;
  auto load = [&](int64_t e) -> uint64_t {
    if (e >= total) return 0ull;
    const int64_t p = e / k_in, j = e % k_in;
    const size_t o = ((size_t)p * n_users + u) * k_in + j;
    const int32_t it = in_i[o];
    return it < 0 ? 0ull : dr::make_key(in_s[o], (uint32_t)it);
  };
  uint64_t key[P];
#pragma unroll
  for (int i = 0; i < P; ++i) key[i] = load((int64_t)lane * P + i);
  dr::wave_sort_desc<P>(key);
  for (int64_t next = 64 * P; next < total; next += 32 * P) {
    if (lane >= 32) {  // elements [1024, 2048): the next input block
#pragma unroll
      for (int i = 0; i < P; ++i) key[i] = load(next + (int64_t)(lane - 32) * P + i);
    }
    dr::wave_sort_desc<P>(key);
  }
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    if (e < k_out) {
      const bool empty = key[i] == 0ull;
      out_s[u * k_out + e] = empty ? -INFINITY : dr::key_score(key[i]);
      out_i[u * k_out + e] = empty ? -1 : (int32_t)dr::key_item(key[i]);
    }
  }
}

}  // namespace

extern "C" size_t dr_score_topk_workspace(int64_t n_users, int64_t n_items, int dtype, int d,
                                          int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  const int w = width_for(dtype, d);
  if (w < 0 || cap_for(w, k) < 0) return 0;
  return make_layout(n_users, n_items, w, k).total() + 256;
}

// The launch plan dr_score_topk would use for these arguments on the current
// device (planner knobs included), for tests that must prove which plan they
// ran. out[0..11] = users per workgroup, user blocks, head blocks, tail chunks,
// chunk items, grid, candidate capacity, sample stride (0 = no guess), sample
// rows, sample rank ks (the safe, second-tier rank), main-scan finalize keys
// of a head user / a tail user; out[12] (n_out >= 13) the first-tier rank ks1
// the main scan starts from (= ks for a one-tier guess).
extern "C" int dr_score_topk_plan(int64_t n_users, int64_t n_items, int dtype, int d, int k,
                                  int64_t* out, int n_out) {
  DR_CHECK_ARG(n_users > 0 && n_items > 0, "sizes must be positive");
  DR_CHECK_ARG(k >= 1 && k <= 1024, "k must be in [1, 1024]");
  const int w = width_for(dtype, d);
  DR_CHECK_ARG(w > 0 && cap_for(w, k) > 0, "unsupported dtype / d / k");
  DR_CHECK_ARG(out && n_out >= 12, "out must hold 12 values");
  const Layout L = make_layout(n_users, n_items, w, k);
  const Plan& p = L.main;
  const int64_t v[13] = {p.users_per_wg, p.n_ublocks, p.n_head, p.tail_chunks, p.chunk_items,
                         p.grid, p.cap, L.g.stride, L.g.S, L.g.ks, head_keys(p, w, k),
                         tail_keys(p, w, k), L.g.ks1};
  const int n = n_out < 13 ? n_out : 13;
  for (int i = 0; i < n; ++i) out[i] = v[i];
  return DR_OK;
}

// Users the guessed thresholds failed in the last dr_score_topk call that
// used this workspace with these arguments: out[0] first tier (rescanned from
// the safe threshold), out[1] second tier (rescanned from -inf). Host query:
// a synchronous copy of the device counters (no counters for plain scans: 0).
// Whether that call ran two tiers is read from the workspace (the call
// records it), not re-derived from the current planner knobs.
extern "C" int dr_score_topk_fail_counts(const void* workspace, int64_t n_users, int64_t n_items,
                                         int dtype, int d, int k, int32_t* out) {
  DR_CHECK_ARG(out, "null out");
  out[0] = out[1] = 0;
  const int w = width_for(dtype, d);
  DR_CHECK_ARG(w > 0 && k >= 1 && k <= 1024 && cap_for(w, k) > 0, "unsupported dtype / d / k");
  DR_CHECK_ARG(workspace && n_users > 0 && n_items > 0, "bad arguments");
  const Layout L = make_layout(n_users, n_items, w, k);
  if (L.g.S == 0) return DR_OK;
  const char* ws = (const char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  int32_t c[3] = {0, 0, 0};  // first tier, second tier, "ran two tiers"
  DR_CHECK_HIP(hipMemcpy(c, ws + L.off_fcnt(), sizeof(c), hipMemcpyDeviceToHost));
  out[0] = c[0];
  out[1] = c[2] ? c[1] : c[0];  // one tier: the first count went straight to the -inf rescan
  return DR_OK;
}

#ifdef DR_TOPK_DIAG
// Diag builds only: byte offset (from the 256-B aligned workspace base) of the
// [grid*8][16] u64 counter block of the main scan, and its grid size.
extern "C" size_t dr_score_topk_diag_offset(int64_t n_users, int64_t n_items, int dtype, int d,
                                            int k, int* grid) {
  Layout L = make_layout(n_users, n_items, width_for(dtype, d), k);
  *grid = L.main.grid;
  return L.off_diag();
}
#endif

extern "C" int dr_score_topk(const void* user_table, const int64_t* user_ids, int64_t n_users,
                             const void* item_table, int64_t n_items, int64_t item_base,
                             int dtype, int d, int k, const int64_t* excl_rowptr,
                             const int32_t* excl_items, float* out_scores, int32_t* out_items,
                             void* workspace, size_t workspace_bytes, dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_items >= 0, "negative size");
  DR_CHECK_ARG(k >= 1 && k <= 1024, "k must be in [1, 1024]");
  DR_CHECK_ARG(dtype == DR_BF16 || dtype == DR_F32, "tables must be DR_BF16 or DR_F32");
  const int w = width_for(dtype, d);
  DR_CHECK_ARG(w > 0, dtype == DR_BF16 ? "bf16 d must be one of 32, 64, 128, 256, 512"
                                       : "fp32 d must be one of 32, 64, 128, 256");
  DR_CHECK_ARG(cap_for(w, k) > 0, "k too large for this d");
  DR_CHECK_ARG(item_base >= 0 && item_base + n_items < 0x7fffffffLL,
               "global item ids must fit int32");
  DR_CHECK_ARG((excl_rowptr == nullptr) == (excl_items == nullptr),
               "excl_rowptr and excl_items must both be set or both be NULL");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(user_table && out_scores && out_items, "null pointer");
  if (n_items == 0) {
    dr::set_error("dr_score_topk: empty catalog");
    return DR_EINVAL;
  }
  DR_CHECK_ARG(item_table, "null item_table");
  hipStream_t s = (hipStream_t)stream;
  const Layout L = make_layout(n_users, n_items, w, k);
  const size_t need = L.total();
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if (!workspace || (size_t)(ws - (char*)workspace) + need > workspace_bytes) {
    dr::set_error("dr_score_topk: workspace too small (need " + std::to_string(need + 256) +
                  " bytes)");
    return DR_EWORKSPACE;
  }
  const Plan& p = L.main;
  TopkArgs a{};
  a.U = (const char*)user_table;
  a.user_ids = user_ids;
  a.n_users = n_users;
  a.n_users_pad = p.n_users_pad;
  a.I = (const char*)item_table;
  a.n_items = n_items;
  a.item_base = item_base;
  a.k = k;
  a.excl_rowptr = excl_rowptr;
  a.excl_items = excl_items;
  a.n_ublocks = p.n_ublocks;
  a.n_head = p.n_head;
  a.tail_chunks = p.tail_chunks;
  a.chunk_items = p.chunk_items;
  a.end_keep = p.end_keep;
  a.head_keep = p.head_keep;
  a.slack = p.slack;
  a.gap = p.gap;
  a.keep_all = p.keep_all;  // the main scan only (small catalogs: no guess, no rescans)
  a.init_thr = nullptr;
  a.n_users_dev = nullptr;
  a.pos_map = nullptr;
  a.cand = (uint64_t*)ws;
  a.cnt = (int32_t*)(ws + L.cand);
  a.diag = (uint64_t*)(ws + L.off_diag());  // written only in DIAG builds
  const BufMap bm = buf_map(p);
  const int64_t head_end = p.head_users() < n_users ? p.head_users() : n_users;

#define DR_SCAN_OR_FAIL(PLAN, ARGS, SEEDED)                                  \
  if (!launch_scan(PLAN, ARGS, dtype, w, SEEDED, s)) {                       \
    dr::set_error("dr_score_topk: internal plan error (no scan instance)"); \
    return DR_EUNSUPPORTED;                                                  \
  }
#define DR_BY_P(PP_EXPR, LAUNCH)                                           \
  switch (PP_EXPR) {                                                       \
    case 4: LAUNCH(4); break;                                              \
    case 8: LAUNCH(8); break;                                              \
    case 16: LAUNCH(16); break;                                            \
    case 32: LAUNCH(32); break;                                            \
    default:                                                               \
      dr::set_error("dr_score_topk: internal plan error (candidate sort)"); \
      return DR_EUNSUPPORTED;                                              \
  }
  // finalize of users [U0, U1) (one wave each), P sized for their key count
#define DR_FIN(PP)                                                                             \
  hipLaunchKernelGGL((topk_finalize_kernel<PP>), dim3((unsigned)dr::ceil_div(U1 - U0, 4)),      \
                     dim3(256), 0, s, a.cand, a.cnt, FMAP, p.cap, U0, U1, k, excl_rowptr,        \
                     excl_items, out_scores, out_items, FPOS, FNDEV, FUIDS, FCNT, frows, fpos,   \
                     FTSRC, fthr)
  // head users (one buffer each), then the split tail's users (their chunks)
#define DR_FIN_ALL()                                                        \
  {                                                                         \
    const BufMap FMAP = bm;                                                 \
    int64_t U0 = 0, U1 = head_end;                                          \
    if (U1 > U0) { DR_BY_P(p_for(head_keys(p, w, k)), DR_FIN) DR_CHECK_LAUNCH(); } \
    U0 = head_end;                                                          \
    U1 = n_users;                                                           \
    if (U1 > U0) { DR_BY_P(p_for(tail_keys(p, w, k)), DR_FIN) DR_CHECK_LAUNCH(); } \
  }

  if (L.g.S == 0) {
    DR_SCAN_OR_FAIL(p, a, false)
    DR_CHECK_LAUNCH();
    int64_t* frows = nullptr;
    int64_t* fpos = nullptr;
    float* fthr = nullptr;
    const int64_t* FPOS = nullptr;
    const int32_t* FNDEV = nullptr;
    const int64_t* FUIDS = user_ids;
    int32_t* FCNT = nullptr;
    const float* FTSRC = nullptr;
    DR_FIN_ALL()
    return DR_OK;
  }

  // ---- guessed thresholds: sample scan -> thresholds -> seeded scan -> verify
  const bool two_tier = L.g.ks1 < L.g.ks;
  float* thr = (float*)(ws + L.off_thr());
  float* thr2 = two_tier ? (float*)(ws + L.off_thr() + L.thr) : nullptr;
  char* samp = ws + L.off_samp();
  int64_t* frows = (int64_t*)(ws + L.off_frows());
  int64_t* fpos = (int64_t*)(ws + L.off_fpos());
  float* fthr = two_tier ? (float*)(ws + L.off_fthr()) : nullptr;
  int64_t* frows2 = (int64_t*)(ws + L.off_frows2());
  int64_t* fpos2 = (int64_t*)(ws + L.off_fpos2());
  // [0] first-tier failures, [1] second-tier, [2] 1 if this call ran two tiers
  int32_t* fcnt = (int32_t*)(ws + L.off_fcnt());
  DR_CHECK_HIP(hipMemsetAsync(fcnt, 0, 2 * sizeof(int32_t), s));
  DR_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)(fcnt + 2), two_tier ? 1 : 0, 1, s));
  {
    const int cpr = w / 8;  // 16-B chunks per row
    const int64_t n16 = L.g.S * cpr;
    hipLaunchKernelGGL(sample_rows_kernel, dim3((unsigned)dr::ceil_div(n16, 256)), dim3(256), 0, s,
                       (const uint4*)item_table, L.g.stride, L.g.S, cpr, (uint4*)samp);
    DR_CHECK_LAUNCH();
  }
  const Plan& ps = L.sample;
  TopkArgs as = a;  // sample ids are sample rows: no exclusions, no item base
  as.I = samp;
  as.n_items = L.g.S;
  as.item_base = 0;
  as.k = L.g.ks;
  as.excl_rowptr = nullptr;
  as.excl_items = nullptr;
  as.n_head = ps.n_head;
  as.tail_chunks = ps.tail_chunks;
  as.chunk_items = ps.chunk_items;
  as.end_keep = ps.end_keep;
  as.head_keep = ps.head_keep;
  as.slack = ps.slack;
  as.gap = ps.gap;
  as.keep_all = 0;
  as.gmax = L.dense ? 2 : kSampleGmax;
  as.tmax = (float*)ws;  // the candidate region
  as.tmax_tiles = L.g.S / kTileItems;
  DR_SCAN_OR_FAIL(ps, as, false)
  DR_CHECK_LAUNCH();
  if (L.dense) {
    if (!launch_threshold_dense(as.tmax, as.tmax_tiles, p.n_users_pad, n_users, L.g.ks, L.g.ks1,
                                thr, thr2, s)) {
      dr::set_error("dr_score_topk: internal plan error (dense threshold rank)");
      return DR_EUNSUPPORTED;
    }
    DR_CHECK_LAUNCH();
  } else {
    const BufMap sm = buf_map(ps);
    const int64_t sh = ps.head_users();
#define DR_THR(PP)                                                                             \
  hipLaunchKernelGGL((topk_threshold_kernel<PP>), dim3((unsigned)dr::ceil_div(T1 - T0, 4)),     \
                     dim3(256), 0, s, a.cand, a.cnt, sm, ps.cap, T0, T1, n_users, L.g.ks,        \
                     L.g.ks1, thr, thr2)
    int64_t T0 = 0, T1 = sh < p.n_users_pad ? sh : p.n_users_pad;
    if (T1 > T0) { DR_BY_P(p_for(head_keys(ps, w, L.g.ks)), DR_THR) DR_CHECK_LAUNCH(); }
    T0 = T1;
    T1 = p.n_users_pad;
    if (T1 > T0) { DR_BY_P(p_for(tail_keys(ps, w, L.g.ks)), DR_THR) DR_CHECK_LAUNCH(); }
#undef DR_THR
  }

  a.init_thr = thr;
  DR_SCAN_OR_FAIL(p, a, true)
  DR_CHECK_LAUNCH();
  {
    const int64_t* FPOS = nullptr;
    const int32_t* FNDEV = nullptr;
    const int64_t* FUIDS = user_ids;
    int32_t* FCNT = fcnt;  // verify: users left with fewer than k keys
    const float* FTSRC = thr2;
    DR_FIN_ALL()
  }

  // ---- second tier (two-tier guesses): the first tier's failures rescanned
  // from their safe thresholds, every failing user block split over the CUs
  // (plan on the device: the count is there), any number of keys per user
  // merged by the streaming finalize; its own failures go to the third tier
  const int64_t* t3_rows = frows;
  const int64_t* t3_pos = fpos;
  const int32_t* t3_cnt = fcnt;
  if (two_tier) {
    TopkArgs a2 = a;
    a2.init_thr = fthr;
    a2.user_ids = frows;
    a2.pos_map = fpos;
    a2.n_users_dev = fcnt;
    a2.n_head = 0;
    a2.end_keep = 0;
    a2.keep_all = 0;
    a2.dev_split = kMaxRescanChunks;
    a2.buf_blocks = p.buf_rows / p.users_per_wg;
    a2.diag = nullptr;
    Plan p2 = p;
    p2.grid = device_cus();
    DR_SCAN_OR_FAIL(p2, a2, true)
    DR_CHECK_LAUNCH();
    DevSplitArgs dsa;
    dsa.upwg = p.users_per_wg;
    dsa.grid = p2.grid;
    dsa.max_c = kMaxRescanChunks;
    dsa.buf_blocks = a2.buf_blocks;
    dsa.n_items = n_items;
    dsa.stage_items = stage_items_for(w, p.cap);
    hipLaunchKernelGGL(topk_finalize_stream_kernel, dim3((unsigned)dr::ceil_div(n_users, 4)),
                       dim3(256), 0, s, a.cand, a.cnt, dsa, p.cap, n_users, k, excl_rowptr,
                       excl_items, out_scores, out_items, fpos, fcnt, frows, fcnt + 1, frows2,
                       fpos2);
    DR_CHECK_LAUNCH();
    t3_rows = frows2;
    t3_pos = fpos2;
    t3_cnt = fcnt + 1;
  }

  // ---- third tier: the users every guess failed (usually none), rescanned
  // from -inf; whole-catalog units only, one buffer per listed user
  TopkArgs af = a;
  af.init_thr = nullptr;
  af.user_ids = t3_rows;
  af.pos_map = t3_pos;
  af.n_users_dev = t3_cnt;
  af.n_head = p.n_ublocks;
  af.tail_chunks = 1;
  af.chunk_items = n_items;
  af.end_keep = 0;
  af.keep_all = 0;
  af.diag = nullptr;
  DR_SCAN_OR_FAIL(p, af, false)
  DR_CHECK_LAUNCH();
  {
    const BufMap FMAP{p.n_users_pad, p.n_users_pad, 0, 1};
    const int64_t U0 = 0, U1 = n_users;
    const int64_t* FPOS = t3_pos;
    const int32_t* FNDEV = t3_cnt;
    const int64_t* FUIDS = t3_rows;
    int32_t* FCNT = nullptr;
    const float* FTSRC = nullptr;
    DR_BY_P(p_for(head_keys(p, w, k)), DR_FIN)
    DR_CHECK_LAUNCH();
  }
#undef DR_FIN_ALL
#undef DR_FIN
#undef DR_BY_P
#undef DR_SCAN_OR_FAIL
  return DR_OK;
}

// ------------------------------------------------------------------ caller-seeded scan
// dr_score_topk_seeded: the top-k, in the key order, of the items scoring
// strictly above the caller's per-user threshold (the item-sharded multi-GPU
// top-k passes thresholds guessed from a sample of the WHOLE catalog, so a
// shard keeps only items that can reach the global top-k; divrec.distributed).
// One seeded scan (split tail allowed) and one finalize; no guess, no verify.
Plan seeded_plan(int64_t n_users, int64_t n_items, int w, int k) {
  return make_plan(n_users, n_items, w, k, true);
}

extern "C" size_t dr_score_topk_seeded_workspace(int64_t n_users, int64_t n_items, int dtype,
                                                 int d, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  const int w = width_for(dtype, d);
  if (w < 0 || cap_for(w, k) < 0) return 0;
  const Plan p = seeded_plan(n_users, n_items, w, k);
  return p.cand_bytes + p.cnt_bytes + diag_bytes() + 256;
}

extern "C" int dr_score_topk_seeded(const void* user_table, const int64_t* user_ids,
                                    int64_t n_users, const void* item_table, int64_t n_items,
                                    int64_t item_base, int dtype, int d, int k,
                                    const float* init_thr, const int64_t* excl_rowptr,
                                    const int32_t* excl_items, float* out_scores,
                                    int32_t* out_items, void* workspace, size_t workspace_bytes,
                                    dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_items >= 0, "negative size");
  DR_CHECK_ARG(k >= 1 && k <= 1024, "k must be in [1, 1024]");
  DR_CHECK_ARG(dtype == DR_BF16 || dtype == DR_F32, "tables must be DR_BF16 or DR_F32");
  const int w = width_for(dtype, d);
  DR_CHECK_ARG(w > 0, dtype == DR_BF16 ? "bf16 d must be one of 32, 64, 128, 256, 512"
                                       : "fp32 d must be one of 32, 64, 128, 256");
  DR_CHECK_ARG(cap_for(w, k) > 0, "k too large for this d");
  DR_CHECK_ARG(item_base >= 0 && item_base + n_items < 0x7fffffffLL,
               "global item ids must fit int32");
  DR_CHECK_ARG((excl_rowptr == nullptr) == (excl_items == nullptr),
               "excl_rowptr and excl_items must both be set or both be NULL");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(user_table && out_scores && out_items && init_thr, "null pointer");
  if (n_items == 0) {
    dr::set_error("dr_score_topk_seeded: empty catalog");
    return DR_EINVAL;
  }
  DR_CHECK_ARG(item_table, "null item_table");
  hipStream_t s = (hipStream_t)stream;
  const Plan p = seeded_plan(n_users, n_items, w, k);
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  const size_t need = p.cand_bytes + p.cnt_bytes + diag_bytes();
  if (!workspace || (size_t)(ws - (char*)workspace) + need > workspace_bytes) {
    dr::set_error("dr_score_topk_seeded: workspace too small (need " +
                  std::to_string(need + 256) + " bytes)");
    return DR_EWORKSPACE;
  }
  TopkArgs a{};
  a.U = (const char*)user_table;
  a.user_ids = user_ids;
  a.n_users = n_users;
  a.n_users_pad = p.n_users_pad;
  a.I = (const char*)item_table;
  a.n_items = n_items;
  a.item_base = item_base;
  a.k = k;
  a.excl_rowptr = excl_rowptr;
  a.excl_items = excl_items;
  a.n_ublocks = p.n_ublocks;
  a.n_head = p.n_head;
  a.tail_chunks = p.tail_chunks;
  a.chunk_items = p.chunk_items;
  a.end_keep = p.end_keep;
  a.head_keep = p.head_keep;
  a.slack = p.slack;
  a.gap = p.gap;
  a.init_thr = init_thr;
  a.cand = (uint64_t*)ws;
  a.cnt = (int32_t*)(ws + p.cand_bytes);
  a.diag = (uint64_t*)(ws + p.cand_bytes + p.cnt_bytes);
  if (!launch_scan(p, a, dtype, w, true, s)) {
    dr::set_error("dr_score_topk_seeded: internal plan error (no scan instance)");
    return DR_EUNSUPPORTED;
  }
  DR_CHECK_LAUNCH();
  const BufMap bm = buf_map(p);
  const int64_t head_end = p.head_users() < n_users ? p.head_users() : n_users;
  int64_t U0 = 0, U1 = head_end;
  for (int part = 0; part < 2; ++part) {
    if (U1 > U0) {
      const int P = p_for(part == 0 ? head_keys(p, w, k) : tail_keys(p, w, k));
      const dim3 grid((unsigned)dr::ceil_div(U1 - U0, 4));
#define DR_FIN_SEEDED(PP)                                                                       \
  hipLaunchKernelGGL((topk_finalize_kernel<PP>), grid, dim3(256), 0, s, a.cand, a.cnt, bm, p.cap, \
                     U0, U1, k, excl_rowptr, excl_items, out_scores, out_items, nullptr, nullptr,  \
                     user_ids, nullptr, nullptr, nullptr, nullptr, nullptr)
      switch (P) {
        case 4: DR_FIN_SEEDED(4); break;
        case 8: DR_FIN_SEEDED(8); break;
        case 16: DR_FIN_SEEDED(16); break;
        case 32: DR_FIN_SEEDED(32); break;
        default:
          dr::set_error("dr_score_topk_seeded: internal plan error (candidate sort)");
          return DR_EUNSUPPORTED;
      }
#undef DR_FIN_SEEDED
      DR_CHECK_LAUNCH();
    }
    U0 = head_end;
    U1 = n_users;
  }
  return DR_OK;
}

// ------------------------------------------------------------------ sample thresholds
// dr_sample_thresholds: the guess of dr_score_topk on a caller-gathered sample
// (divrec.distributed.global_thresholds): tile-transposed copy of the whole
// tiles of the sample, the GMAX sample scan (k = ks), thresholds at ranks ks1
// and ks. Workspace: [cand | cnt | transposed sample].
struct SampleThrLayout {
  Plan p;
  int64_t S = 0;
  bool dense = false;
  size_t cand = 0, cnt = 0, samp = 0;
  size_t total() const { return cand + cnt + samp; }
};

SampleThrLayout sample_thr_layout(int64_t n_users, int64_t n_sample, int w, int ks) {
  SampleThrLayout L;
  L.S = n_sample / kTileItems * kTileItems;
  if (L.S == 0) return L;
  L.p = make_plan(n_users, L.S, w, ks, false);
  L.p.slack = kSampleSlack;
  L.p.gap = kSampleGap;
  L.dense = sample_dense(ks, L.p.n_users_pad, L.S);
  L.cand = al256(L.dense ? dense_bytes(L.p.n_users_pad, L.S) : L.p.cand_bytes);
  L.cnt = al256(L.p.cnt_bytes);
  L.samp = al256((size_t)L.S * w * 2);
  return L;
}

// out row p = 32 r + q <- sample row q T + r (T = S / 32), 16 B per thread
__global__ __launch_bounds__(256) void transpose_tiles_kernel(const uint4* __restrict__ in,
                                                              int64_t S, int cpr,
                                                              uint4* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= S * cpr) return;
  const int64_t p = t / cpr, c = t % cpr;
  const int64_t T = S / kTileItems;
  out[t] = in[((p % kTileItems) * T + p / kTileItems) * cpr + c];
}

__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ a, float* __restrict__ b,
                                                       int64_t n, float v) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n) {
    a[t] = v;
    b[t] = v;
  }
}

extern "C" size_t dr_sample_thresholds_workspace(int64_t n_users, int64_t n_sample, int dtype,
                                                 int d, int ks) {
  if (n_users <= 0 || n_sample < 0 || ks <= 0 || ks > 256) return 0;
  const int w = width_for(dtype, d);
  if (w < 0 || cap_for(w, ks) < 0) return 0;
  return sample_thr_layout(n_users, n_sample, w, ks).total() + 256;
}

extern "C" int dr_sample_thresholds(const void* user_table, const int64_t* user_ids,
                                    int64_t n_users, const void* sample_rows, int64_t n_sample,
                                    int dtype, int d, int ks1, int ks, float* thr1, float* thr2,
                                    void* workspace, size_t workspace_bytes, dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_sample >= 0, "negative size");
  DR_CHECK_ARG(ks >= 1 && ks <= 256 && ks1 >= 1 && ks1 <= ks, "need 1 <= ks1 <= ks <= 256");
  DR_CHECK_ARG(dtype == DR_BF16 || dtype == DR_F32, "tables must be DR_BF16 or DR_F32");
  const int w = width_for(dtype, d);
  DR_CHECK_ARG(w > 0 && cap_for(w, ks) > 0, "unsupported dtype / d");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(user_table && thr1 && thr2, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const SampleThrLayout L = sample_thr_layout(n_users, n_sample, w, ks);
  if (L.S == 0) {  // no whole tile of sample rows: no guess
    hipLaunchKernelGGL(fill_f32_kernel, dim3((unsigned)dr::ceil_div(n_users, 256)), dim3(256), 0, s,
                       thr1, thr2, n_users, -INFINITY);
    DR_CHECK_LAUNCH();
    return DR_OK;
  }
  DR_CHECK_ARG(sample_rows, "null sample_rows");
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if (!workspace || (size_t)(ws - (char*)workspace) + L.total() > workspace_bytes) {
    dr::set_error("dr_sample_thresholds: workspace too small (need " +
                  std::to_string(L.total() + 256) + " bytes)");
    return DR_EWORKSPACE;
  }
  char* samp = ws + L.cand + L.cnt;
  {
    const int cpr = w / 8;
    hipLaunchKernelGGL(transpose_tiles_kernel, dim3((unsigned)dr::ceil_div(L.S * cpr, 256)),
                       dim3(256), 0, s, (const uint4*)sample_rows, L.S, cpr, (uint4*)samp);
    DR_CHECK_LAUNCH();
  }
  const Plan& p = L.p;
  TopkArgs a{};
  a.U = (const char*)user_table;
  a.user_ids = user_ids;
  a.n_users = n_users;
  a.n_users_pad = p.n_users_pad;
  a.I = samp;
  a.n_items = L.S;
  a.k = ks;
  a.n_ublocks = p.n_ublocks;
  a.n_head = p.n_head;
  a.tail_chunks = p.tail_chunks;
  a.chunk_items = p.chunk_items;
  a.end_keep = p.end_keep;
  a.head_keep = p.head_keep;
  a.slack = p.slack;
  a.gap = p.gap;
  a.gmax = L.dense ? 2 : 1;
  a.tmax = (float*)ws;
  a.tmax_tiles = L.S / kTileItems;
  a.cand = (uint64_t*)ws;
  a.cnt = (int32_t*)(ws + L.cand);
  if (!launch_scan(p, a, dtype, w, false, s)) {
    dr::set_error("dr_sample_thresholds: internal plan error (no scan instance)");
    return DR_EUNSUPPORTED;
  }
  DR_CHECK_LAUNCH();
  if (L.dense) {
    if (!launch_threshold_dense(a.tmax, a.tmax_tiles, n_users, n_users, ks, ks1, thr1, thr2, s)) {
      dr::set_error("dr_sample_thresholds: internal plan error (dense threshold rank)");
      return DR_EUNSUPPORTED;
    }
    DR_CHECK_LAUNCH();
    return DR_OK;
  }
  const BufMap sm = buf_map(p);
  const int64_t sh = p.head_users() < n_users ? p.head_users() : n_users;
  int64_t T0 = 0, T1 = sh;
  for (int part = 0; part < 2; ++part) {
    if (T1 > T0) {
      const int P = p_for(part == 0 ? head_keys(p, w, ks) : tail_keys(p, w, ks));
#define DR_STHR(PP)                                                                              \
  hipLaunchKernelGGL((topk_threshold_kernel<PP>), dim3((unsigned)dr::ceil_div(T1 - T0, 4)),      \
                     dim3(256), 0, s, a.cand, a.cnt, sm, p.cap, T0, T1, n_users, ks, ks1, thr1, thr2)
      switch (P) {
        case 4: DR_STHR(4); break;
        case 8: DR_STHR(8); break;
        case 16: DR_STHR(16); break;
        case 32: DR_STHR(32); break;
        default:
          dr::set_error("dr_sample_thresholds: internal plan error (candidate sort)");
          return DR_EUNSUPPORTED;
      }
#undef DR_STHR
      DR_CHECK_LAUNCH();
    }
    T0 = sh;
    T1 = n_users;
  }
  return DR_OK;
}

extern "C" int dr_topk_merge(const float* in_scores, const int32_t* in_items, int parts,
                             int64_t n_users, int k_in, int k_out, float* out_scores,
                             int32_t* out_items, dr_stream_t stream) {
  DR_CHECK_ARG(parts >= 1 && k_in >= 1 && k_out >= 1, "parts, k_in, k_out must be >= 1");
  DR_CHECK_ARG((int64_t)k_out <= (int64_t)parts * k_in, "k_out must be <= parts * k_in");
  const int64_t total = (int64_t)parts * k_in;
  DR_CHECK_ARG(total <= 2048 || k_out <= 1024,
               "k_out must be <= 1024 when parts * k_in > 2048");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(in_scores && in_items && out_scores && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)dr::ceil_div(n_users, 4);
  if (total > 2048) {
    hipLaunchKernelGGL(topk_merge_stream_kernel, dim3(grid), dim3(256), 0, s, in_scores, in_items,
                       parts, n_users, k_in, k_out, out_scores, out_items);
    DR_CHECK_LAUNCH();
    return DR_OK;
  }
#define DR_MERGE(PP)                                                                        \
  hipLaunchKernelGGL((topk_merge_kernel<PP>), dim3(grid), dim3(256), 0, s, in_scores,       \
                     in_items, parts, n_users, k_in, k_out, out_scores, out_items)
  switch (p_for((int)total)) {
    case 2: DR_MERGE(2); break;
    case 4: DR_MERGE(4); break;
    case 8: DR_MERGE(8); break;
    case 16: DR_MERGE(16); break;
    default: DR_MERGE(32); break;
  }
#undef DR_MERGE
  DR_CHECK_LAUNCH();
  return DR_OK;
}
