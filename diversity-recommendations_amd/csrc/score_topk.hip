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
#include "score_scan.h"

namespace {

using namespace dr_topk;

// ------------------------------------------------------------------ per-user gather
// One user's candidate keys of every chunk into registers (element e = lane*P
// + i), excluded items dropped; 0 = empty.
template <int P>
__device__ __forceinline__ void gather_candidates(const uint64_t* __restrict__ cand,
                                                  const int32_t* __restrict__ cnt, int n_chunks,
                                                  int cap, int64_t u, int64_t n_users_pad,
                                                  const int64_t* __restrict__ excl_rowptr,
                                                  const int32_t* __restrict__ excl_items,
                                                  int64_t er, uint64_t (&key)[P]) {
  const int lane = dr::lane_id();
  int off[9];
  off[0] = 0;
  for (int c = 0; c < 8; ++c)
    off[c + 1] = off[c] + (c < n_chunks ? cnt[(size_t)c * n_users_pad + u] : 0);
  const int total = off[8];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    uint64_t v = 0ull;
    if (e < total) {
      int c = 0;
#pragma unroll
      for (int q = 1; q < 8; ++q) c += (e >= off[q]) ? 1 : 0;
      int base = off[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) base = (c == q) ? off[q] : base;
      v = cand[((size_t)c * n_users_pad + u) * cap + (e - base)];
    }
    key[i] = v;
  }
  if (excl_rowptr) {  // er: the user's exclusion row
    const int64_t e0 = excl_rowptr[er], e1 = excl_rowptr[er + 1];
#pragma unroll
    for (int i = 0; i < P; ++i)
      if (key[i] != 0ull &&
          sorted_contains(excl_items + e0, (int)(e1 - e0), (int32_t)dr::key_item(key[i])))
        key[i] = 0ull;
  }
}

// ------------------------------------------------------------------ finalize
// One wave per user: all chunks' candidate keys -> drop excluded items ->
// wave-wide register bitonic sort -> k best, decoded.
//   * Guessed-threshold scans (fail_cnt != NULL): a user left with fewer than
//     k keys may have lost items to a threshold guessed too high; it is
//     appended to the fail list (its user row and position) for the rescan.
//   * The rescan's finalize (pos_map != NULL): list entry u is written to the
//     caller's position pos_map[u]; the count comes from the device.
template <int P>
__global__ __launch_bounds__(256) void topk_finalize_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, int n_chunks, int cap,
    int64_t n_users, int64_t n_users_pad, int k, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, float* __restrict__ out_s,
    int32_t* __restrict__ out_i, const int64_t* __restrict__ pos_map,
    const int32_t* __restrict__ n_users_dev, const int64_t* __restrict__ user_ids,
    int32_t* __restrict__ fail_cnt, int64_t* __restrict__ fail_rows,
    int64_t* __restrict__ fail_pos) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (n_users_dev) {
    const int64_t n = *n_users_dev;
    n_users = n < n_users ? n : n_users;
  }
  if (u >= n_users) return;  // wave-uniform
  const int64_t op = pos_map ? pos_map[u] : u;  // output and exclusion row
  uint64_t key[P];
  gather_candidates<P>(cand, cnt, n_chunks, cap, u, n_users_pad, excl_rowptr, excl_items, op, key);
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
  if (fail_cnt && lane == (k - 1) / P && dr::select_reg<P>(key, (k - 1) % P) == 0ull) {
    const int32_t f = atomicAdd(fail_cnt, 1);
    fail_rows[f] = user_ids ? user_ids[u] : u;
    fail_pos[f] = u;
  }
}

// ------------------------------------------------------------------ threshold
// One wave per user position of the sample scan: the starting threshold of the
// main scan, strictly below the user's k-th best (non-excluded) sample score,
// so every score >= it passes the scan's `score > thr` test. -inf when the
// sample holds fewer than k candidates; +inf for padding positions (no user).
template <int P>
__global__ __launch_bounds__(256) void topk_threshold_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, int n_chunks, int cap,
    int64_t n_users, int64_t n_users_pad, int k, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, float* __restrict__ thr) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users_pad) return;  // wave-uniform
  if (u >= n_users) {
    if (lane == 0) thr[u] = INFINITY;
    return;
  }
  uint64_t key[P];
  gather_candidates<P>(cand, cnt, n_chunks, cap, u, n_users_pad, excl_rowptr, excl_items, u, key);
  dr::wave_sort_desc<P>(key);
  const int e = k - 1;
  if (lane == e / P) {
    const uint64_t kk = dr::select_reg<P>(key, e % P);
    float t = -INFINITY;
    if (kk != 0ull) {
      const float s = dr::key_score(kk);
      const float below = s - fmaxf(fabsf(s) * 0x1p-20f, 0x1p-100f);
      t = below < s ? below : -INFINITY;  // NaN / inf scores: no pruning
    }
    thr[u] = t;
  }
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
int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return cus > 0 ? cus : 256;
}

int64_t stage_items_for(int w) {
  return (int64_t)(stage_bytes_for(w) / (kTileItems * w * 2)) * kTileItems;
}

// Smallest candidate capacity that leaves at least 32 keys of headroom above
// k + kSlack once a stage's worth of new keys (the margin) is reserved.
int cap_for(int w, int k) {
  const int margin = (int)stage_items_for(w);
  for (int cap = 512; cap <= 2048; cap <<= 1)
    if (k + kSlack + 32 <= cap - margin) return cap;
  return -1;
}

Plan make_plan(int64_t n_users, int64_t n_items, int w, int k) {
  Plan p{};
  p.cap = cap_for(w, k);
  p.users_per_wg = nut_for(w) * 32 * kWaves;
  p.n_ublocks = dr::ceil_div(n_users, p.users_per_wg);
  p.n_users_pad = p.n_ublocks * p.users_per_wg;
  const int slots = device_cus();  // one 512-thread workgroup per CU
  const int64_t stage_items = stage_items_for(w);
  // Split the catalog into chunks only to balance the tail of the grid; each
  // chunk must stay long enough to amortise its start, and the finalize
  // kernel sorts at most 2048 candidates per user.
  const int64_t min_chunk = 65536;
  int best_s = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && n_items / s < min_chunk) break;
    if ((int64_t)s * p.cap > 2048) break;
    const int64_t units = p.n_ublocks * s;
    const int64_t rounds = dr::ceil_div(units, slots);
    const double eff = (double)units / (double)(rounds * slots);
    if (eff > best_eff + 0.02) {
      best_eff = eff;
      best_s = s;
    }
  }
  p.n_chunks = best_s;
  p.chunk_items = dr::ceil_div(dr::ceil_div(n_items, best_s), stage_items) * stage_items;
  const int64_t units = p.n_ublocks * p.n_chunks;
  p.grid = (int)(units < slots ? units : slots);
  p.cand_bytes = (size_t)p.n_chunks * p.n_users_pad * p.cap * sizeof(uint64_t);
  p.cnt_bytes = ((size_t)p.n_chunks * p.n_users_pad * sizeof(int32_t) + 255) & ~(size_t)255;
  return p;
}

// Guessed thresholds (DR_GUESS). A scan that starts at -inf stores every
// running top-k record of a user: ~k * (1 + ln(I / k)) keys, the survivor
// stream that dominates short catalogs (47 % of wave time at d=64 over 1M
// items). Instead a first scan over a strided sample of S = I / kGuessStride
// rows keeps each user's ks best, and the main scan starts from just below the
// ks-th best sample score. ks is the mean number of the user's true top k
// inside the sample plus DR_GUESS_SIGMA standard deviations (+3), so for
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
  int ks = 0;          // rank of the guessed threshold in the sample
};

#ifndef DR_GUESS
#define DR_GUESS 1
#endif
#ifndef DR_GUESS_SIGMA
#define DR_GUESS_SIGMA 6.0
#endif
#ifndef DR_GUESS_STRIDE
#define DR_GUESS_STRIDE 32
#endif
constexpr int64_t kGuessStride = DR_GUESS_STRIDE;
constexpr int64_t kGuessMinItems = 1 << 18;
#ifndef DR_GUESS_MAX_LOG2
#define DR_GUESS_MAX_LOG2 23  // measured: +1.7 % at 5M rows, -0.3 % at 10M
#endif
constexpr int64_t kGuessMaxItems = 1ll << DR_GUESS_MAX_LOG2;
// Long lists pay a survivor stream of ~k (1 + ln(I / k)) keys per user from
// -inf (10K keys at k = 1000 over 10M items: 3.5x the k = 100 scan), which the
// guess removes at any catalog length.
#ifndef DR_GUESS_LONG_K
#define DR_GUESS_LONG_K 256
#endif

Guess guess_for(int64_t n_items, int k) {
  Guess g;
  if (!DR_GUESS || n_items < kGuessMinItems) return g;
  if (n_items > kGuessMaxItems && k < DR_GUESS_LONG_K) return g;
  g.stride = kGuessStride;
  g.S = n_items / kGuessStride;
  const double mu = (double)k * (double)g.S / (double)n_items;
  int ks = (int)ceil(mu + DR_GUESS_SIGMA * sqrt(mu) + 3.0);
  g.ks = ks < k ? ks : k;
  return g;
}

size_t diag_bytes() {
#ifdef DR_TOPK_DIAG
  return (size_t)device_cus() * kWaves * kDgSlots * sizeof(uint64_t);
#else
  return 0;
#endif
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout, 256-B aligned pieces:
//   [cand | cnt | thr | sample rows | fail rows | fail positions | fail count | diag].
// The sample scan, the main scan and the rescan run one after the other on
// the stream and share the candidate region.
struct Layout {
  Plan main, sample;
  Guess g;
  size_t cand = 0, cnt = 0, thr = 0, samp = 0, frows = 0, fpos = 0, fcnt = 0, diag = 0;
  size_t off_thr() const { return cand + cnt; }
  size_t off_samp() const { return off_thr() + thr; }
  size_t off_frows() const { return off_samp() + samp; }
  size_t off_fpos() const { return off_frows() + frows; }
  size_t off_fcnt() const { return off_fpos() + fpos; }
  size_t off_diag() const { return off_fcnt() + fcnt; }
  size_t total() const { return off_diag() + diag; }
};

Layout make_layout(int64_t n_users, int64_t n_items, int w, int k) {
  Layout L{};
  L.main = make_plan(n_users, n_items, w, k);
  L.g = guess_for(n_items, k);
  L.cand = L.main.cand_bytes;
  L.cnt = L.main.cnt_bytes;
  if (L.g.S > 0) {
    L.sample = make_plan(n_users, L.g.S, w, L.g.ks);
    L.cand = L.cand > L.sample.cand_bytes ? L.cand : L.sample.cand_bytes;
    L.cnt = L.cnt > L.sample.cnt_bytes ? L.cnt : L.sample.cnt_bytes;
    L.thr = al256((size_t)L.main.n_users_pad * sizeof(float));
    L.samp = al256((size_t)L.g.S * w * 2);
    L.frows = al256((size_t)n_users * sizeof(int64_t));
    L.fpos = al256((size_t)n_users * sizeof(int64_t));
    L.fcnt = 256;
  }
  L.diag = diag_bytes();
  return L;
}

// Sample rows: out[i] = I[i * stride], 16 B per thread.
__global__ __launch_bounds__(256) void sample_rows_kernel(const uint4* __restrict__ I,
                                                          int64_t stride, int64_t S, int cpr,
                                                          uint4* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= S * cpr) return;
  const int64_t r = t / cpr, c = t % cpr;
  out[t] = I[r * stride * cpr + c];
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
  a.n_chunks = p.n_chunks;
  a.chunk_items = p.chunk_items;
  a.n_ublocks = p.n_ublocks;
  a.init_thr = nullptr;
  a.n_users_dev = nullptr;
  a.pos_map = nullptr;
  a.cand = (uint64_t*)ws;
  a.cnt = (int32_t*)(ws + L.cand);
  a.diag = (uint64_t*)(ws + L.off_diag());  // written only in DIAG builds
  const int fin_grid = (int)dr::ceil_div(n_users, 4);
  const int P = p_for(p.n_chunks * p.cap);

#define DR_SCAN_OR_FAIL(PLAN, ARGS, SEEDED)                                  \
  if (!launch_scan(PLAN, ARGS, dtype, w, SEEDED, s)) {                       \
    dr::set_error("dr_score_topk: internal plan error (no scan instance)"); \
    return DR_EUNSUPPORTED;                                                  \
  }
#define DR_BY_P(PP_EXPR, LAUNCH)                                           \
  switch (PP_EXPR) {                                                       \
    case 8: LAUNCH(8); break;                                              \
    case 16: LAUNCH(16); break;                                            \
    case 32: LAUNCH(32); break;                                            \
    default:                                                               \
      dr::set_error("dr_score_topk: internal plan error (candidate sort)"); \
      return DR_EUNSUPPORTED;                                              \
  }
#define DR_FIN(PP, POS, NDEV, FCNT)                                                             \
  hipLaunchKernelGGL((topk_finalize_kernel<PP>), dim3(fin_grid), dim3(256), 0, s, a.cand, a.cnt, \
                     p.n_chunks, p.cap, n_users, p.n_users_pad, k, excl_rowptr, excl_items,     \
                     out_scores, out_items, POS, NDEV, user_ids, FCNT, frows, fpos)

  if (L.g.S == 0) {
    DR_SCAN_OR_FAIL(p, a, false)
    DR_CHECK_LAUNCH();
    int64_t* frows = nullptr;
    int64_t* fpos = nullptr;
#define DR_FIN_PLAIN(PP) DR_FIN(PP, nullptr, nullptr, nullptr)
    DR_BY_P(P, DR_FIN_PLAIN)
#undef DR_FIN_PLAIN
    DR_CHECK_LAUNCH();
    return DR_OK;
  }

  // ---- guessed thresholds: sample scan -> thresholds -> seeded scan -> verify
  float* thr = (float*)(ws + L.off_thr());
  char* samp = ws + L.off_samp();
  int64_t* frows = (int64_t*)(ws + L.off_frows());
  int64_t* fpos = (int64_t*)(ws + L.off_fpos());
  int32_t* fcnt = (int32_t*)(ws + L.off_fcnt());
  DR_CHECK_HIP(hipMemsetAsync(fcnt, 0, sizeof(int32_t), s));
  {
    const int cpr = w / 8;  // 16-B chunks per row
    const int64_t n16 = L.g.S * cpr;
    hipLaunchKernelGGL(sample_rows_kernel, dim3((unsigned)dr::ceil_div(n16, 256)), dim3(256), 0, s,
                       (const uint4*)item_table, L.g.stride, L.g.S, cpr, (uint4*)samp);
    DR_CHECK_LAUNCH();
  }
  TopkArgs as = a;  // sample ids are sample rows: no exclusions, no item base
  as.I = samp;
  as.n_items = L.g.S;
  as.item_base = 0;
  as.k = L.g.ks;
  as.excl_rowptr = nullptr;
  as.excl_items = nullptr;
  as.n_chunks = L.sample.n_chunks;
  as.chunk_items = L.sample.chunk_items;
  DR_SCAN_OR_FAIL(L.sample, as, false)
  DR_CHECK_LAUNCH();
  const int thr_grid = (int)dr::ceil_div(p.n_users_pad, 4);
#define DR_THR(PP)                                                                              \
  hipLaunchKernelGGL((topk_threshold_kernel<PP>), dim3(thr_grid), dim3(256), 0, s, a.cand,       \
                     a.cnt, L.sample.n_chunks, L.sample.cap, n_users, p.n_users_pad, L.g.ks,      \
                     nullptr, nullptr, thr)
  DR_BY_P(p_for(L.sample.n_chunks * L.sample.cap), DR_THR)
#undef DR_THR
  DR_CHECK_LAUNCH();

  a.init_thr = thr;
  DR_SCAN_OR_FAIL(p, a, true)
  DR_CHECK_LAUNCH();
#define DR_FIN_VERIFY(PP) DR_FIN(PP, nullptr, nullptr, fcnt)
  DR_BY_P(P, DR_FIN_VERIFY)
#undef DR_FIN_VERIFY
  DR_CHECK_LAUNCH();

  // ---- rescan of the users whose guess was too high (usually none)
  TopkArgs af = a;
  af.init_thr = nullptr;
  af.user_ids = frows;
  af.pos_map = fpos;
  af.n_users_dev = fcnt;
  af.diag = nullptr;
  DR_SCAN_OR_FAIL(p, af, false)
  DR_CHECK_LAUNCH();
#define DR_FIN_RESCAN(PP) DR_FIN(PP, fpos, fcnt, nullptr)
  DR_BY_P(P, DR_FIN_RESCAN)
#undef DR_FIN_RESCAN
#undef DR_FIN
#undef DR_BY_P
#undef DR_SCAN_OR_FAIL
  DR_CHECK_LAUNCH();
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
