// Full-catalog user x item scoring with a fused top-K: the MI355X form of
// get_model_recommendations (reference divrec/train/utils.py:53-77), whose
// per-user loop scores every RankingDataset candidate (base_datasets.py:136-171)
// with MatrixFactorization.forward (matrix_factorization.py:26-28) and keeps
// candidates[argsort(scores, descending=True)][:k].
//
// Design:
//  * One 512-thread workgroup (8 waves, two per SIMD) owns UPWG = 8*NU_T*32
//    users (NU_T = 2 below d=256: 512 users) and streams a chunk of the
//    item catalog in 32-item tiles. A wave keeps the
//    bf16 embeddings of its NU_T*32 users resident in registers as MFMA B
//    fragments for the whole scan; item tiles go HBM -> LDS by LDS-DMA
//    (global_load_lds_dwordx4, double buffered, XOR-swizzled on the source
//    address so the A-fragment ds_read_b128s are conflict-free) and are shared
//    by all 8 waves. MFMAs of tile t+1 are issued ahead of tile t's epilogue,
//    and the two waves of a SIMD cover each other's epilogues.
//  * Scores come from v_mfma_f32_32x32x16_bf16 with items on the M (row) axis
//    and users on the N (column) axis: a lane then holds 16 scores of ONE user,
//    so the epilogue is a 16-way max and one compare against that user's
//    running threshold (the current k-th best score). Scores are never stored.
//  * Survivors (score > threshold; rare once the threshold is established:
//    ~k*ln(n/CAP) per user) are appended to a per-user candidate buffer of CAP
//    64-bit keys in global memory. When a buffer is nearly full the wave
//    "flushes" that user: load, drop excluded items, wave-wide bitonic sort,
//    keep the best k, raise the threshold to the k-th key's score.
//  * Keys encode (score desc, item asc) so the result is a deterministic total
//    order and any item partition (chunks, GPUs) merges bit-identically.
#include "common.h"

namespace {

using dr::bf16x8;
using dr::f32x16;

constexpr int kWaves = 8;  // two waves per SIMD: 256-register budget each
constexpr int kThreads = kWaves * 64;
constexpr int kTileItems = 32;

template <int D>
struct TileGeom {
  static constexpr int KSTEPS = D / 16;                     // MFMA k-steps per row
  static constexpr int CPR = D / 8;                         // 16-B chunks per row
  static constexpr int TILE_BYTES = kTileItems * D * 2;     // one 32-item tile
  static constexpr int TILE_CHUNKS = TILE_BYTES / 16;       // = glds lane-loads per tile
  static constexpr int RPB = (2 * D >= 256) ? 1 : 256 / (2 * D);  // rows per 256-B bank row
  static constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  // physical chunk = logical chunk ^ swz(row): spreads the 32 rows that one
  // A-fragment ds_read_b128 touches over distinct 16-B bank slots.
  __device__ static int swz(int r) { return (r / RPB) & SWM; }
};

template <int D>
struct NuT {  // user tiles (of 32) per wave: B fragments NU_T*KSTEPS*4 <= 64 VGPRs,
  // two accumulator sets (pipelined) 2*NU_T*16 <= 64 VGPRs
  static constexpr int value = (D >= 256) ? 1 : 2;
};

// Stage one 32-item tile [tile_row0, tile_row0+32) of the slice into LDS.
// LDS image is lane-linear (glds writes base + lane*16); the XOR swizzle is
// applied to the per-lane global source address (cdna_hip_programming.md §5.4
// rule 21). Rows past the slice end are clamped to the last row (masked later).
template <int D>
__device__ __forceinline__ void stage_tile(const __bf16* __restrict__ I, int64_t n_items,
                                           int64_t tile_row0, char* lds_tile) {
  using G = TileGeom<D>;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
#pragma unroll
  for (int j = 0; j < (G::TILE_CHUNKS + kThreads - 1) / kThreads; ++j) {
    const int wave_first = j * kThreads + wave * 64;  // wave-uniform
    if (wave_first < G::TILE_CHUNKS) {
      const int idx = wave_first + (tid & 63);
      const int r = idx / G::CPR;
      const int pc = idx % G::CPR;
      const int lc = pc ^ G::swz(r);
      int64_t row = tile_row0 + r;
      row = row < n_items ? row : n_items - 1;
      const __bf16* src = I + row * D + lc * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(lds_tile + wave_first * 16),
                                       16, 0, 0);
    }
  }
}

// Binary search of `item` in a sorted global list.
__device__ __forceinline__ bool sorted_contains(const int32_t* __restrict__ list, int n,
                                                int32_t item) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (list[mid] < item) lo = mid + 1; else hi = mid;
  }
  return lo < n && list[lo] == item;
}

__device__ __forceinline__ void wave_lds_sync() {
  // Order this wave's LDS writes before its later LDS reads (one wave only).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Bitonic sort, DESCENDING, of n (power of two, 64 <= n) 64-bit keys in this
// wave's LDS scratch. A compact loop (register-light) because it runs inside
// the MFMA kernel next to the resident user fragments.
__device__ __forceinline__ void wave_lds_sort_desc(uint64_t* s, int n) {
  const int lane = dr::lane_id();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int jl = __builtin_ctz(j);
      for (int p = lane; p < (n >> 1); p += 64) {
        const int i = ((p >> jl) << (jl + 1)) | (p & (j - 1));
        const uint64_t x = s[i], y = s[i + j];
        const bool desc = (i & k) == 0;
        if (desc ? (x < y) : (x > y)) {
          s[i] = y;
          s[i + j] = x;
        }
      }
      wave_lds_sync();
    }
  }
}

// Wave-cooperative flush of one user's candidate buffer (cnt keys).
//   final == false: compact to the best k in place; return new count/threshold.
//   final == true : write the best k to the output (decoded, or raw keys).
template <int CAP>
__device__ __forceinline__ void flush_user(uint64_t* __restrict__ buf, int cnt, int k,
                                           const int32_t* __restrict__ excl, int excl_n,
                                           uint64_t* __restrict__ lds, bool final,
                                           float* __restrict__ out_s, int32_t* __restrict__ out_i,
                                           uint64_t* __restrict__ out_keys, int* new_cnt,
                                           float* new_thr) {
  const int lane = dr::lane_id();
  int n = 64;
  while (n < cnt) n <<= 1;  // cnt <= CAP
  // The candidate stores came from this wave: wait for them to leave it and
  // read around this CU's L1 (sc1 loads) so no stale line is served.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int e = lane; e < n; e += 64) {
    uint64_t v = 0ull;
    if (e < cnt) {
      v = __hip_atomic_load(buf + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (excl_n > 0 && sorted_contains(excl, excl_n, (int32_t)dr::key_item(v))) v = 0ull;
    }
    lds[e] = v;
  }
  wave_lds_sync();
  wave_lds_sort_desc(lds, n);
  int total = 0;  // non-empty keys (sorted to the front)
  for (int e0 = 0; e0 < n; e0 += 64) total += __popcll(__ballot(lds[e0 + lane] != 0ull));
  if (!final) {
    const int keep = total < k ? total : k;
    for (int e = lane; e < keep; e += 64) buf[e] = lds[e];
    *new_cnt = keep;
    *new_thr = total >= k ? dr::key_score(lds[k - 1]) : -INFINITY;
  } else {
    for (int e = lane; e < k; e += 64) {
      const uint64_t v = e < n ? lds[e] : 0ull;
      if (out_keys) {
        out_keys[e] = v;
      } else {
        const bool empty = v == 0ull;
        out_s[e] = empty ? -INFINITY : dr::key_score(v);
        out_i[e] = empty ? -1 : (int32_t)dr::key_item(v);
      }
    }
  }
  wave_lds_sync();  // scratch is reused by the next flush
}

struct TopkArgs {
  const __bf16* U;
  const int64_t* user_ids;
  int64_t n_users;
  const __bf16* I;
  int64_t n_items;
  int64_t item_base;
  int k;
  const int64_t* excl_rowptr;
  const int32_t* excl_items;
  int n_chunks;
  int64_t chunk_items;  // multiple of kTileItems
  int64_t n_ublocks;
  uint64_t* cand;   // [gridDim.x][UPWG][CAP]
  uint64_t* part;   // [n_chunks][n_users][k] when n_chunks > 1
  float* out_s;
  int32_t* out_i;
};

template <int D, int CAP>
__global__ __launch_bounds__(kThreads, 2) void score_topk_kernel(TopkArgs a) {
  using G = TileGeom<D>;
  constexpr int NU_T = NuT<D>::value;
  constexpr int KS = G::KSTEPS;
  constexpr int UPW = NU_T * 32;        // users per wave
  constexpr int UPWG = UPW * kWaves;    // users per workgroup
  __shared__ __attribute__((aligned(16))) char smem[2 * G::TILE_BYTES + kWaves * CAP * 8];
  char* tiles = smem;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int col = lane & 31;
  uint64_t* lds_sort = reinterpret_cast<uint64_t*>(smem + 2 * G::TILE_BYTES) + wave * CAP;
  uint64_t* cand_wave = a.cand + ((size_t)blockIdx.x * UPWG + (size_t)wave * UPW) * CAP;
  // Byte offset of this lane's A-fragment chunk for k-step 0 inside a tile;
  // k-step s reads chunk (2s + h) ^ swz(col).
  const int a_row_off = col * (2 * D);
  const int a_swz = G::swz(col);

  const int64_t n_units = a.n_ublocks * a.n_chunks;
  for (int64_t unit = blockIdx.x; unit < n_units; unit += gridDim.x) {
    const int64_t chunk = unit / a.n_ublocks;
    const int64_t ub = unit % a.n_ublocks;
    const int64_t i_beg = chunk * a.chunk_items;
    int64_t i_end = i_beg + a.chunk_items;
    i_end = i_end < a.n_items ? i_end : a.n_items;
    const int ntiles = (int)((i_end - i_beg + kTileItems - 1) / kTileItems);
    const int64_t upos0 = ub * UPWG + (int64_t)wave * UPW;  // first user position of the wave

    // Resident B fragments: lane holds user (ut*32+col), k = 16s + 8h .. +7.
    bf16x8 bfr[NU_T][KS];
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) {
      const int64_t pos = upos0 + ut * 32 + col;
      int64_t row = 0;
      if (pos < a.n_users) row = a.user_ids ? a.user_ids[pos] : pos;
      const uint4* src = reinterpret_cast<const uint4*>(a.U + row * D + 8 * h);
#pragma unroll
      for (int s = 0; s < KS; ++s) bfr[ut][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
    }
    float thr[NU_T];
    int cnt[NU_T];
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) {
      thr[ut] = -INFINITY;
      cnt[ut] = 0;
    }

    // MFMA pass over one staged tile: acc[ut] = items(32) x users(32).
    auto mma_tile = [&](int t, f32x16 (&acc)[NU_T]) {
      const char* tb = tiles + (t & 1) * G::TILE_BYTES + a_row_off;
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) acc[ut] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 af =
            *reinterpret_cast<const bf16x8*>(tb + (((2 * s + h) ^ a_swz) << 4));
#pragma unroll
        for (int ut = 0; ut < NU_T; ++ut)
          acc[ut] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[ut][s], acc[ut], 0, 0, 0);
      }
    };

    // Hot half of the epilogue (branch-free, so it can interleave with the next
    // tile's MFMAs): per user tile, one lane-local 16-way max and a compare
    // with the running threshold. Returns a bit per user tile with any hit.
    auto any_hits = [&](f32x16 (&acc)[NU_T]) -> uint32_t {
      uint32_t bits = 0;
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        float m = acc[ut][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, acc[ut][r]);
        bits |= (__ballot(m > thr[ut]) != 0ull ? 1u : 0u) << ut;
      }
      return bits;
    };

    // Cold half: append survivors, then flush users that could overflow.
    auto insert_and_flush = [&](int t, f32x16 (&acc)[NU_T], uint32_t hit_bits) {
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid_rows = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        if (hit_bits & (1u << ut)) {
          uint32_t mask = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            mask |= ((acc[ut][r] > thr[ut]) && row < valid_rows ? 1u : 0u) << r;
          }
          const int cs = __popc(mask);
          const int co = __shfl_xor(cs, 32);
          int pos = cnt[ut] + (h ? co : 0);
          uint64_t* ubuf = cand_wave + (size_t)(ut * 32 + col) * CAP;
          const uint32_t gbase = (uint32_t)(a.item_base + tile0);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (mask & (1u << r)) {
              const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
              ubuf[pos] = dr::make_key(acc[ut][r], gbase + (uint32_t)row);
              ++pos;
            }
          }
          cnt[ut] += cs + co;
        }
      }
      // Flush users whose buffer could overflow on the next tile.
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        uint64_t need = __ballot(cnt[ut] + 32 > CAP) & 0xffffffffull;
        while (need) {
          const int c = __builtin_ctzll(need);
          need &= need - 1;
          const int ucnt = __builtin_amdgcn_readlane(cnt[ut], c);
          const int64_t upos = upos0 + ut * 32 + c;
          const int32_t* ex = nullptr;
          int exn = 0;
          if (a.excl_rowptr && upos < a.n_users) {
            const int64_t e0 = a.excl_rowptr[upos], e1 = a.excl_rowptr[upos + 1];
            ex = a.excl_items + e0;
            exn = (int)(e1 - e0);
          }
          int ncnt;
          float nthr;
          flush_user<CAP>(cand_wave + (size_t)(ut * 32 + c) * CAP, ucnt, a.k, ex, exn, lds_sort,
                          false, nullptr, nullptr, nullptr, &ncnt, &nthr);
          if (col == c) {
            cnt[ut] = ncnt;
            thr[ut] = nthr;
          }
        }
      }
    };

    // ------------------------------------------------------------ tile scan
    // Software pipeline: the MFMAs of tile t+1 are issued before the VALU
    // epilogue of tile t, so one wave per SIMD keeps the matrix pipe busy.
    // Barrier B_t (top of step t) guarantees tile t+1 has landed in LDS and
    // every wave has finished reading tile t, whose buffer then receives t+2.
    if (ntiles > 0) stage_tile<D>(a.I, a.n_items, i_beg, tiles);
    if (ntiles > 1) stage_tile<D>(a.I, a.n_items, i_beg + kTileItems, tiles + G::TILE_BYTES);
    __syncthreads();  // drains the LDS-DMA (vmcnt(0)) before any read
    f32x16 accA[NU_T], accB[NU_T];
    if (ntiles > 0) mma_tile(0, accA);
    auto step = [&](int t, f32x16 (&cur)[NU_T], f32x16 (&nxt)[NU_T]) {
      __syncthreads();  // B_t
      if (t + 2 < ntiles)
        stage_tile<D>(a.I, a.n_items, i_beg + (int64_t)(t + 2) * kTileItems,
                      tiles + (t & 1) * G::TILE_BYTES);
      uint32_t hit_bits;
      if (t + 1 < ntiles) {
        mma_tile(t + 1, nxt);
        hit_bits = any_hits(cur);
        // Interleave: per MFMA one or two VALU of the previous tile's epilogue.
#pragma unroll
        for (int i = 0; i < KS * NU_T; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
        }
      } else {
        hit_bits = any_hits(cur);
      }
      // Users fold the same bits through SGPRs: the branch is wave-uniform.
      hit_bits = __builtin_amdgcn_readfirstlane(hit_bits);
      // A flush can only become necessary after an insert.
      if (hit_bits != 0u) insert_and_flush(t, cur, hit_bits);
    };
    for (int t = 0; t < ntiles; t += 2) {
      step(t, accA, accB);
      if (t + 1 < ntiles) step(t + 1, accB, accA);
    }

    // ------------------------------------------------------------ final flush
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) {
      for (int c = 0; c < 32; ++c) {
        const int64_t upos = upos0 + ut * 32 + c;
        if (upos >= a.n_users) break;  // wave-uniform
        const int ucnt = __builtin_amdgcn_readlane(cnt[ut], c);
        const int32_t* ex = nullptr;
        int exn = 0;
        if (a.excl_rowptr) {
          const int64_t e0 = a.excl_rowptr[upos], e1 = a.excl_rowptr[upos + 1];
          ex = a.excl_items + e0;
          exn = (int)(e1 - e0);
        }
        uint64_t* okeys = a.n_chunks > 1 ? a.part + ((size_t)chunk * a.n_users + upos) * a.k
                                         : nullptr;
        flush_user<CAP>(cand_wave + (size_t)(ut * 32 + c) * CAP, ucnt, a.k, ex, exn, lds_sort,
                        true, a.out_s + upos * a.k, a.out_i + upos * a.k, okeys, nullptr,
                        nullptr);
      }
    }
    __syncthreads();  // LDS tiles are reused by the next unit
  }
}

// ------------------------------------------------------------------ merge
// One wave per user: gather parts*k_in keys, bitonic sort, keep k_out.
template <int P, bool FROM_KEYS>
__global__ __launch_bounds__(256) void topk_merge_kernel(const uint64_t* __restrict__ keys,
                                                         const float* __restrict__ in_s,
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
      const size_t off = ((size_t)p * n_users + u) * k_in + j;
      if (FROM_KEYS) {
        kk = keys[off];
      } else {
        const int32_t it = in_i[off];
        kk = it < 0 ? 0ull : dr::make_key(in_s[off], (uint32_t)it);
      }
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

template <bool FROM_KEYS>
int launch_merge(const uint64_t* keys, const float* in_s, const int32_t* in_i, int parts,
                 int64_t n_users, int k_in, int k_out, float* out_s, int32_t* out_i,
                 hipStream_t s) {
  const int total = parts * k_in;
  const int grid = (int)dr::ceil_div(n_users, 4);
#define DR_MERGE(PP)                                                                         \
  hipLaunchKernelGGL((topk_merge_kernel<PP, FROM_KEYS>), dim3(grid), dim3(256), 0, s, keys, \
                     in_s, in_i, parts, n_users, k_in, k_out, out_s, out_i)
  if (total <= 64 * 2) DR_MERGE(2);
  else if (total <= 64 * 4) DR_MERGE(4);
  else if (total <= 64 * 8) DR_MERGE(8);
  else if (total <= 64 * 16) DR_MERGE(16);
  else if (total <= 64 * 32) DR_MERGE(32);
  else {
    dr::set_error("topk merge: parts * k_in must be <= 2048");
    return DR_EUNSUPPORTED;
  }
#undef DR_MERGE
  return DR_OK;
}

// ------------------------------------------------------------------ planning
struct Plan {
  int cap;
  int users_per_wg;
  int64_t n_ublocks;
  int n_chunks;
  int64_t chunk_items;
  int grid;
  size_t cand_bytes;
  size_t part_bytes;
};

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return cus > 0 ? cus : 256;
}

int cap_for_k(int k) { return k <= 256 ? 1024 : 2048; }

Plan make_plan(int64_t n_users, int64_t n_items, int d, int k) {
  Plan p{};
  p.cap = cap_for_k(k);
  const int nut = d >= 256 ? 1 : 2;
  p.users_per_wg = nut * 32 * kWaves;
  p.n_ublocks = dr::ceil_div(n_users, p.users_per_wg);
  const int slots = device_cus();  // one 512-thread workgroup per CU
  // Split the catalog into chunks only to balance the tail of the grid; each
  // chunk must stay long enough to amortise its warm-up (first CAP inserts).
  const int64_t min_chunk = 16384;
  int best_s = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && n_items / s < min_chunk) break;
    if (s * k > 2048) break;  // merge capacity
    const int64_t units = p.n_ublocks * s;
    const int64_t rounds = dr::ceil_div(units, slots);
    const double eff = (double)units / (double)(rounds * slots);
    if (eff > best_eff + 0.02) {
      best_eff = eff;
      best_s = s;
    }
  }
  p.n_chunks = best_s;
  p.chunk_items = dr::ceil_div(dr::ceil_div(n_items, best_s), kTileItems) * kTileItems;
  const int64_t units = p.n_ublocks * p.n_chunks;
  p.grid = (int)(units < slots ? units : slots);
  p.cand_bytes = (size_t)p.grid * p.users_per_wg * p.cap * sizeof(uint64_t);
  p.part_bytes = p.n_chunks > 1 ? (size_t)p.n_chunks * n_users * k * sizeof(uint64_t) : 0;
  return p;
}

}  // namespace

extern "C" size_t dr_score_topk_workspace(int64_t n_users, int64_t n_items, int d, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  Plan p = make_plan(n_users, n_items, d, k);
  return p.cand_bytes + p.part_bytes + 256;
}

extern "C" int dr_score_topk(const void* user_table, const int64_t* user_ids, int64_t n_users,
                             const void* item_table, int64_t n_items, int64_t item_base, int d,
                             int k, const int64_t* excl_rowptr, const int32_t* excl_items,
                             float* out_scores, int32_t* out_items, void* workspace,
                             size_t workspace_bytes, dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_items >= 0, "negative size");
  DR_CHECK_ARG(k >= 1 && k <= 1024, "k must be in [1, 1024]");
  DR_CHECK_ARG(d == 32 || d == 64 || d == 128 || d == 256,
               "d must be one of 32, 64, 128, 256");
  DR_CHECK_ARG(item_base >= 0 && item_base + n_items < 0x7fffffffLL,
               "global item ids must fit int32");
  DR_CHECK_ARG((excl_rowptr == nullptr) == (excl_items == nullptr),
               "excl_rowptr and excl_items must both be set or both be NULL");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(user_table && out_scores && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (n_items == 0) {
    // No candidates at all: every slot is empty.
    dr::set_error("dr_score_topk: empty catalog");
    return DR_EINVAL;
  }
  DR_CHECK_ARG(item_table, "null item_table");
  Plan p = make_plan(n_users, n_items, d, k);
  const size_t need = p.cand_bytes + p.part_bytes;
  if (!workspace || workspace_bytes < need) {
    dr::set_error("dr_score_topk: workspace too small (need " + std::to_string(need) +
                  " bytes)");
    return DR_EWORKSPACE;
  }
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if ((size_t)(ws - (char*)workspace) + need > workspace_bytes) {
    dr::set_error("dr_score_topk: workspace too small after alignment");
    return DR_EWORKSPACE;
  }
  TopkArgs a;
  a.U = (const __bf16*)user_table;
  a.user_ids = user_ids;
  a.n_users = n_users;
  a.I = (const __bf16*)item_table;
  a.n_items = n_items;
  a.item_base = item_base;
  a.k = k;
  a.excl_rowptr = excl_rowptr;
  a.excl_items = excl_items;
  a.n_chunks = p.n_chunks;
  a.chunk_items = p.chunk_items;
  a.n_ublocks = p.n_ublocks;
  a.cand = (uint64_t*)ws;
  a.part = p.part_bytes ? (uint64_t*)(ws + p.cand_bytes) : nullptr;
  a.out_s = out_scores;
  a.out_i = out_items;

#define DR_TOPK(DD, CC) \
  hipLaunchKernelGGL((score_topk_kernel<DD, CC>), dim3(p.grid), dim3(kThreads), 0, s, a)
  if (p.cap == 1024) {
    switch (d) {
      case 32: DR_TOPK(32, 1024); break;
      case 64: DR_TOPK(64, 1024); break;
      case 128: DR_TOPK(128, 1024); break;
      default: DR_TOPK(256, 1024); break;
    }
  } else {
    switch (d) {
      case 32: DR_TOPK(32, 2048); break;
      case 64: DR_TOPK(64, 2048); break;
      case 128: DR_TOPK(128, 2048); break;
      default: DR_TOPK(256, 2048); break;
    }
  }
#undef DR_TOPK
  DR_CHECK_LAUNCH();
  if (p.n_chunks > 1) {
    int rc = launch_merge<true>(a.part, nullptr, nullptr, p.n_chunks, n_users, k, k, out_scores,
                                out_items, s);
    if (rc != DR_OK) return rc;
    DR_CHECK_LAUNCH();
  }
  return DR_OK;
}

extern "C" int dr_topk_merge(const float* in_scores, const int32_t* in_items, int parts,
                             int64_t n_users, int k_in, int k_out, float* out_scores,
                             int32_t* out_items, dr_stream_t stream) {
  DR_CHECK_ARG(parts >= 1 && k_in >= 1 && k_out >= 1, "parts, k_in, k_out must be >= 1");
  DR_CHECK_ARG(k_out <= parts * k_in, "k_out must be <= parts * k_in");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(in_scores && in_items && out_scores && out_items, "null pointer");
  int rc = launch_merge<false>(nullptr, in_scores, in_items, parts, n_users, k_in, k_out,
                               out_scores, out_items, (hipStream_t)stream);
  if (rc != DR_OK) return rc;
  DR_CHECK_LAUNCH();
  return DR_OK;
}
