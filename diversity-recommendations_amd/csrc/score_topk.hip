// Full-catalog user x item scoring with a fused top-K: the MI355X form of
// get_model_recommendations (reference divrec/train/utils.py:53-77), whose
// per-user loop scores every RankingDataset candidate (base_datasets.py:136-171)
// with MatrixFactorization.forward (matrix_factorization.py:26-28) and keeps
// candidates[argsort(scores, descending=True)][:k].
//
// Two kernels:
//
// score_scan_kernel — one 512-thread workgroup (8 waves, two per SIMD) owns
//   UPWG = 8*NU_T*32 users and streams one chunk of the item catalog.
//   * Each wave keeps the bf16 embeddings of its NU_T*32 users resident in
//     registers as MFMA B fragments for the whole scan.
//   * Item rows go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) into a ring
//     of 16-KB stages filled kRing-1 stages ahead; the LDS image is
//     XOR-swizzled through the per-lane source address so the A-fragment
//     ds_read_b128s are bank-conflict-free. All 8 waves share every stage.
//   * v_mfma_f32_32x32x16_bf16 puts items on M and users on N, so a lane holds
//     16 scores of ONE user: the hot epilogue is a 16-way max and one compare
//     with that user's running threshold. Scores never leave registers. The
//     two waves of a SIMD cover each other's epilogues.
//   * Survivors (rare once thresholds settle) go to a per-wave LDS queue; the
//     queue is drained in batches into per-user candidate buffers in HBM. When
//     a buffer nears capacity the wave compacts it with an in-register radix
//     select, keeping only keys that can still reach the top k, and raises the
//     user's threshold to the selected bound.
//   * All VMEM traffic inside the scan (LDS-DMA and candidate stores) is
//     issued from inline asm and counted by the wave, so each stage wait is an
//     exact s_waitcnt vmcnt(N): no drain of the ring.
// topk_finalize_kernel — one wave per user: gather the candidates of all
//   chunks, drop excluded items, bitonic sort, write the k best.
//
// Keys encode (score desc, item asc) as one 64-bit unsigned order, so the
// result is a deterministic total order and any item partition (chunks,
// GPUs) gives bit-identical top-k lists.
#include "common.h"

namespace {

using dr::bf16x8;
using dr::f32x16;

// Diagnostic build (-DDR_TOPK_DIAG, libdivrec_hip_diag.so only): per-wave
// s_memtime cycle counters of each phase of the scan, written to the tail of
// the workspace. Never compiled into the product library.
#ifdef DR_TOPK_DIAG
#define DG_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define DG_ADD(slot, t0) dg[slot] += __builtin_amdgcn_s_memtime() - (t0)
#define DG_CNT(slot) dg[slot] += 1
#else
#define DG_T0(v) ((void)0)
#define DG_ADD(slot, t0) ((void)0)
#define DG_CNT(slot) ((void)0)
#endif
enum {
  kDgTotal, kDgPrologue, kDgBoundary, kDgMma, kDgHits, kDgEnqueue, kDgDrain, kDgFlush,
  kDgNTiles, kDgNEnqueue, kDgNDrain, kDgNFlush, kDgNStages, kDgSlots = 16
};

constexpr int kWaves = 8;  // two waves per SIMD: 256-register budget each
constexpr int kThreads = kWaves * 64;
constexpr int kTileItems = 32;
constexpr int kStageBytes = 16384;                  // one LDS ring slot
constexpr int kLpt = kStageBytes / 16 / kThreads;  // LDS-DMA per thread per stage (= 2)
constexpr int kRing = 4;                            // stages resident / in flight
constexpr int kQcap = 512;                          // per-wave survivor queue (entries)
constexpr int kSlack = 32;                          // keys kept beyond k by a compaction

template <int D>
struct TileGeom {
  static constexpr int KSTEPS = D / 16;                 // MFMA k-steps per row
  static constexpr int CPR = D / 8;                     // 16-B chunks per row
  static constexpr int TILE_BYTES = kTileItems * D * 2;
  static constexpr int SR = kStageBytes / TILE_BYTES;   // row tiles per stage
  static constexpr int RPB = (2 * D >= 256) ? 1 : 256 / (2 * D);  // rows per 256-B bank row
  static constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  static constexpr int MARGIN = SR * kTileItems;  // max new keys per user per stage
  // physical chunk = logical chunk ^ swz(row): spreads the 32 rows that one
  // A-fragment ds_read_b128 touches over distinct 16-B bank slots.
  __device__ static int swz(int r) { return (r / RPB) & SWM; }
};

template <int D>
struct NuT {  // user tiles (of 32) per wave: B fragments NU_T*KSTEPS*4 <= 64 VGPRs
  static constexpr int value = (D >= 256) ? 1 : 2;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ asm VMEM
// The scan issues its VMEM traffic from inline asm so that hipcc does not put
// its own conservative s_waitcnt vmcnt(0) in front of the MFMAs (it cannot
// prove a C++ ds_read does not alias an in-flight LDS-DMA); the wave counts
// every instruction it issues and waits with exact counts. M0 is used by no
// other code in the kernel.
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_wave_base);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(m0)
               : "memory", "m0");
#pragma clang diagnostic pop
}
__device__ __forceinline__ void st64(uint64_t* p, uint64_t v) {
  asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(p), "v"(v) : "memory");
}
// A store of more than 64 data bits reads its data VGPRs after issue: the
// trailing s_nop 1 keeps hipcc's next instruction from overwriting them first.
__device__ __forceinline__ void st128(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 ds_read_b128_asm(uint32_t lds_addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr));
  return v;
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their maxima).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {  // n is wave-uniform
  if constexpr (N == 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else wait_vmcnt_le<N - 1>(n);
  }
}
// Wait until at most n (wave-uniform) VMEM ops are outstanding; n >= 63
// saturates at 63, which waits for more than required (still correct).
__device__ __forceinline__ void wait_vmcnt_dyn(int n) { wait_vmcnt_le<63>(n); }

// Issue the LDS-DMA of one stage: rows [row0, row0 + SR*32) of the slice into
// the ring slot at LDS byte address `lds_stage`. The image is lane-linear
// (glds writes base + lane*16); the swizzle is on the SOURCE address
// (cdna_hip_programming.md §5.4 rule 21). Rows past the slice end are
// clamped to its last row; their scores are masked in the epilogue.
template <int D>
__device__ __forceinline__ void issue_stage(const __bf16* __restrict__ I, int64_t n_items,
                                            int64_t row0, uint32_t lds_stage) {
  using G = TileGeom<D>;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
#pragma unroll
  for (int j = 0; j < kLpt; ++j) {
    const int wave_first = j * kThreads + wave * 64;  // wave-uniform chunk index
    const int idx = wave_first + (tid & 63);
    const int r = idx / G::CPR;
    const int pc = idx % G::CPR;
    const int lc = pc ^ G::swz(r & 31);
    int64_t row = row0 + r;
    row = row < n_items ? row : n_items - 1;
    glds16(I + row * D + lc * 8, lds_stage + wave_first * 16);
  }
}

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
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_prefix(uint64_t bal) {  // set bits of bal below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

struct CompactResult {
  int kept;
  float thr;
};

// Compaction of one candidate buffer (cold path, out of line so its registers
// do not raise the pressure of the MFMA loop). Keeps only the keys that can
// still be in the top k: radix select (8 bits per level, wave-wide LDS
// histogram) down to the bucket holding the k-th largest key, until at most
// k + kSlack keys remain at or above the bucket's lower bound. The bound's
// score is the new threshold: >= k kept keys rank above any later item of
// equal or lower score. Excluded items are dropped first.
template <int P>
__device__ __noinline__ CompactResult compact_buffer(uint64_t* __restrict__ buf, int n_in, int k,
                                                     const int32_t* __restrict__ ex, int exn,
                                                     uint32_t* __restrict__ hist) {
  const int lane = dr::lane_id();
  wait_vmcnt<0>();  // this wave's candidate stores have landed
  uint64_t key[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    key[i] = e < n_in ? __hip_atomic_load(buf + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : 0ull;
  }
  if (exn > 0) {
#pragma unroll
    for (int i = 0; i < P; ++i)
      if (key[i] != 0ull && sorted_contains(ex, exn, (int32_t)dr::key_item(key[i])))
        key[i] = 0ull;
  }
  int total = 0;
#pragma unroll
  for (int i = 0; i < P; ++i) total += __popcll(__ballot(key[i] != 0ull));
  uint64_t lo = 1ull;  // keep keys >= lo (key 0 = empty slot)
  CompactResult res{total, -INFINITY};
  if (total > k + kSlack) {
    uint64_t pfx = 0ull;
    int need = k, above = 0, inb = total;
    for (int shift = 56; shift >= 0; shift -= 8) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hist[lane * 4 + j] = 0u;
      wave_lds_sync();
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const bool in = key[i] != 0ull &&
                        (shift == 56 || (key[i] >> (shift + 8)) == (pfx >> (shift + 8)));
        if (in) atomicAdd(&hist[(uint32_t)(key[i] >> shift) & 255u], 1u);
      }
      wave_lds_sync();
      uint32_t hv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[j] = hist[lane * 4 + j];
      const uint32_t s4 = hv[0] + hv[1] + hv[2] + hv[3];
      uint32_t sfx = s4;  // inclusive suffix sum over lanes >= this lane
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
        const uint32_t o = __shfl_down(sfx, m);
        sfx += (lane + m < 64) ? o : 0u;
      }
      // this lane's bins from the top (4l+3 .. 4l): the one holding rank `need`
      uint32_t cum = sfx - s4;  // keys in bins above 4l+3
      int fb = -1;
      uint32_t fexcl = 0, fcnt = 0;
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        const uint32_t nx = cum + hv[j];
        if (fb < 0 && cum < (uint32_t)need && (uint32_t)need <= nx) {
          fb = lane * 4 + j;
          fexcl = cum;
          fcnt = hv[j];
        }
        cum = nx;
      }
      const int src = __builtin_ctzll(__ballot(fb >= 0));
      const int b = __builtin_amdgcn_readlane(fb, src);
      const int excl = __builtin_amdgcn_readlane((int)fexcl, src);
      inb = __builtin_amdgcn_readlane((int)fcnt, src);
      pfx |= (uint64_t)b << shift;
      need -= excl;
      above += excl;
      wave_lds_sync();  // hist is re-zeroed by the next level
      if (above + inb <= k + kSlack) break;
    }
    lo = pfx;
    res.kept = above + inb;
    res.thr = dr::key_score(pfx);                // smallest score with the kept prefix
    if (res.thr != res.thr) res.thr = -INFINITY;  // prefix below -FLT_MAX decodes to NaN
  }
  // write the kept keys back densely (order is irrelevant)
  int base = 0;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const bool keep = key[i] >= lo;  // lo >= 1 also drops empty keys
    const uint64_t bal = __ballot(keep);
    if (keep) buf[base + lane_prefix(bal)] = key[i];
    base += __popcll(bal);
  }
  wait_vmcnt<0>();
  return res;
}

// Drain a wave's survivor queue into the per-user candidate buffers (cold
// path). Returns the number of store instructions issued (one per 64 entries).
__device__ __noinline__ int drain_queue(const uint64_t* __restrict__ qkey,
                                        const uint32_t* __restrict__ qslot,
                                        uint32_t* __restrict__ ucnt, int qlen,
                                        uint64_t* __restrict__ cbase, int cap) {
  const int lane = dr::lane_id();
  wave_lds_sync();
  int n = 0;
  for (int b0 = 0; b0 < qlen; b0 += 64) {
    const int i = b0 + lane;
    if (i < qlen) {
      const uint64_t key = qkey[i];
      const uint32_t slot = qslot[i];
      const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
      st64(cbase + (size_t)slot * cap + pos, key);
    }
    ++n;
  }
  wave_lds_sync();
  return n;
}

struct TopkArgs {
  const __bf16* U;
  const int64_t* user_ids;
  int64_t n_users;
  int64_t n_users_pad;  // n_ublocks * UPWG: candidate buffers exist for padded users too
  const __bf16* I;
  int64_t n_items;
  int64_t item_base;
  int k;
  const int64_t* excl_rowptr;
  const int32_t* excl_items;
  int n_chunks;
  int64_t chunk_items;  // multiple of the stage's item count
  int64_t n_ublocks;
  uint64_t* cand;  // [n_chunks][n_users_pad][CAP] keys (unsorted)
  int32_t* cnt;    // [n_chunks][n_users_pad] valid keys per buffer
  uint64_t* diag;  // [gridDim.x * kWaves][kDgSlots] in DR_TOPK_DIAG builds
};

template <int D, int CAP>
__global__ __launch_bounds__(kThreads, 2) void score_scan_kernel(TopkArgs a) {
  using G = TileGeom<D>;
  constexpr int NU_T = NuT<D>::value;
  constexpr int KS = G::KSTEPS;
  constexpr int SR = G::SR;
  constexpr int UPW = NU_T * 32;      // users per wave
  constexpr int UPWG = UPW * kWaves;  // users per workgroup
  constexpr int FLUSH_AT = CAP - G::MARGIN;        // compact when a buffer holds more
  constexpr int WARM = FLUSH_AT / kTileItems;      // warm-up tiles written without a test
  constexpr int P = CAP / 64;                      // keys per lane in a compaction
  constexpr int RING_BYTES = kRing * kStageBytes;
  constexpr int WAVE_BYTES = kQcap * 8 + kQcap * 4 + UPW * 4 + 256 * 4;
  static_assert(RING_BYTES + kWaves * WAVE_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[RING_BYTES + kWaves * WAVE_BYTES];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int col = lane & 31;
  char* wbase = smem + RING_BYTES + wave * WAVE_BYTES;
  uint64_t* qkey = reinterpret_cast<uint64_t*>(wbase);
  uint32_t* qslot = reinterpret_cast<uint32_t*>(wbase + kQcap * 8);
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(wbase + kQcap * 12);
  uint32_t* hist = reinterpret_cast<uint32_t*>(wbase + kQcap * 12 + UPW * 4);
  const uint32_t lds_ring = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  uint32_t a_off[KS];  // this lane's A-fragment byte offset for k-step s in a tile
#pragma unroll
  for (int s = 0; s < KS; ++s)
    a_off[s] = (uint32_t)(col * (2 * D) + (((2 * s + h) ^ G::swz(col)) << 4));

#ifdef DR_TOPK_DIAG
  uint64_t dg[kDgSlots] = {};
  DG_T0(t_kernel);
#endif
  const int64_t n_units = a.n_ublocks * a.n_chunks;
  for (int64_t unit = blockIdx.x; unit < n_units; unit += gridDim.x) {
    DG_T0(t_pro);
    const int64_t chunk = unit / a.n_ublocks;
    const int64_t ub = unit % a.n_ublocks;
    const int64_t i_beg = chunk * a.chunk_items;
    int64_t i_end = i_beg + a.chunk_items;
    i_end = i_end < a.n_items ? i_end : a.n_items;
    const int ntiles = i_end > i_beg ? (int)((i_end - i_beg + kTileItems - 1) / kTileItems) : 0;
    const int nst = (ntiles + SR - 1) / SR;
    const int64_t upos0 = ub * UPWG + (int64_t)wave * UPW;  // first user position of the wave
    uint64_t* cbase = a.cand + ((size_t)chunk * a.n_users_pad + upos0) * CAP;

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
    // Retire those loads where the compiler can see it (else it waits for them
    // inside the loop, draining the ring).
    wait_vmcnt<0>();
    for (int s = lane; s < UPW; s += 64) ucnt[s] = 0;
    float thr[NU_T];
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) thr[ut] = -INFINITY;
    int qlen = 0;       // survivor queue length (wave-uniform)
    int vmc = 0;        // VMEM instructions issued by this wave in this unit
    int vm_done = 0;    // every op issued before this count has completed
    int vs[kRing - 1];  // vmc right after each outstanding stage's DMA
#pragma unroll
    for (int i = 0; i < kRing - 1; ++i) vs[i] = 0;
    DG_ADD(kDgPrologue, t_pro);

    // -------------------------------------------------------------- MFMA tile
    auto mma_tile = [&](int t, f32x16 (&acc)[NU_T]) {
      const uint32_t tb = lds_ring + ((t / SR) % kRing) * kStageBytes + (t % SR) * G::TILE_BYTES;
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) acc[ut] = f32x16{};
      constexpr int HALF = KS >= 4 ? KS / 2 : KS;
#pragma unroll
      for (int s0 = 0; s0 < KS; s0 += HALF) {
        u32x4 af[HALF];
#pragma unroll
        for (int s = 0; s < HALF; ++s) af[s] = ds_read_b128_asm(tb + a_off[s0 + s]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < HALF; ++s)
#pragma unroll
          for (int ut = 0; ut < NU_T; ++ut)
            acc[ut] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf16x8, af[s]), bfr[ut][s0 + s], acc[ut], 0, 0, 0);
      }
    };

    // -------------------------------------------------------------- cold paths
    auto compact = [&](int ut, int c, int n_in) {
      DG_T0(t_f);
      const int slot = ut * 32 + c;
      const int64_t upos = upos0 + slot;
      const int32_t* ex = nullptr;
      int exn = 0;
      if (a.excl_rowptr && upos < a.n_users) {
        const int64_t e0 = a.excl_rowptr[upos], e1 = a.excl_rowptr[upos + 1];
        ex = a.excl_items + e0;
        exn = (int)(e1 - e0);
      }
      const CompactResult r = compact_buffer<P>(cbase + (size_t)slot * CAP, n_in, a.k, ex, exn, hist);
      vm_done = vmc;
      if (lane == 0) ucnt[slot] = (uint32_t)r.kept;
      wave_lds_sync();
#pragma unroll
      for (int u2 = 0; u2 < NU_T; ++u2)
        if (u2 == ut && col == c) thr[u2] = r.thr;
      DG_ADD(kDgFlush, t_f);
      DG_CNT(kDgNFlush);
    };

    auto drain = [&]() {
      DG_T0(t_d);
      vmc += drain_queue(qkey, qslot, ucnt, qlen, cbase, CAP);
      qlen = 0;
      DG_ADD(kDgDrain, t_d);
      DG_CNT(kDgNDrain);
    };

    auto check_compact = [&]() {
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        const uint32_t c_cnt = ucnt[ut * 32 + col];
        uint64_t need = __ballot(c_cnt > (uint32_t)FLUSH_AT) & 0xffffffffull;
        while (need) {
          const int c = __builtin_ctzll(need);
          need &= need - 1;
          compact(ut, c, __builtin_amdgcn_readlane((int)c_cnt, c));
        }
      }
    };

    // -------------------------------------------------------------- epilogues
    // Warm-up: the first WARM tiles are written to the buffers unconditionally
    // (position = item offset), then every buffer is compacted once.
    auto warm_fill = [&](int t, f32x16 (&acc)[NU_T]) {
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        uint64_t* dst = cbase + (size_t)(ut * 32 + col) * CAP + t * kTileItems;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint64_t kk[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = 8 * g + 4 * h + j;
            kk[j] = row < valid ? dr::make_key(acc[ut][4 * g + j], gbase + (uint32_t)row) : 0ull;
          }
          uint64_t* p = dst + 8 * g + 4 * h;
          st128(p, u32x4{(uint32_t)kk[0], (uint32_t)(kk[0] >> 32), (uint32_t)kk[1],
                         (uint32_t)(kk[1] >> 32)});
          st128(p + 2, u32x4{(uint32_t)kk[2], (uint32_t)(kk[2] >> 32), (uint32_t)kk[3],
                             (uint32_t)(kk[3] >> 32)});
          vmc += 2;
        }
      }
      if (t == WARM - 1 || t == ntiles - 1) {
        const int n_in = (t + 1) * kTileItems;
        for (int s = lane; s < UPW; s += 64) ucnt[s] = (uint32_t)n_in;
        wave_lds_sync();
#pragma unroll
        for (int ut = 0; ut < NU_T; ++ut)
          for (int c = 0; c < 32; ++c) compact(ut, c, n_in);
      }
    };

    // Hot test (branch-free): per user tile, a 16-way max against the threshold.
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

    // Append survivors to the LDS queue: one key per lane per round.
    auto enqueue = [&](int t, f32x16 (&acc)[NU_T], uint32_t hit_bits) {
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        if (!(hit_bits & (1u << ut))) continue;
        uint32_t mask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          mask |= ((acc[ut][r] > thr[ut]) && row < valid ? 1u : 0u) << r;
        }
        while (true) {
          const uint64_t act = __ballot(mask != 0u);
          if (act == 0ull) break;
          if (qlen > kQcap - 64) drain();
          const bool has = mask != 0u;
          const int r = has ? __builtin_ctz(mask) : 0;
          mask &= mask - 1u;
          float v = acc[ut][0];
#pragma unroll
          for (int q = 1; q < 16; ++q) v = (r == q) ? acc[ut][q] : v;
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int pos = qlen + lane_prefix(act);
          if (has) {
            qkey[pos] = dr::make_key(v, gbase + (uint32_t)row);
            qslot[pos] = (uint32_t)(ut * 32 + col);
          }
          qlen += __popcll(act);
        }
      }
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };

    // -------------------------------------------------------------- tile scan
    // Stage boundary s: wait (exact count) for this wave's DMA of stage s, a
    // raw barrier publishes the whole stage, then stage s+kRing-1 is issued
    // into the slot of stage s-1, which every wave finished reading.
    auto boundary = [&](int st) {
      DG_T0(t_b);
      if (vs[0] > vm_done) wait_vmcnt_dyn(vmc - vs[0]);
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int i = 0; i + 1 < kRing - 1; ++i) vs[i] = vs[i + 1];
      if (st + kRing - 1 < nst) {
        issue_stage<D>(a.I, a.n_items, i_beg + (int64_t)(st + kRing - 1) * SR * kTileItems,
                       lds_ring + ((st + kRing - 1) % kRing) * kStageBytes);
        vmc += kLpt;
      }
      vs[kRing - 2] = vmc;
      DG_ADD(kDgBoundary, t_b);
      DG_CNT(kDgNStages);
    };
    for (int st = 0; st < kRing - 1 && st < nst; ++st) {
      issue_stage<D>(a.I, a.n_items, i_beg + (int64_t)st * SR * kTileItems,
                     lds_ring + st * kStageBytes);
      vmc += kLpt;
#pragma unroll
      for (int i = 0; i < kRing - 1; ++i)
        if (i == st) vs[i] = vmc;
    }
    auto epilogue = [&](int t, f32x16 (&acc)[NU_T]) {
      if (t < WARM) {
        warm_fill(t, acc);
      } else {
        DG_T0(t_h);
        uint32_t hit_bits = any_hits(acc);
        DG_ADD(kDgHits, t_h);
        hit_bits = __builtin_amdgcn_readfirstlane(hit_bits);  // ballots: uniform
        if (hit_bits != 0u) enqueue(t, acc, hit_bits);
        // end of a stage: publish the survivors and compact full buffers
        if ((t + 1) % SR == 0 || t + 1 == ntiles) {
          if (qlen > 0) drain();
          check_compact();
        }
      }
    };
    // One accumulator set: the partner wave on the same SIMD issues its MFMAs
    // while this wave runs the epilogue (two waves per SIMD by design).
    f32x16 acc[NU_T];
    for (int t = 0; t < ntiles; ++t) {
      DG_CNT(kDgNTiles);
      if (t % SR == 0) boundary(t / SR);
      DG_T0(t_m);
      mma_tile(t, acc);
      DG_ADD(kDgMma, t_m);
      epilogue(t, acc);
    }
    if (qlen > 0) drain();
    wait_vmcnt<0>();
    wave_lds_sync();
    for (int s = lane; s < UPW; s += 64)
      a.cnt[(size_t)chunk * a.n_users_pad + upos0 + s] = (int32_t)ucnt[s];
    __syncthreads();  // the ring is refilled by the next unit
  }
#ifdef DR_TOPK_DIAG
  DG_ADD(kDgTotal, t_kernel);
  if (lane == 0) {
    uint64_t* o = a.diag + ((size_t)blockIdx.x * kWaves + wave) * kDgSlots;
#pragma unroll
    for (int i = 0; i < kDgSlots; ++i) o[i] = dg[i];
  }
#endif
}

// ------------------------------------------------------------------ finalize
// One wave per user: all chunks' candidate keys -> drop excluded items ->
// wave-wide register bitonic sort -> k best, decoded.
template <int P>
__global__ __launch_bounds__(256) void topk_finalize_kernel(
    const uint64_t* __restrict__ cand, const int32_t* __restrict__ cnt, int n_chunks, int cap,
    int64_t n_users, int64_t n_users_pad, int k, const int64_t* __restrict__ excl_rowptr,
    const int32_t* __restrict__ excl_items, float* __restrict__ out_s,
    int32_t* __restrict__ out_i) {
  const int lane = dr::lane_id();
  const int64_t u = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (u >= n_users) return;  // wave-uniform
  int off[9];
  off[0] = 0;
  for (int c = 0; c < 8; ++c)
    off[c + 1] = off[c] + (c < n_chunks ? cnt[(size_t)c * n_users_pad + u] : 0);
  const int total = off[8];
  uint64_t key[P];
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
  if (excl_rowptr) {
    const int64_t e0 = excl_rowptr[u], e1 = excl_rowptr[u + 1];
#pragma unroll
    for (int i = 0; i < P; ++i)
      if (key[i] != 0ull &&
          sorted_contains(excl_items + e0, (int)(e1 - e0), (int32_t)dr::key_item(key[i])))
        key[i] = 0ull;
  }
  dr::wave_sort_desc<P>(key);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int e = lane * P + i;
    if (e < k) {
      const bool empty = key[i] == 0ull;
      out_s[u * k + e] = empty ? -INFINITY : dr::key_score(key[i]);
      out_i[u * k + e] = empty ? -1 : (int32_t)dr::key_item(key[i]);
    }
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
struct Plan {
  int cap;
  int users_per_wg;
  int64_t n_ublocks;
  int64_t n_users_pad;
  int n_chunks;
  int64_t chunk_items;
  int grid;
  size_t cand_bytes;
  size_t cnt_bytes;
};

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return cus > 0 ? cus : 256;
}

// Smallest candidate capacity that still has a quarter of its compaction
// threshold free after a compaction to k + kSlack keys.
int cap_for(int d, int k) {
  const int margin = (kStageBytes / (kTileItems * d * 2)) * kTileItems;
  for (int cap = 512; cap <= 2048; cap <<= 1)
    if ((k + kSlack) * 4 <= (cap - margin) * 3) return cap;
  return -1;
}

Plan make_plan(int64_t n_users, int64_t n_items, int d, int k) {
  Plan p{};
  p.cap = cap_for(d, k);
  const int nut = d >= 256 ? 1 : 2;
  p.users_per_wg = nut * 32 * kWaves;
  p.n_ublocks = dr::ceil_div(n_users, p.users_per_wg);
  p.n_users_pad = p.n_ublocks * p.users_per_wg;
  const int slots = device_cus();  // one 512-thread workgroup per CU
  const int64_t stage_items = (kStageBytes / (kTileItems * d * 2)) * kTileItems;
  // Split the catalog into chunks only to balance the tail of the grid; each
  // chunk must stay long enough to amortise its warm-up, and the finalize
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

size_t diag_bytes(const Plan& p) {
#ifdef DR_TOPK_DIAG
  return (size_t)p.grid * kWaves * kDgSlots * sizeof(uint64_t);
#else
  (void)p;
  return 0;
#endif
}

}  // namespace

extern "C" size_t dr_score_topk_workspace(int64_t n_users, int64_t n_items, int d, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  if (d != 32 && d != 64 && d != 128 && d != 256) return 0;
  if (cap_for(d, k) < 0) return 0;
  Plan p = make_plan(n_users, n_items, d, k);
  return p.cand_bytes + p.cnt_bytes + diag_bytes(p) + 256;
}

#ifdef DR_TOPK_DIAG
// Diag builds only: byte offset (from the 256-B aligned workspace base) of the
// [grid*8][16] u64 counter block, and the grid size.
extern "C" size_t dr_score_topk_diag_offset(int64_t n_users, int64_t n_items, int d, int k,
                                            int* grid) {
  Plan p = make_plan(n_users, n_items, d, k);
  *grid = p.grid;
  return p.cand_bytes + p.cnt_bytes;
}
#endif

extern "C" int dr_score_topk(const void* user_table, const int64_t* user_ids, int64_t n_users,
                             const void* item_table, int64_t n_items, int64_t item_base, int d,
                             int k, const int64_t* excl_rowptr, const int32_t* excl_items,
                             float* out_scores, int32_t* out_items, void* workspace,
                             size_t workspace_bytes, dr_stream_t stream) {
  DR_CHECK_ARG(n_users >= 0 && n_items >= 0, "negative size");
  DR_CHECK_ARG(k >= 1 && k <= 1024, "k must be in [1, 1024]");
  DR_CHECK_ARG(d == 32 || d == 64 || d == 128 || d == 256,
               "d must be one of 32, 64, 128, 256");
  DR_CHECK_ARG(cap_for(d, k) > 0, "k too large for this d");
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
  Plan p = make_plan(n_users, n_items, d, k);
  const size_t need = p.cand_bytes + p.cnt_bytes + diag_bytes(p);
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if (!workspace || (size_t)(ws - (char*)workspace) + need > workspace_bytes) {
    dr::set_error("dr_score_topk: workspace too small (need " + std::to_string(need + 256) +
                  " bytes)");
    return DR_EWORKSPACE;
  }
  TopkArgs a;
  a.U = (const __bf16*)user_table;
  a.user_ids = user_ids;
  a.n_users = n_users;
  a.n_users_pad = p.n_users_pad;
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
  a.cnt = (int32_t*)(ws + p.cand_bytes);
  a.diag = (uint64_t*)(ws + p.cand_bytes + p.cnt_bytes);  // written only in DIAG builds

#define DR_SCAN(DD, CC) \
  hipLaunchKernelGGL((score_scan_kernel<DD, CC>), dim3(p.grid), dim3(kThreads), 0, s, a)
#define DR_SCAN_D(CC)                  \
  switch (d) {                         \
    case 32: DR_SCAN(32, CC); break;   \
    case 64: DR_SCAN(64, CC); break;   \
    case 128: DR_SCAN(128, CC); break; \
    default: DR_SCAN(256, CC); break;  \
  }
  if (p.cap == 512) {
    DR_SCAN_D(512)
  } else if (p.cap == 1024) {
    DR_SCAN_D(1024)
  } else {
    DR_SCAN_D(2048)
  }
#undef DR_SCAN_D
#undef DR_SCAN
  DR_CHECK_LAUNCH();

  const int P = p_for(p.n_chunks * p.cap);
  const int grid = (int)dr::ceil_div(n_users, 4);
#define DR_FIN(PP)                                                                            \
  hipLaunchKernelGGL((topk_finalize_kernel<PP>), dim3(grid), dim3(256), 0, s, a.cand, a.cnt,  \
                     p.n_chunks, p.cap, n_users, p.n_users_pad, k, excl_rowptr, excl_items,   \
                     out_scores, out_items)
  switch (P) {
    case 8: DR_FIN(8); break;
    case 16: DR_FIN(16); break;
    case 32: DR_FIN(32); break;
    default:
      dr::set_error("dr_score_topk: internal plan error (finalize size)");
      return DR_EUNSUPPORTED;
  }
#undef DR_FIN
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_topk_merge(const float* in_scores, const int32_t* in_items, int parts,
                             int64_t n_users, int k_in, int k_out, float* out_scores,
                             int32_t* out_items, dr_stream_t stream) {
  DR_CHECK_ARG(parts >= 1 && k_in >= 1 && k_out >= 1, "parts, k_in, k_out must be >= 1");
  DR_CHECK_ARG(k_out <= parts * k_in, "k_out must be <= parts * k_in");
  const int P = p_for(parts * k_in);
  DR_CHECK_ARG(P > 0, "parts * k_in must be <= 2048");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(in_scores && in_items && out_scores && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)dr::ceil_div(n_users, 4);
#define DR_MERGE(PP)                                                                        \
  hipLaunchKernelGGL((topk_merge_kernel<PP>), dim3(grid), dim3(256), 0, s, in_scores,       \
                     in_items, parts, n_users, k_in, k_out, out_scores, out_items)
  switch (P) {
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
