// Full-catalog user x item scoring with a fused top-K: the MI355X form of
// get_model_recommendations (reference divrec/train/utils.py:53-77), whose
// per-user loop scores every RankingDataset candidate (base_datasets.py:136-171)
// with MatrixFactorization.forward (matrix_factorization.py:26-28) and keeps
// candidates[argsort(scores, descending=True)][:k].
//
// Kernels:
//
// score_scan_kernel — one 512-thread workgroup (8 waves, two per SIMD) owns
//   UPWG = 8*NU_T*32 users (2048 for d <= 64, 1024 for d = 128) and streams one chunk of the
//   item catalog, so every item byte staged in LDS feeds UPWG flop.
//   * Each wave keeps the bf16 embeddings of its NU_T*32 users resident in
//     registers as MFMA B fragments for the whole scan.
//   * Item rows go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) into a ring
//     of stages (d = 128: two 64-KB slots, one stage ahead; else three
//     32-KB slots, two ahead), one s_barrier per stage; the LDS image is
//     XOR-swizzled through the per-lane source address so the A-fragment
//     ds_read_b128s are bank-conflict-free. All 8 waves share every stage.
//     A fragments are read two k-steps ahead of the MFMAs that use them.
//   * v_mfma_f32_32x32x16_bf16 puts items on M and users on N, so a lane holds
//     16 scores of ONE user: the hot epilogue is a 16-way max and one compare
//     with that user's running threshold. Scores never leave registers. The
//     two waves of a SIMD cover each other's epilogues.
//   * Survivors are stored straight into per-user candidate buffers in HBM
//     (slot from a per-user LDS counter). Once a buffer holds more than
//     k + kSlack + kFlushGap keys the wave compacts it with an in-register
//     radix select, keeping only keys that can still reach the top k, and
//     raises the user's threshold to the selected bound.
//   * Guessed thresholds (SEEDED = true, catalogs of 2^18 .. 2^23 rows): a
//     scan of a strided sample sets each user's starting threshold; users the
//     guess failed (fewer than k keys at the end) are rescanned from -inf.
//   * All VMEM traffic inside the scan (LDS-DMA and candidate stores) is
//     issued from inline asm and counted by the wave, so each stage wait is an
//     exact s_waitcnt vmcnt(N): no drain of the ring.
// topk_threshold_kernel — one wave per user: ks-th best key of the sample scan.
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
  kDgNTiles, kDgNEnqueue, kDgNDrain, kDgNFlush, kDgNStages, kDgRealtime, kDgSlots = 16
};

// Geometry knobs. The defaults are the product configuration; the -D
// overrides exist so tools/variant_bench.py can time alternatives side by side
// (build_native.py --variant NAME -D KEY=VAL).
#ifndef DR_STAGE_BYTES
#define DR_STAGE_BYTES 32768  // one LDS ring slot, d != 128
#endif
#ifndef DR_RING
#define DR_RING 3  // ring slots (RING - 1 stages in flight), d != 128
#endif
#ifndef DR_STAGE_BYTES_WIDE
#define DR_STAGE_BYTES_WIDE 65536  // ring slot for d = 128
#endif
#ifndef DR_RING_WIDE
#define DR_RING_WIDE 2  // ring slots for d = 128
#endif
#ifndef DR_NUT
#define DR_NUT 4  // user tiles of 32 per wave for d = 128
#endif
#ifndef DR_NUT_NARROW
#define DR_NUT_NARROW 8  // user tiles of 32 per wave for d <= 64 (measured: 8 is +14 % at d=64, 1M x 1M)
#endif
#ifndef DR_PRIO
#define DR_PRIO 0  // static s_setprio 1 for waves 4-7 (measured: no gain)
#endif
#ifndef DR_APIPE
#define DR_APIPE 1  // A fragments read two k-steps ahead
#endif
#ifndef DR_FLUSH_GAP
#define DR_FLUSH_GAP 96  // new keys a buffer takes past k + kSlack before compaction
#endif
#ifndef DR_ENQ_STAGED
// survivors: 0 = direct per-lane enqueue, 1 = stage lane blocks in LDS and
// resolve them per stage, 2 = staged for d <= 64 only (measured: staged is 4%
// faster at d=64, where survivors per MFMA are twice as dense, and 4% slower
// at d=128)
#define DR_ENQ_STAGED 2
#endif
#ifndef DR_ENQ_FAST
#define DR_ENQ_FAST 1  // direct enqueue: one-survivor lanes store their max (no value select)
#endif
#ifndef DR_STAGE_BLOCKS
#define DR_STAGE_BLOCKS 64  // staged lane blocks per wave (>= 64: one user tile always fits)
#endif
#ifndef DR_COMPACT_INLINE
#define DR_COMPACT_INLINE __noinline__
#endif

constexpr int kWaves = 8;  // two waves per SIMD: 256-register budget each
constexpr int kThreads = kWaves * 64;
constexpr int kTileItems = 32;
#ifndef DR_SLACK
#define DR_SLACK 32
#endif
constexpr int kSlack = DR_SLACK;  // keys kept beyond k by a compaction
constexpr int kFlushGap = DR_FLUSH_GAP;

// Stage geometry per row width. d = 128: two 64-KB slots (one barrier per
// 8 tiles at d=128; measured against three 32-KB slots: +2 % at 10M items,
// +6 % at 1.25M, where the survivor stream makes per-stage wave imbalance
// larger). d <= 64: three 32-KB slots (its LDS survivor staging needs room;
// 64-KB stages measured -10 % there; d = 256 spills with them).
constexpr int stage_bytes_for(int d) { return d == 128 ? DR_STAGE_BYTES_WIDE : DR_STAGE_BYTES; }
constexpr int ring_for(int d) { return d == 128 ? DR_RING_WIDE : DR_RING; }

template <int D>
struct TileGeom {
  static constexpr int STAGE_BYTES = stage_bytes_for(D);  // one LDS ring slot
  static constexpr int RING = ring_for(D);                // slots (RING - 1 stages in flight)
  static constexpr int LPT = STAGE_BYTES / 16 / kThreads;  // LDS-DMA per thread per stage
  static constexpr int KSTEPS = D / 16;                 // MFMA k-steps per row
  static constexpr int CPR = D / 8;                     // 16-B chunks per row
  static constexpr int TILE_BYTES = kTileItems * D * 2;
  static constexpr int SR = STAGE_BYTES / TILE_BYTES;   // row tiles per stage
  static_assert(LPT >= 1 && STAGE_BYTES % (16 * kThreads) == 0, "stage geometry");
  static_assert(RING >= 2, "ring depth");
  static constexpr int RPB = (2 * D >= 256) ? 1 : 256 / (2 * D);  // rows per 256-B bank row
  static constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  static constexpr int MARGIN = SR * kTileItems;  // max new keys per user per stage
  static_assert(SR >= 1, "a stage holds at least one tile");
  // physical chunk = logical chunk ^ swz(row): spreads the 32 rows that one
  // A-fragment ds_read_b128 touches over distinct 16-B bank slots.
  __device__ static int swz(int r) { return (r / RPB) & SWM; }
};

// User tiles (of 32) per wave. The B fragments take NU_T*KSTEPS*4 VGPRs (128 at
// d=128, NU_T=4; 128 at d=64, NU_T=8). The tiles are scored in groups of at
// most four against each item tile, one accumulator set (4*16 VGPRs) reused
// by the groups, so narrow rows can hold more users per wave.
constexpr int nut_for(int d) { return d >= 256 ? 2 : (d <= 64 ? DR_NUT_NARROW : DR_NUT); }
constexpr int ngroup_for(int d) { return nut_for(d) > 4 ? 4 : nut_for(d); }
template <int V>
struct IC {
  static constexpr int value = V;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ asm VMEM
// The scan issues its VMEM traffic from inline asm so that hipcc does not put
// its own conservative s_waitcnt vmcnt(0) in front of the MFMAs (it cannot
// prove a C++ ds_read does not alias an in-flight LDS-DMA); the wave counts
// every instruction it issues and waits with exact counts. M0 is used by no
// other code in the kernel.
__device__ __forceinline__ void st64(uint64_t* p, uint64_t v) {
  asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 ds_read_b128_asm(uint32_t lds_addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr));
  return v;
}
// LDS waits that name the fragment they retire ("+v"): no consumer of it can
// be scheduled above the wait. lgkmcnt(1) = every LDS read but the youngest
// has returned (LDS reads return in order; extra younger reads only make the
// wait stricter).
__device__ __forceinline__ void lds_wait1(u32x4& v) {
  asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(v) : : "memory");
}
__device__ __forceinline__ void lds_wait0(u32x4& v) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) : : "memory");
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their maxima).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
// Wait until at most n (wave-uniform) VMEM ops are outstanding, rounding n
// down to a power of two (waits for a little more than required, always
// correct): six scalar compares instead of a 64-step ladder at every stage.
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  if (n >= 32) wait_vmcnt<32>();
  else if (n >= 16) wait_vmcnt<16>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else if (n >= 2) wait_vmcnt<2>();
  else if (n >= 1) wait_vmcnt<1>();
  else wait_vmcnt<0>();
}

// Issue the LDS-DMA of one stage: rows [row0, row0 + SR*32) of the slice into
// the ring slot at LDS byte address `lds_stage`. The image is lane-linear
// (glds writes base + lane*16); the swizzle is on the SOURCE address
// (cdna_hip_programming.md §5.4 rule 21). Rows past the slice end are
// clamped to its last row; their scores are masked in the epilogue.
// Addressing is SGPR base (the stage's first row) + a 32-bit per-lane offset
// recomputed at every stage from the thread id: the empty asm makes the id
// opaque, so hipcc cannot hoist 64-bit per-lane addresses out of the tile loop
// (they cost registers the loop does not have, and their spill reloads wait
// vmcnt(0), draining the ring).
template <int D>
__device__ __forceinline__ void issue_stage(const __bf16* __restrict__ I, int64_t n_items,
                                            int64_t row0, uint32_t lds_stage) {
  using G = TileGeom<D>;
  constexpr int ROWS = G::SR * kTileItems;
  uint32_t tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = (int)(tid & 63u);
  const int wave = (int)(__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
  const char* base = reinterpret_cast<const char*>(I + row0 * D);
  const int64_t left = n_items - 1 - row0;
  const int rmax = left < ROWS - 1 ? (int)left : ROWS - 1;
#pragma unroll
  for (int j = 0; j < G::LPT; ++j) {
    const int wave_first = j * kThreads + wave * 64;  // wave-uniform chunk index
    const int idx = wave_first + lane;
    const int r = idx / G::CPR;
    const int lc = (idx % G::CPR) ^ G::swz(r & 31);
    const int rr = r < rmax ? r : rmax;
    const uint32_t off = (uint32_t)(rr * (2 * D) + lc * 16);
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_stage + wave_first * 16);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(off), "s"(base), "s"(m0)
                 : "memory", "m0");
#pragma clang diagnostic pop
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
__device__ DR_COMPACT_INLINE CompactResult compact_buffer(uint64_t* __restrict__ buf, int n_in, int k,
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
  const float* init_thr;  // [n_users_pad] starting thresholds (SEEDED scans only)
  // Fallback rescan only: the user count lives on the device (n_users and
  // n_ublocks above are its upper bounds), and pos_map[p] is the caller's
  // position of list entry p (its exclusion row). NULL otherwise.
  const int32_t* n_users_dev;
  const int64_t* pos_map;
  uint64_t* cand;  // [n_chunks][n_users_pad][CAP] keys (unsorted)
  int32_t* cnt;    // [n_chunks][n_users_pad] valid keys per buffer
  uint64_t* diag;  // [gridDim.x * kWaves][kDgSlots] in DR_TOPK_DIAG builds
};

template <int D, int CAP, bool SEEDED>
__global__ __launch_bounds__(kThreads, 2) void score_scan_kernel(TopkArgs a) {
  using G = TileGeom<D>;
  constexpr int NU_T = nut_for(D);
  constexpr int NG = ngroup_for(D);  // user tiles per accumulator group
  constexpr int NGRP = NU_T / NG;    // groups scored against each item tile
  static_assert(NGRP * NG == NU_T && NGRP <= 2, "user tile groups");
  constexpr int KS = G::KSTEPS;
  constexpr int SR = G::SR;
  constexpr int UPW = NU_T * 32;      // users per wave
  constexpr int UPWG = UPW * kWaves;  // users per workgroup
  constexpr int P = CAP / 64;         // keys per lane in a compaction
  constexpr int kRing = G::RING;
  constexpr int kStageBytes = G::STAGE_BYTES;
  constexpr int kLpt = G::LPT;
  constexpr int RING_BYTES = kRing * kStageBytes;
  // per wave: per-user key counts, radix histogram, staged survivor blocks
  // (16 scores + item base + slot + threshold each)
  constexpr bool STAGED = DR_ENQ_STAGED == 1 || (DR_ENQ_STAGED == 2 && D <= 64);
  constexpr int SB = STAGED ? DR_STAGE_BLOCKS : 0;
  // stage_hits resolves a full stage area, then stages up to 64 lanes of one
  // user tile: the area must hold a whole wave's worth of blocks
  static_assert(!STAGED || SB >= 64, "staging area smaller than a wave");
  constexpr int WAVE_BYTES = UPW * 4 + 256 * 4 + SB * (64 + 12);
  static_assert(RING_BYTES + kWaves * WAVE_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[RING_BYTES + kWaves * WAVE_BYTES];

  // A buffer is compacted once it holds more than flush_at keys; a stage adds
  // at most MARGIN keys per user, so flush_at + MARGIN <= CAP. A small gap
  // above k + kSlack keeps the thresholds close to the running k-th score.
  // Unseeded scans start at -inf: every score of the first stages is a
  // survivor until the first compaction sets a real threshold.
  int flush_at = a.k + kSlack + kFlushGap;
  flush_at = flush_at < CAP - G::MARGIN ? flush_at : CAP - G::MARGIN;

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int col = lane & 31;
#if DR_PRIO
  // The second-dispatched half of the workgroup loses VALU arbitration to its
  // SIMD partner on every segment; one static priority bump evens the pair
  // (cdna_hip_programming.md T5, static form). Wave-uniform by readfirstlane.
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
  char* wbase = smem + RING_BYTES + wave * WAVE_BYTES;
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(wbase);
  uint32_t* hist = reinterpret_cast<uint32_t*>(wbase + UPW * 4);
  float* blk_val = reinterpret_cast<float*>(wbase + UPW * 4 + 1024);  // [SB][16], 16-B aligned
  uint32_t* blk_gbase = reinterpret_cast<uint32_t*>(blk_val + SB * 16);
  uint32_t* blk_slot = blk_gbase + SB;  // slot | h << 16 | valid rows << 17
  float* blk_thr = reinterpret_cast<float*>(blk_slot + SB);
  const uint32_t lds_ring = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  // This lane's A-fragment byte offset for k-step s in a tile is
  // col*2D + ((2s + h) ^ swz(col)) * 16 = a_row + ((2s) ^ a_sw) * 16: two VALU
  // per read instead of KS resident offsets (registers are the budget here).
  const uint32_t a_row = (uint32_t)(col * (2 * D));
  const uint32_t a_sw = (uint32_t)(h ^ G::swz(col));
  auto a_off = [&](int s) -> uint32_t { return a_row + ((((uint32_t)(2 * s)) ^ a_sw) << 4); };

#ifdef DR_TOPK_DIAG
  uint64_t dg[kDgSlots] = {};
  DG_T0(t_kernel);
  const uint64_t rt_kernel = __builtin_amdgcn_s_memrealtime();  // 100 MHz: clock = cycles / time
#endif
  int64_t n_users = a.n_users, n_ublocks = a.n_ublocks;
  if (a.n_users_dev) {  // fallback rescan: only the users the guess failed
    const int64_t n = __builtin_amdgcn_readfirstlane(*a.n_users_dev);
    n_users = n < n_users ? n : n_users;
    n_ublocks = (n_users + UPWG - 1) / UPWG;
  }
  const int64_t n_units = n_ublocks * a.n_chunks;
  for (int64_t unit = blockIdx.x; unit < n_units; unit += gridDim.x) {
    DG_T0(t_pro);
    const int64_t chunk = unit / n_ublocks;
    const int64_t ub = unit % n_ublocks;
    const int64_t i_beg = chunk * a.chunk_items;
    int64_t i_end = i_beg + a.chunk_items;
    i_end = i_end < a.n_items ? i_end : a.n_items;
    const int ntiles = i_end > i_beg ? (int)((i_end - i_beg + kTileItems - 1) / kTileItems) : 0;
    const int nst = (ntiles + SR - 1) / SR;
    const int64_t upos0 = ub * UPWG + (int64_t)wave * UPW;  // first user position of the wave
    uint64_t* cbase = a.cand + ((size_t)chunk * a.n_users_pad + upos0) * CAP;

    // Resident B fragments: lane holds user (ut*32+col), k = 16s + 8h .. +7.
    bf16x8 bfr[NU_T][KS];
    float thr[NU_T];
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) {
      const int64_t pos = upos0 + ut * 32 + col;
      int64_t row = 0;
      if (pos < n_users) row = a.user_ids ? a.user_ids[pos] : pos;
      const uint4* src = reinterpret_cast<const uint4*>(a.U + row * D + 8 * h);
#pragma unroll
      for (int s = 0; s < KS; ++s) bfr[ut][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
      thr[ut] = SEEDED ? a.init_thr[pos] : -INFINITY;
    }
    // Retire those loads where the compiler can see it (else it waits for them
    // inside the loop, draining the ring).
    wait_vmcnt<0>();
    for (int s = lane; s < UPW; s += 64) ucnt[s] = 0;
    int vmc = 0;        // VMEM instructions issued by this wave in this unit
    int vm_done = 0;    // every op issued before this count has completed
    int vs[kRing - 1];  // vmc right after each outstanding stage's DMA
#pragma unroll
    for (int i = 0; i < kRing - 1; ++i) vs[i] = 0;
    DG_ADD(kDgPrologue, t_pro);

    // -------------------------------------------------------------- MFMA tile
    auto mma_tile = [&](int t, f32x16 (&acc)[NG], auto GI) {
      constexpr int g0 = decltype(GI)::value * NG;
      const uint32_t tb = lds_ring + ((t / SR) % kRing) * kStageBytes + (t % SR) * G::TILE_BYTES;
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) acc[ut] = f32x16{};
#if DR_APIPE
      // Fragment s is read two k-steps before its MFMAs; each wait retires
      // exactly the fragment the next MFMAs consume.
      u32x4 af[KS];
      af[0] = ds_read_b128_asm(tb + a_off(0));
      if constexpr (KS > 1) af[1] = ds_read_b128_asm(tb + a_off(1));
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (s + 1 < KS) lds_wait1(af[s]);
        else lds_wait0(af[s]);
        if (s + 2 < KS) af[s + 2] = ds_read_b128_asm(tb + a_off(s + 2));
#pragma unroll
        for (int ut = 0; ut < NG; ++ut)
          acc[ut] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[s]),
                                                            bfr[g0 + ut][s], acc[ut], 0, 0, 0);
      }
#else
      constexpr int HALF = KS >= 4 ? KS / 2 : KS;
#pragma unroll
      for (int s0 = 0; s0 < KS; s0 += HALF) {
        u32x4 af[HALF];
#pragma unroll
        for (int s = 0; s < HALF; ++s) af[s] = ds_read_b128_asm(tb + a_off(s0 + s));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < HALF; ++s)
#pragma unroll
          for (int ut = 0; ut < NG; ++ut)
            acc[ut] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf16x8, af[s]), bfr[g0 + ut][s0 + s], acc[ut], 0, 0, 0);
      }
#endif
    };

    // -------------------------------------------------------------- cold paths
    auto compact = [&](int ut, int c, int n_in) {
      DG_T0(t_f);
      const int slot = ut * 32 + c;
      const int64_t upos = upos0 + slot;
      const int32_t* ex = nullptr;
      int exn = 0;
      if (a.excl_rowptr && upos < n_users) {
        const int64_t er = a.pos_map ? a.pos_map[upos] : upos;
        const int64_t e0 = a.excl_rowptr[er], e1 = a.excl_rowptr[er + 1];
        ex = a.excl_items + e0;
        exn = (int)(e1 - e0);
      }
      const CompactResult r = compact_buffer<P>(cbase + (size_t)slot * CAP, n_in, a.k, ex, exn, hist);
      vm_done = vmc;
      if (lane == 0) ucnt[slot] = (uint32_t)r.kept;
      wave_lds_sync();
#pragma unroll
      for (int u2 = 0; u2 < NU_T; ++u2)
        if (u2 == ut && col == c) thr[u2] = fmaxf(thr[u2], r.thr);  // both bounds are valid
      DG_ADD(kDgFlush, t_f);
      DG_CNT(kDgNFlush);
    };

    auto check_compact = [&]() {
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        const uint32_t c_cnt = ucnt[ut * 32 + col];
        uint64_t need = __ballot(c_cnt > (uint32_t)flush_at) & 0xffffffffull;
        while (need) {
          const int c = __builtin_ctzll(need);
          need &= need - 1;
          compact(ut, c, __builtin_amdgcn_readlane((int)c_cnt, c));
        }
      }
    };

    // -------------------------------------------------------------- epilogues
    // Hot test (branch-free): per user tile, a 16-way max against the threshold.
    auto any_hits = [&](f32x16 (&acc)[NG], auto GI) -> uint32_t {
      constexpr int g0 = decltype(GI)::value * NG;
      uint32_t bits = 0;
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        float m = acc[ut][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, acc[ut][r]);
        bits |= (__ballot(m > thr[g0 + ut]) != 0ull ? 1u : 0u) << ut;
      }
      return bits;
    };

    // Append survivors straight to their users' candidate buffers in HBM: one
    // key per lane per round, its slot from the user's LDS key counter. No
    // call and no queue in the hot loop, so nothing forces the accumulators
    // and B fragments out of registers. A stage adds at most MARGIN keys per
    // user, so a buffer compacted at the stage end never overflows.
    auto enqueue = [&](int t, f32x16 (&acc)[NG], uint32_t hit_bits, auto GI) {
      constexpr int g0 = decltype(GI)::value * NG;
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
      uint32_t vmask = 0xffffu;  // rows past the slice end (last tile only)
      if (valid < kTileItems) {
        vmask = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          vmask |= (row < valid ? 1u : 0u) << r;
        }
      }
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        if (!(hit_bits & (1u << ut))) continue;
        uint32_t mask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) mask |= (acc[ut][r] > thr[g0 + ut] ? 1u : 0u) << r;
        mask &= vmask;
        const int slot = (g0 + ut) * 32 + col;
        uint64_t* ubuf = cbase + (size_t)slot * CAP;  // this lane's user buffer
#if DR_ENQ_FAST
        // Common case: every hitting lane holds ONE survivor. It is then the
        // lane's maximum (all other scores are <= thr < it), so one round
        // stores it without the 16-way value select. Full tiles only (the
        // max of a partial tile may sit in a row past the slice end).
        if (vmask == 0xffffu && __ballot((mask & (mask - 1u)) != 0u) == 0ull) {
          if (__ballot(mask != 0u) != 0ull) {
            float m = acc[ut][0];
#pragma unroll
            for (int q = 1; q < 16; ++q) m = fmaxf(m, acc[ut][q]);
            if (mask != 0u) {
              const int r = __builtin_ctz(mask);
              const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
              const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
              if (pos < (uint32_t)CAP) st64(ubuf + pos, dr::make_key(m, gbase + (uint32_t)row));
            }
            vmc += 1;  // the store above issued once (some lane had a key)
          }
          continue;
        }
#endif
        while (__ballot(mask != 0u) != 0ull) {
          const bool has = mask != 0u;
          const int r = has ? __builtin_ctz(mask) : 0;
          mask &= mask - 1u;
          float v = acc[ut][0];
#pragma unroll
          for (int q = 1; q < 16; ++q) v = (r == q) ? acc[ut][q] : v;
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          if (has) {
            const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
            if (pos < (uint32_t)CAP)  // always true (flush_at + MARGIN <= CAP): a guard only
              st64(ubuf + pos, dr::make_key(v, gbase + (uint32_t)row));
          }
          vmc += 1;  // the store above issued once (some lane had a key)
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
    // Staged survivors. In the tile loop a lane whose 16 scores of a user tile
    // beat the user's threshold only copies them to an LDS block (four
    // ds_write_b128 + its item base, slot and threshold); resolve() later
    // turns the staged blocks into candidate keys with one lane per block, so
    // the per-score tests, value selects and LDS counter atomics run in
    // parallel across blocks, off the MFMA loop. A block's threshold is the one
    // at staging time: thresholds only rise, so it admits a superset.
    int nblk = 0;  // staged blocks (wave-uniform)
    auto resolve = [&]() {
      DG_T0(t_d);
      wave_lds_sync();
#pragma unroll 1
      for (int b0 = 0; b0 < nblk; b0 += 64) {
        const int i = b0 + lane;
        const bool live = i < nblk;
        const int ii = live ? i : 0;
        const uint32_t gb = blk_gbase[ii];
        const uint32_t info = blk_slot[ii];  // slot | h << 16 | valid rows << 17
        const float th = blk_thr[ii];
        const uint32_t slot = info & 0xffffu;
        const int hh = (int)((info >> 16) & 1u);
        const int vld = live ? (int)(info >> 17) : 0;
        uint64_t* ubuf = cbase + (size_t)slot * CAP;
        const float4* src = reinterpret_cast<const float4*>(blk_val + ii * 16);
        // four registers (one float4) at a time: few VGPRs, so this also runs
        // inside stage_hits with the accumulators live
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {
          const float4 v4 = src[q];
          const float vq[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = j + 8 * q + 4 * hh;  // score register r = 4q + j
            const bool hit = row < vld && vq[j] > th;
            if (__ballot(hit) != 0ull) {
              if (hit) {
                const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
                // pos < CAP always holds (flush_at + MARGIN <= CAP); the test
                // keeps a broken invariant from ever writing past the buffer
                if (pos < (uint32_t)CAP) st64(ubuf + pos, dr::make_key(vq[j], gb + (uint32_t)row));
              }
              vmc += 1;  // one store instruction (some lane had a key)
            }
          }
        }
      }
      nblk = 0;
      wave_lds_sync();
      DG_ADD(kDgDrain, t_d);
      DG_CNT(kDgNDrain);
    };
    auto stage_hits = [&](int t, f32x16 (&acc)[NG], uint32_t hit_bits, auto GI) {
      constexpr int g0 = decltype(GI)::value * NG;
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        if (!(hit_bits & (1u << ut))) continue;
        float m = acc[ut][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, acc[ut][r]);
        const bool hit = m > thr[g0 + ut];
        const uint64_t bal = __ballot(hit);
        if (bal == 0ull) continue;
        const int n = __popcll(bal);
        if (nblk + n > SB) resolve();  // rare (a scan's first stages): few registers
        if (hit) {
          const int i = nblk + lane_prefix(bal);
          float4* dst = reinterpret_cast<float4*>(blk_val + i * 16);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            dst[q] = make_float4(acc[ut][4 * q], acc[ut][4 * q + 1], acc[ut][4 * q + 2],
                                 acc[ut][4 * q + 3]);
          blk_gbase[i] = gbase;
          blk_slot[i] =
              (uint32_t)((g0 + ut) * 32 + col) | ((uint32_t)h << 16) | ((uint32_t)valid << 17);
          blk_thr[i] = thr[g0 + ut];
        }
        nblk += n;
      }
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    auto epilogue = [&](int t, f32x16 (&acc)[NG], auto GI) {
      DG_T0(t_h);
      uint32_t hit_bits = any_hits(acc, GI);
      DG_ADD(kDgHits, t_h);
      hit_bits = __builtin_amdgcn_readfirstlane(hit_bits);  // ballots: uniform
      // the stage-end work runs after the last group of the tile
      constexpr bool last_group = decltype(GI)::value == NGRP - 1;
      if constexpr (STAGED) {
        if (hit_bits != 0u) stage_hits(t, acc, hit_bits, GI);
        // end of a stage: resolve the staged blocks, compact full buffers
        if (last_group && ((t + 1) % SR == 0 || t + 1 == ntiles)) {
          if (nblk > 0) resolve();
          check_compact();
        }
      } else {
        if (hit_bits != 0u) enqueue(t, acc, hit_bits, GI);
        // end of a stage: compact the buffers that passed flush_at
        if (last_group && ((t + 1) % SR == 0 || t + 1 == ntiles)) check_compact();
      }
    };
    // One accumulator set: the partner wave on the same SIMD issues its MFMAs
    // while this wave runs the epilogue (two waves per SIMD by design).
    f32x16 acc[NG];
    for (int t = 0; t < ntiles; ++t) {
      DG_CNT(kDgNTiles);
      if (t % SR == 0) boundary(t / SR);
      DG_T0(t_m);
      mma_tile(t, acc, IC<0>{});
      DG_ADD(kDgMma, t_m);
      epilogue(t, acc, IC<0>{});
      if constexpr (NGRP > 1) {
        DG_T0(t_m2);
        mma_tile(t, acc, IC<1>{});
        DG_ADD(kDgMma, t_m2);
        epilogue(t, acc, IC<1>{});
      }
    }
    wait_vmcnt<0>();
    wave_lds_sync();
    for (int s = lane; s < UPW; s += 64)
      a.cnt[(size_t)chunk * a.n_users_pad + upos0 + s] = (int32_t)ucnt[s];
    __syncthreads();  // the ring is refilled by the next unit
  }
#ifdef DR_TOPK_DIAG
  DG_ADD(kDgTotal, t_kernel);
  dg[kDgRealtime] = __builtin_amdgcn_s_memrealtime() - rt_kernel;
  if (lane == 0 && a.diag) {  // the rescan (usually empty) leaves the main scan's record
    uint64_t* o = a.diag + ((size_t)blockIdx.x * kWaves + wave) * kDgSlots;
#pragma unroll
    for (int i = 0; i < kDgSlots; ++i) o[i] = dg[i];
  }
#endif
}


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

int64_t stage_items_for(int d) {
  return (int64_t)(stage_bytes_for(d) / (kTileItems * d * 2)) * kTileItems;
}

// Smallest candidate capacity that leaves at least 32 keys of headroom above
// k + kSlack once a stage's worth of new keys (the margin) is reserved.
int cap_for(int d, int k) {
  const int margin = (int)stage_items_for(d);
  for (int cap = 512; cap <= 2048; cap <<= 1)
    if (k + kSlack + 32 <= cap - margin) return cap;
  return -1;
}

Plan make_plan(int64_t n_users, int64_t n_items, int d, int k) {
  Plan p{};
  p.cap = cap_for(d, k);
  p.users_per_wg = nut_for(d) * 32 * kWaves;
  p.n_ublocks = dr::ceil_div(n_users, p.users_per_wg);
  p.n_users_pad = p.n_ublocks * p.users_per_wg;
  const int slots = device_cus();  // one 512-thread workgroup per CU
  const int64_t stage_items = stage_items_for(d);
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

Guess guess_for(int64_t n_items, int k) {
  Guess g;
  if (!DR_GUESS || n_items < kGuessMinItems || n_items > kGuessMaxItems) return g;
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

Layout make_layout(int64_t n_users, int64_t n_items, int d, int k) {
  Layout L{};
  L.main = make_plan(n_users, n_items, d, k);
  L.g = guess_for(n_items, k);
  L.cand = L.main.cand_bytes;
  L.cnt = L.main.cnt_bytes;
  if (L.g.S > 0) {
    L.sample = make_plan(n_users, L.g.S, d, L.g.ks);
    L.cand = L.cand > L.sample.cand_bytes ? L.cand : L.sample.cand_bytes;
    L.cnt = L.cnt > L.sample.cnt_bytes ? L.cnt : L.sample.cnt_bytes;
    L.thr = al256((size_t)L.main.n_users_pad * sizeof(float));
    L.samp = al256((size_t)L.g.S * d * 2);
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

template <bool SEEDED>
void launch_scan(const Plan& p, const TopkArgs& a, int d, hipStream_t s) {
#define DR_SCAN(DD, CC) \
  hipLaunchKernelGGL((score_scan_kernel<DD, CC, SEEDED>), dim3(p.grid), dim3(kThreads), 0, s, a)
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
}

}  // namespace

extern "C" size_t dr_score_topk_workspace(int64_t n_users, int64_t n_items, int d, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  if (d != 32 && d != 64 && d != 128 && d != 256) return 0;
  if (cap_for(d, k) < 0) return 0;
  return make_layout(n_users, n_items, d, k).total() + 256;
}

#ifdef DR_TOPK_DIAG
// Diag builds only: byte offset (from the 256-B aligned workspace base) of the
// [grid*8][16] u64 counter block of the main scan, and its grid size.
extern "C" size_t dr_score_topk_diag_offset(int64_t n_users, int64_t n_items, int d, int k,
                                            int* grid) {
  Layout L = make_layout(n_users, n_items, d, k);
  *grid = L.main.grid;
  return L.off_diag();
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
  const Layout L = make_layout(n_users, n_items, d, k);
  const size_t need = L.total();
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if (!workspace || (size_t)(ws - (char*)workspace) + need > workspace_bytes) {
    dr::set_error("dr_score_topk: workspace too small (need " + std::to_string(need + 256) +
                  " bytes)");
    return DR_EWORKSPACE;
  }
  const Plan& p = L.main;
  TopkArgs a{};
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
  a.init_thr = nullptr;
  a.n_users_dev = nullptr;
  a.pos_map = nullptr;
  a.cand = (uint64_t*)ws;
  a.cnt = (int32_t*)(ws + L.cand);
  a.diag = (uint64_t*)(ws + L.off_diag());  // written only in DIAG builds
  const int fin_grid = (int)dr::ceil_div(n_users, 4);
  const int P = p_for(p.n_chunks * p.cap);

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
    launch_scan<false>(p, a, d, s);
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
  __bf16* samp = (__bf16*)(ws + L.off_samp());
  int64_t* frows = (int64_t*)(ws + L.off_frows());
  int64_t* fpos = (int64_t*)(ws + L.off_fpos());
  int32_t* fcnt = (int32_t*)(ws + L.off_fcnt());
  DR_CHECK_HIP(hipMemsetAsync(fcnt, 0, sizeof(int32_t), s));
  {
    const int cpr = d / 8;
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
  launch_scan<false>(L.sample, as, d, s);
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
  launch_scan<true>(p, a, d, s);
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
  launch_scan<false>(p, af, d, s);
  DR_CHECK_LAUNCH();
#define DR_FIN_RESCAN(PP) DR_FIN(PP, fpos, fcnt, nullptr)
  DR_BY_P(P, DR_FIN_RESCAN)
#undef DR_FIN_RESCAN
#undef DR_FIN
#undef DR_BY_P
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
