// The streaming score scan of dr_score_topk (csrc/score_topk.hip), shared by
// the per-dtype translation units score_scan_bf16.hip and score_scan_f32.hip.
//
// score_scan_kernel<W, CAP, SEEDED, F32> — one 512-thread workgroup (8 waves,
//   two per SIMD) owns UPWG = 8*NU_T*32 users and streams one chunk of the item
//   catalog, so every item byte staged in LDS feeds UPWG products.
//   * W is the row width in bf16 units (row bytes / 2): a bf16 table of width d
//     has W = d, an fp32 table W = 2d. Geometry (stages, user tiles, LDS
//     swizzle, 16-B fragments) depends only on the row bytes, so both dtypes
//     share it; only the MFMA differs (kstep_mma).
//   * Each wave keeps the rows of its NU_T*32 users resident in registers as
//     MFMA B fragments for the whole scan.
//   * Item rows go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) into a ring
//     of stages (W = 128: two 72-KB slots, one stage ahead; W <= 64: two
//     56-KB slots; W >= 256: three 32-KB slots, two ahead), one s_barrier per
//     stage; the LDS image is
//     XOR-swizzled through the per-lane source address so the A-fragment
//     ds_read_b128s are bank-conflict-free. All 8 waves share every stage.
//     A fragments are read two k-steps ahead of the MFMAs that use them.
//   * The 32x32 MFMAs put items on M and users on N, so a lane holds 16 scores
//     of ONE user: the hot epilogue is a 16-way max and one compare with that
//     user's running threshold. Scores never leave registers. The two waves of
//     a SIMD cover each other's epilogues.
//   * Survivors are stored straight into per-user candidate buffers in HBM
//     (slot from a per-user LDS counter), or for W <= 64 staged in LDS and
//     resolved per stage. Once a buffer holds more than k + kSlack + kFlushGap
//     keys the wave compacts it with an in-register radix select, keeping only
//     keys that can still reach the top k, and raises the user's threshold to
//     the selected bound.
//   * Guessed thresholds (SEEDED = true): a scan of a strided sample sets each
//     user's starting threshold; users the guess failed are rescanned.
//   * All VMEM traffic inside the scan (LDS-DMA and candidate stores) is
//     issued from inline asm and counted by the wave, so each stage wait is an
//     exact s_waitcnt vmcnt(N): no drain of the ring.
#pragma once

#include "common.h"

namespace dr_topk {


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

// Geometry. Every alternative measured against these values lost and was
// removed (DESIGN.md §3.1, A/B records under profiles/): one wave per SIMD
// (rounds 2 and 5), 12 / 16 waves at d <= 64, SIMD-pair priorities, two
// accumulator sets in ping-pong, the A fragments read per half chain, other
// stage sizes, slacks and flush gaps. The one -D knob kept is the d = 128
// stage size (DR_STAGE_BYTES_WIDE, tools/build_variants.sh), re-measured in
// round 6 with PMC FETCH beside the time at the headline (1M x 10M, k = 100;
// profiles/r06/stage_fetch/): 72 KB 1770 ms, main-scan FETCH 227.6 GB;
// 64 KB 1776 ms, 243.0 GB. 72 KB wins both.
#ifndef DR_STAGE_BYTES_WIDE
#define DR_STAGE_BYTES_WIDE 73728  // ring slot for d = 128 (9 tiles: 72 KB)
#endif
constexpr int kStageBytesOther = 32768;  // ring slot for d = 256 / 512 (three slots)
constexpr int kRingOther = 3;
constexpr int kRingWide = 2;          // d = 128: two slots, one stage ahead
constexpr int kNutWide = 4;           // user tiles of 32 per wave for d = 128
constexpr int kNutNarrow = 8;         // for d <= 64 (+14 % at d = 64, 1M x 1M, against 4)
constexpr int kFlushGapDefault = 96;  // new keys a buffer takes past k + kSlack before compaction
// Survivors are staged in LDS and resolved per stage for d <= 64 (twice as
// dense per MFMA there: 4 % faster) and for d = 128 long lists (below),
// stored directly for other d >= 128 (4 % faster there at k = 100).
constexpr int kStageBlocks = 64;  // staged lane blocks per wave (>= 64: one user tile always fits)

// Waves per workgroup of a scan (one workgroup per CU): two per SIMD, 256
// VGPRs each.
constexpr int kWavesScan = 8;
constexpr int waves_for(int) { return kWavesScan; }
constexpr int kMaxWaves = kWavesScan;
constexpr int kTileItems = 32;
constexpr int kSlack = 32;  // keys kept beyond k by a compaction
constexpr int kFlushGap = kFlushGapDefault;

// Stage geometry per row width. d = 128: two 72-KB slots (one barrier per
// 9 tiles; measured against three 32-KB slots: +2 % at 10M items, +6 % at
// 1.25M, where the survivor stream makes per-stage wave imbalance larger;
// round 5: against two 64-KB slots -0.4 to -0.8 % at 10M, -0.35 to -0.65 % at
// k = 1000, +0.1 % at 1.25M; three 48-KB slots +1 to +2.6 %). d <= 64 (its
// LDS survivor staging needs room): two 56-KB slots, a barrier every 14 tiles
// at d = 64 (round 5, two 48-KB slots against three 32-KB: -0.4 to -0.9 % at
// config 2, -1.6 % at d = 32; four 24-KB slots +3.5 %; 56 KB, with the
// compaction histogram moved into the staging area, against 48 KB: -0.7 to
// -1.7 % at config 2, -0.25 % at d = 32; the stage margin of 448 keys puts
// k = 100 on CAP 1024 there). d = 256 spills with 64-KB stages.
constexpr int kStageBytesNarrow = 57344;  // ring slot for d <= 64
// Long lists at d = 128 (CAP 2048, k > ~670): survivors are dense enough
// (k = 1000: direct stores were 16 % of wave time) that the d <= 64 staging
// pays there too (round 6: 2046 -> 2009 ms at 1M x 10M, k = 1000, lists
// identical, profiles/r06/long_staged/); its LDS area (8 waves x 4.6 KB) fits
// beside two 56-KB slots (7 tiles) instead of 72-KB ones.
constexpr bool long_staged(int w, int cap) { return w == 128 && cap == 2048; }
constexpr int kStageBytesLong = 57344;
constexpr int stage_bytes_for(int w, int cap) {
  return long_staged(w, cap) ? kStageBytesLong
       : w == 128 ? DR_STAGE_BYTES_WIDE : (w <= 64 ? kStageBytesNarrow : kStageBytesOther);
}
constexpr int kRingNarrow = 2;  // ring slots for d <= 64
constexpr int ring_for(int w) { return w == 128 ? kRingWide : (w <= 64 ? kRingNarrow : kRingOther); }

template <int D, int CAP>  // D = W, the row's width in bf16 units (row bytes / 2)
struct TileGeom {
  static constexpr int WAVES = waves_for(D);
  static constexpr int THREADS = WAVES * 64;
  static constexpr int STAGE_BYTES = stage_bytes_for(D, CAP);  // one LDS ring slot
  static constexpr int RING = ring_for(D);                // slots (RING - 1 stages in flight)
  static constexpr int LPT = STAGE_BYTES / 16 / THREADS;  // LDS-DMA per thread per stage
  static constexpr int KSTEPS = D / 16;                 // MFMA k-steps per row
  static constexpr int CPR = D / 8;                     // 16-B chunks per row
  static constexpr int TILE_BYTES = kTileItems * D * 2;
  static constexpr int SR = STAGE_BYTES / TILE_BYTES;   // row tiles per stage
  static_assert(LPT >= 1 && STAGE_BYTES % (16 * THREADS) == 0, "stage geometry");
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
constexpr int nut_for(int w) {
  return w >= 512 ? 1 : (w >= 256 ? 2 : (w <= 64 ? kNutNarrow : kNutWide));
}
constexpr int ngroup_for(int w) { return nut_for(w) > 4 ? nut_for(w) / 2 : nut_for(w); }
template <int V>
struct IC {
  static constexpr int value = V;
};
// f(IC<I>{}), f(IC<I + 1>{}), ..., f(IC<N - 1>{}): compile-time indices for
// register arrays (a runtime index would put them in scratch)
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<I + 1, N>(f);
  }
}

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
template <int N>
__device__ __forceinline__ void lds_waitn(u32x4& v) {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%c1)" : "+v"(v) : "i"(N) : "memory");
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

// Wave-uniform 64-bit value, forced into SGPRs.
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
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
template <int D, int CAP>
__device__ __forceinline__ void issue_stage(const char* __restrict__ I, int64_t n_items,
                                            int64_t row0, uint32_t lds_stage) {
  using G = TileGeom<D, CAP>;
  constexpr int ROWS = G::SR * kTileItems;
  uint32_t tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = (int)(tid & 63u);
  const int wave = (int)(__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
  // readfirstlane: the base is wave-uniform; the asm takes it as an SGPR pair
  const char* base = reinterpret_cast<const char*>(uni64((int64_t)(I + row0 * (2 * D))));
  const int64_t left = n_items - 1 - row0;
  const int rmax = left < ROWS - 1 ? (int)left : ROWS - 1;
#pragma unroll
  for (int j = 0; j < G::LPT; ++j) {
    const int wave_first = j * G::THREADS + wave * 64;  // wave-uniform chunk index
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

// Max of a lane's 16 scores of one user tile, as a VALUE (stored in keys):
// IEEE maxNum, NaN scores ignored; hipcc forms v_max3_f32 from the chain, with
// canonicalising copies of the MFMA results in front (10 VALU per tile).
__device__ __forceinline__ float max16(const f32x16& a) {
  float m = a[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) m = fmaxf(m, a[r]);
  return m;
}

// The hot test's max: IEEE-754-2019 maximum (gfx950 v_maximum3_f32: NaN
// propagates, no operand canonicalisation), 8 VALU per tile instead of 10.
// Only ever compared through hot(): a NaN max counts as a hit, so the exact
// per-score tests behind it see the tile (NaN scores are never admitted there,
// as with maxNum, where they were skipped by the max).
__device__ __forceinline__ float hot_max16(const f32x16& a) {
  float m = __builtin_elementwise_maximum(a[0], a[1]);
#pragma unroll
  for (int r = 2; r < 16; ++r) m = __builtin_elementwise_maximum(m, a[r]);
  return m;
}
// "some score of the tile may beat thr": a superset of `max > thr` (NaN = hit)
__device__ __forceinline__ bool hot(float m, float thr) { return !(m <= thr); }

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
//
// The buffer is streamed in chunks of 64 * P keys (P per lane) at every level
// instead of being held in registers, so the function's register footprint is
// the same for every capacity: a register-resident 2048-key buffer (CAP =
// 2048, k up to 1024) made the callee clobber so many registers that the
// caller spilled its B fragments inside the MFMA loop (5x slower tiles).
template <int P>
__device__ __noinline__ CompactResult compact_buffer_chunked(uint64_t* __restrict__ buf, int n_in, int k,
                                                     int slack, const int32_t* __restrict__ ex,
                                                     int exn, uint32_t* __restrict__ hist) {
  constexpr int CH = 64 * P;
  const int lane = dr::lane_id();
  const int nch = (n_in + CH - 1) / CH;
  wait_vmcnt<0>();  // this wave's candidate stores have landed
  auto load = [&](int c, uint64_t (&key)[P]) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int e = c * CH + lane * P + i;
      key[i] = e < n_in ? __hip_atomic_load(buf + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0ull;
    }
  };
  // pass 0: drop excluded items (zeroed in place) and count the live keys
  int total = 0;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    uint64_t key[P];
    load(c, key);
    if (exn > 0) {
#pragma unroll
      for (int i = 0; i < P; ++i)
        if (key[i] != 0ull && sorted_contains(ex, exn, (int32_t)dr::key_item(key[i]))) {
          key[i] = 0ull;
          buf[c * CH + lane * P + i] = 0ull;
        }
    }
#pragma unroll
    for (int i = 0; i < P; ++i) total += __popcll(__ballot(key[i] != 0ull));
  }
  if (exn > 0) wait_vmcnt<0>();  // the zeroed slots are visible to the passes below
  uint64_t lo = 1ull;  // keep keys >= lo (key 0 = empty slot)
  CompactResult res{total, -INFINITY};
  if (total > k + slack) {
    uint64_t pfx = 0ull;
    int need = k, above = 0, inb = total;
    for (int shift = 56; shift >= 0; shift -= 8) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hist[lane * 4 + j] = 0u;
      wave_lds_sync();
#pragma unroll 1
      for (int c = 0; c < nch; ++c) {
        uint64_t key[P];
        load(c, key);
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const bool in = key[i] != 0ull &&
                          (shift == 56 || (key[i] >> (shift + 8)) == (pfx >> (shift + 8)));
          if (in) atomicAdd(&hist[(uint32_t)(key[i] >> shift) & 255u], 1u);
        }
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
      if (above + inb <= k + slack) break;
    }
    lo = pfx;
    res.kept = above + inb;
    res.thr = dr::key_score(pfx);                // smallest score with the kept prefix
    if (res.thr != res.thr) res.thr = -INFINITY;  // prefix below -FLT_MAX decodes to NaN
  }
  // write the kept keys back densely (order is irrelevant), chunk by chunk: a
  // chunk is in registers before any of its slots is overwritten, and the
  // write cursor never passes the start of the next chunk
  int base = 0;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    uint64_t key[P];
    load(c, key);
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const bool keep = key[i] >= lo;  // lo >= 1 also drops empty keys
      const uint64_t bal = __ballot(keep);
      if (keep) buf[base + lane_prefix(bal)] = key[i];
      base += __popcll(bal);
    }
  }
  wait_vmcnt<0>();
  return res;
}

// The same with the whole buffer (<= 64 * P keys) resident in registers:
// the CAP = 512 scans (k <= 224), whose footprint this exact code fixes
// (the chunked form measured slower at d = 64, and letting it keep chunk 0
// in registers spilled the d = 64 tile loop).
template <int P>
__device__ __noinline__ CompactResult compact_buffer_resident(uint64_t* __restrict__ buf, int n_in, int k,
                                                     int slack, const int32_t* __restrict__ ex,
                                                     int exn, uint32_t* __restrict__ hist) {
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
  if (total > k + slack) {
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
      if (above + inb <= k + slack) break;
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

// One k-step (one 16-B A fragment per lane) against NG user tiles.
//   bf16: one v_mfma_f32_32x32x16_bf16 per tile (lane (col, h) holds row col,
//         k = 16s + 8h .. +7).
//   fp32: the same 16 B are four floats k = 8s + 4h + j, j = 0..3; four
//         v_mfma_f32_32x32x2_f32 per tile, MFMA j summing k = 8s + j and
//         8s + 4 + j over the two lane halves. The user fragment holds the
//         same k, so every product of the row pair is taken once. The result
//         is an exact fp32 fmaf chain (cdna_hip_programming.md, FP32-input MFMA).
template <bool F32, int NG, int NB, int KS>
__device__ __forceinline__ void kstep_mma(const u32x4& a, const u32x4 (&bfr)[NB][KS], int g0, int s,
                                          f32x16 (&acc)[NG]) {
  if constexpr (F32) {
    const dr::f32x4 av = __builtin_bit_cast(dr::f32x4, a);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        const dr::f32x4 bv = __builtin_bit_cast(dr::f32x4, bfr[g0 + ut][s]);
        acc[ut] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[j], acc[ut], 0, 0, 0);
      }
  } else {
#pragma unroll
    for (int ut = 0; ut < NG; ++ut)
      acc[ut] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                        __builtin_bit_cast(bf16x8, bfr[g0 + ut][s]),
                                                        acc[ut], 0, 0, 0);
  }
}

struct TopkArgs {
  const char* U;  // user table rows: W * 2 bytes each
  const int64_t* user_ids;
  int64_t n_users;
  int64_t n_users_pad;  // n_ublocks * UPWG: candidate buffers exist for padded users too
  const char* I;  // item slice rows: W * 2 bytes each
  int64_t n_items;
  int64_t item_base;
  int k;
  const int64_t* excl_rowptr;
  const int32_t* excl_items;
  // Units (one workgroup pass each; DESIGN.md §3.1 "grid tail"): the first
  // n_head user blocks scan the whole catalog in one unit; each of the other
  // n_ublocks - n_head ("tail") blocks is split into tail_chunks catalog chunks
  // of chunk_items rows, so the last round of a grid of whole-catalog units
  // does not leave CUs idle. Chunk 0 of every block uses the user's buffer
  // row = its position; chunk j >= 1 of tail block b uses row n_users_pad +
  // ((j - 1) * n_tail + b - n_head) * UPWG + (position within the block).
  int64_t n_ublocks;
  int64_t n_head;
  int tail_chunks;
  int64_t chunk_items;  // multiple of the stage's item count
  int end_keep;         // tail chunk units compact buffers above this count at their end
  int head_keep;        // whole-catalog units compact buffers above this count at their end (0: none)
  int slack;            // keys a compaction keeps beyond k (kSlack; smaller for sample scans)
  int gap;              // new keys a buffer takes past k + slack before it is compacted
  const float* init_thr;  // [n_users_pad] starting thresholds (SEEDED scans only)
  // Second-tier rescan only (dev_split > 0): the user count is on the device,
  // so the grid's units are planned there: every user block is split into up
  // to dev_split catalog chunks (dev_split_plan), chunk buffers past the
  // blocks' chunk-0 rows, bounded by buf_blocks user blocks of buffer rows.
  int dev_split;
  int64_t buf_blocks;
  // Sample scans of the guessed thresholds (the GMAX instantiation): a user
  // keeps only the MAX of its 32 scores of a tile (one key per tile) instead of
  // every score above the threshold. The k-th best tile max is a lower bound
  // of the k-th best score (the best k tiles' maxima are k distinct items), so
  // the guessed threshold stays a valid lower bound — it only drops below the
  // exact sample rank when two of the best k sample items share a tile
  // (~k^2 / (2 S / 32) of users; the tile-transposed sample puts samples T
  // apart in a tile) — while the survivor stream of a scan from -inf shrinks
  // up to 32-fold. Keys name the tile (its row base), not an item: only their
  // scores are read.
  //   gmax == 2 (dense tile maxima, ks <= kDenseMaxKs): no keys, no
  //   counters, no compaction: every (user, tile) maximum is stored to
  //   tmax[(user / 32) * tmax_tiles + tile][user % 32] (one 128-B line per
  //   job), and topk_threshold_dense_kernel ranks each user's column. The
  //   compaction path paid one serialized buffer round trip per user when
  //   every user's buffer filled in the same stage (the whole workgroup
  //   waits at the next ring barrier).
  int gmax;
  float* tmax;
  int64_t tmax_tiles;
  // Small catalogs (round 6): the plan made CAP >= n_items, so every key of
  // the unit fits its buffer and nothing is ever compacted (keep_all = 1):
  // the finalize sorts all of them. An unseeded scan of a short catalog
  // otherwise compacted each user's buffer several times from -inf, serially
  // per wave, while the catalog's few tiles left the MFMA idle.
  int keep_all;
  // Fallback rescan only: the user count lives on the device (n_users and
  // n_ublocks above are its upper bounds), and pos_map[p] is the caller's
  // position of list entry p (its exclusion row). NULL otherwise.
  const int32_t* n_users_dev;
  const int64_t* pos_map;
  uint64_t* cand;  // [buffer rows][CAP] keys (unsorted)
  int32_t* cnt;    // [buffer rows] valid keys per buffer
  uint64_t* diag;  // [gridDim.x * waves][kDgSlots] in DR_TOPK_DIAG builds
};

// Chunking of a second-tier rescan, computed where the failing-user count is
// (on the device; the scan and its finalize compute the same plan): nb user
// blocks share `grid` workgroups, so each block's catalog is split into
// c ~ grid / nb chunks (at most max_c, at least min_chunk rows each, and no
// more chunk buffers than buf_blocks blocks of rows hold); chunk length is a
// whole number of stages.
struct DevSplit {
  int chunks;
  int64_t chunk_items;
};
__host__ __device__ inline DevSplit dev_split_plan(int64_t nb, int64_t grid, int max_c,
                                                   int64_t buf_blocks, int64_t n_items,
                                                   int64_t stage_items) {
  constexpr int64_t kMinChunk = 16384;
  int64_t c = nb > 0 ? grid / nb : 1;
  c = c < max_c ? c : max_c;
  const int64_t by_buf = nb > 0 ? buf_blocks / nb : 1;
  c = c < by_buf ? c : by_buf;
  const int64_t by_len = n_items / kMinChunk;
  c = c < by_len ? c : by_len;
  if (c < 1) c = 1;
  int64_t per = (n_items + c - 1) / c;
  per = (per + stage_items - 1) / stage_items * stage_items;
  DevSplit d;
  d.chunk_items = per;
  d.chunks = (int)((n_items + per - 1) / per);
  return d;
}

template <int W, int CAP, bool SEEDED, bool F32, bool GMAX = false>
__global__ __launch_bounds__(waves_for(W) * 64, waves_for(W) / 4) void score_scan_kernel(TopkArgs a) {
  static_assert(!(GMAX && SEEDED), "tile-max scans are the (unseeded) sample scans");
  constexpr int D = W;  // geometry is by row bytes: an fp32 row of d is a bf16 row of 2d
  using G = TileGeom<D, CAP>;
  constexpr int NU_T = nut_for(D);
  constexpr int NG = ngroup_for(D);  // user tiles per accumulator group
  constexpr int NGRP = NU_T / NG;    // groups scored against each item tile
  static_assert(NGRP * NG == NU_T && NGRP <= 2, "user tile groups");
  constexpr int KS = G::KSTEPS;
  constexpr int SR = G::SR;
  constexpr int UPW = NU_T * 32;      // users per wave
  constexpr int kWaves = G::WAVES;
  constexpr int UPWG = UPW * kWaves;  // users per workgroup
  constexpr int P = 8;                // keys per lane per compaction chunk (any CAP)
  constexpr int kRing = G::RING;
  constexpr int kStageBytes = G::STAGE_BYTES;
  constexpr int kLpt = G::LPT;
  constexpr int RING_BYTES = kRing * kStageBytes;
  // per wave: per-user key counts, radix histogram, staged survivor blocks
  // (16 scores + one 8-B record: tile | slot | h, threshold)
  constexpr bool STAGED = D <= 64 || long_staged(D, CAP);
  constexpr int SB = STAGED ? kStageBlocks : 0;
  // stage_hits resolves a full stage area, then stages up to 64 lanes of one
  // user tile: the area must hold a whole wave's worth of blocks
  static_assert(!STAGED || SB >= 64, "staging area smaller than a wave");
  static_assert(!STAGED || NU_T * 32 <= 256, "staged slot field is 8 bits");
  // The compaction's radix histogram (1 KB) shares the staging area: it is
  // used only by check_compact, which runs after resolve() has emptied the
  // staged blocks (stage ends, unit end).
  constexpr int STAGE_AREA = SB * (64 + 8);
  constexpr int WAVE_BYTES = UPW * 4 + (STAGE_AREA > 1024 ? STAGE_AREA : 1024);
  static_assert(RING_BYTES + kWaves * WAVE_BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[RING_BYTES + kWaves * WAVE_BYTES];

  // A buffer is compacted once it holds more than flush_at keys; a stage adds
  // at most MARGIN keys per user, so flush_at + MARGIN <= CAP. A small gap
  // above k + kSlack keeps the thresholds close to the running k-th score.
  // Unseeded scans start at -inf: every score of the first stages is a
  // survivor until the first compaction sets a real threshold.
  int flush_at = a.k + a.slack + a.gap;
  flush_at = flush_at < CAP - G::MARGIN ? flush_at : CAP - G::MARGIN;
  if (a.keep_all) flush_at = 0x7fffffff;  // at most n_items <= CAP keys per buffer

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int col = lane & 31;
  char* wbase = smem + RING_BYTES + wave * WAVE_BYTES;
  uint32_t* ucnt = reinterpret_cast<uint32_t*>(wbase);
  uint32_t* hist = reinterpret_cast<uint32_t*>(wbase + UPW * 4);
  float* blk_val = reinterpret_cast<float*>(wbase + UPW * 4);  // [SB][16], 16-B aligned
  // [SB] {tile within the stage | slot << 8 | h << 16, threshold bits}: one
  // ds_write_b64 per staged lane. A stage's blocks are always resolved before
  // the next stage begins (stage end, or an overflow inside the stage), so
  // the tile is named relative to the stage's first tile (stage_t0; SR <= 255
  // tiles): no bound on the catalog length
  uint2* blk_meta = reinterpret_cast<uint2*>(blk_val + SB * 16);
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
  int64_t n_head = a.n_head < n_ublocks ? a.n_head : n_ublocks;
  int tail_chunks = a.tail_chunks;
  int64_t chunk_items = a.chunk_items, pad_rows = a.n_users_pad;
  if (a.dev_split > 0) {  // second-tier rescan: every failing block split over the grid
    const DevSplit ds = dev_split_plan(n_ublocks, gridDim.x, a.dev_split, a.buf_blocks, a.n_items,
                                       (int64_t)SR * kTileItems);
    n_head = 0;
    tail_chunks = ds.chunks;
    chunk_items = ds.chunk_items;
    pad_rows = n_ublocks * UPWG;
  }
  const int64_t n_tail = n_ublocks - n_head;
  const int64_t n_units = n_head + n_tail * tail_chunks;
  for (int64_t unit = blockIdx.x; unit < n_units; unit += gridDim.x) {
    DG_T0(t_pro);
    int64_t ub, i_beg = 0, i_end = a.n_items, brow;
    bool chunked = false;  // a tail chunk unit: compacted down to end_keep at its end
    if (unit < n_head) {
      ub = unit;
      brow = ub * UPWG;
    } else {
      const int64_t idx = unit - n_head;
      const int64_t j = idx / n_tail, tb = idx % n_tail;
      ub = n_head + tb;
      i_beg = j * chunk_items;
      i_end = i_beg + chunk_items < a.n_items ? i_beg + chunk_items : a.n_items;
      brow = j == 0 ? ub * UPWG : pad_rows + ((j - 1) * n_tail + tb) * UPWG;
      chunked = tail_chunks > 1;
    }
    const int ntiles = i_end > i_beg ? (int)((i_end - i_beg + kTileItems - 1) / kTileItems) : 0;
    const int nst = (ntiles + SR - 1) / SR;
    const int64_t upos0 = ub * UPWG + (int64_t)wave * UPW;  // first user position of the wave
    const int64_t brow0 = brow + (int64_t)wave * UPW;      // its first buffer row
    // the unit's last compaction test: a chunk of a split tail block keeps at
    // most end_keep keys per user, so the finalize gathers a bounded count
    const int keep = chunked ? a.end_keep : a.head_keep;
    const int last_lim = (keep > 0 && keep < flush_at) ? keep : flush_at;
    uint64_t* cbase = a.cand + (size_t)brow0 * CAP;
    // dense tile maxima (gmax == 2): the 32 floats of user tile u, tile t of
    // the unit (unit slices start on tile boundaries; a partial tile's rows
    // past the slice end repeat its last row, so its max is still one of its
    // own items' scores)
    auto dense_tmax = [&](int u, int t) -> float* {
      return a.tmax + ((size_t)((upos0 >> 5) + u) * (size_t)a.tmax_tiles +
                       (size_t)((i_beg >> 5) + t)) * 32;
    };

    // Resident B fragments: lane holds user (ut*32+col), k = 16s + 8h .. +7.
    u32x4 bfr[NU_T][KS];  // bf16x8 (bf16 tables) or f32x4 (fp32 tables) per k-step
    float thr[NU_T];
#pragma unroll
    for (int ut = 0; ut < NU_T; ++ut) {
      const int64_t pos = upos0 + ut * 32 + col;
      int64_t row = 0;
      if (pos < n_users) row = a.user_ids ? a.user_ids[pos] : pos;
      const uint4* src = reinterpret_cast<const uint4*>(a.U + row * (2 * D) + 16 * h);
#pragma unroll
      for (int s = 0; s < KS; ++s) bfr[ut][s] = __builtin_bit_cast(u32x4, src[2 * s]);
      thr[ut] = SEEDED ? (pos < n_users ? a.init_thr[pos] : INFINITY) : -INFINITY;
    }
    // Retire those loads where the compiler can see it (else it waits for them
    // inside the loop, draining the ring).
    wait_vmcnt<0>();
    for (int s = lane; s < UPW; s += 64) ucnt[s] = 0;
    int stage_t0 = 0;   // first tile of the stage being scanned (staged blocks are relative to it)
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
        kstep_mma<F32, NG>(af[s], bfr, g0, s, acc);
      }
    };

    // -------------------------------------------------------------- cold paths
    auto compact = [&](int ut, int c, int n_in, int slack) {
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
      CompactResult r;
      if constexpr (CAP <= 64 * P)
        r = compact_buffer_resident<CAP / 64>(cbase + (size_t)slot * CAP, n_in, a.k, slack, ex,
                                              exn, hist);
      else
        r = compact_buffer_chunked<P>(cbase + (size_t)slot * CAP, n_in, a.k, slack, ex, exn,
                                      hist);
      vm_done = vmc;
      if (lane == 0) ucnt[slot] = (uint32_t)r.kept;
      wave_lds_sync();
#pragma unroll
      for (int u2 = 0; u2 < NU_T; ++u2)
        if (u2 == ut && col == c) thr[u2] = fmaxf(thr[u2], r.thr);  // both bounds are valid
      DG_ADD(kDgFlush, t_f);
      DG_CNT(kDgNFlush);
    };

    // buffers above lim are compacted down to k + slack keys
    auto check_compact = [&](int lim, int slack) {
#pragma unroll
      for (int ut = 0; ut < NU_T; ++ut) {
        const uint32_t c_cnt = ucnt[ut * 32 + col];
        uint64_t need = __ballot(c_cnt > (uint32_t)lim) & 0xffffffffull;
        while (need) {
          const int c = __builtin_ctzll(need);
          need &= need - 1;
          compact(ut, c, __builtin_amdgcn_readlane((int)c_cnt, c), slack);
        }
      }
    };

    // -------------------------------------------------------------- epilogues
    // Hot test (branch-free): per user tile, a 16-way max against the threshold.
    // The per-tile ballots are the v_cmp results themselves (SGPR pairs); their
    // OR is the one uniform branch of the common no-hit case.
    auto any_hits = [&](f32x16 (&acc)[NG], uint64_t (&hb)[NG], auto GI) -> uint64_t {
      constexpr int g0 = decltype(GI)::value * NG;
      uint64_t any = 0ull;
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        hb[ut] = __ballot(hot(hot_max16(acc[ut]), thr[g0 + ut]));
        any |= hb[ut];
      }
      return any;
    };

    // Append survivors straight to their users' candidate buffers in HBM: one
    // key per lane per round, its slot from the user's LDS key counter. No
    // call and no queue in the hot loop, so nothing forces the accumulators
    // and B fragments out of registers. A stage adds at most MARGIN keys per
    // user, so a buffer compacted at the stage end never overflows.
    auto enqueue = [&](int t, f32x16 (&acc)[NG], const uint64_t (&hb)[NG], auto GI) {
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
        if (hb[ut] == 0ull) continue;
        uint32_t mask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) mask |= (acc[ut][r] > thr[g0 + ut] ? 1u : 0u) << r;
        mask &= vmask;
        const int slot = (g0 + ut) * 32 + col;
        uint64_t* ubuf = cbase + (size_t)slot * CAP;  // this lane's user buffer
        // Common case: every hitting lane holds ONE survivor. It is then the
        // lane's maximum (all other scores are <= thr < it), so one round
        // stores it without the 16-way value select. Full tiles only (the
        // max of a partial tile may sit in a row past the slice end).
        if (vmask == 0xffffu && __ballot((mask & (mask - 1u)) != 0u) == 0ull) {
          if (__ballot(mask != 0u) != 0ull) {
            float m = max16(acc[ut]);
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
      stage_t0 = st * SR;
      if (vs[0] > vm_done) wait_vmcnt_dyn(vmc - vs[0]);
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int i = 0; i + 1 < kRing - 1; ++i) vs[i] = vs[i + 1];
      if (st + kRing - 1 < nst) {
        issue_stage<D, CAP>(a.I, a.n_items, i_beg + (int64_t)(st + kRing - 1) * SR * kTileItems,
                       lds_ring + ((st + kRing - 1) % kRing) * kStageBytes);
        vmc += kLpt;
      }
      vs[kRing - 2] = vmc;
      DG_ADD(kDgBoundary, t_b);
      DG_CNT(kDgNStages);
    };
    for (int st = 0; st < kRing - 1 && st < nst; ++st) {
      issue_stage<D, CAP>(a.I, a.n_items, i_beg + (int64_t)st * SR * kTileItems,
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
    static_assert(SR <= 255, "stage-relative tile field is 8 bits");
    // BATCHED: the stage-end form (accumulators dead there); the in-loop
    // overflow call keeps the light per-score form, whose few registers fit
    // beside the live accumulators
    auto resolve = [&](auto BATCHED) {
      DG_T0(t_d);
      wave_lds_sync();
#pragma unroll 1
      for (int b0 = 0; b0 < nblk; b0 += 64) {
        const int i = b0 + lane;
        const bool live = i < nblk;
        const int ii = live ? i : 0;
        const uint2 meta = blk_meta[ii];
        const uint32_t tl = (uint32_t)stage_t0 + (meta.x & 0xffu);  // tile of the unit
        const uint32_t slot = (meta.x >> 8) & 0xffu;
        const int hh = (int)((meta.x >> 16) & 1u);
        const float th = __uint_as_float(meta.y);
        const int64_t row0 = i_beg + (int64_t)tl * kTileItems;
        const uint32_t gb = (uint32_t)(a.item_base + row0);
        const int64_t left = i_end - row0;  // rows past the slice end are not scores
        const int vld = live ? (left < kTileItems ? (int)left : kTileItems) : 0;
        uint64_t* ubuf = cbase + (size_t)slot * CAP;
        const float4* src = reinterpret_cast<const float4*>(blk_val + ii * 16);
        if constexpr (decltype(BATCHED)::value != 0) {
        // One pass over the block's 16 scores builds the survivor mask and
        // keeps the survivor's value and row (the common case is one); ONE
        // LDS atomic per block then reserves all its slots. The per-score
        // atomics this replaces were a serial chain of LDS round trips.
        uint32_t mask = 0u;
        float hv = 0.f;
        int hr = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v4 = src[q];
          const float vq[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = j + 8 * q + 4 * hh;  // score register r = 4q + j
            const bool hit = row < vld && vq[j] > th;
            mask |= (hit ? 1u : 0u) << (4 * q + j);
            hv = hit ? vq[j] : hv;
            hr = hit ? row : hr;
          }
        }
        const uint32_t n = (uint32_t)__popc(mask);
        uint32_t pos = 0u;
        if (n) pos = atomicAdd(&ucnt[slot], n);
        // pos + n <= CAP always holds (flush_at + MARGIN <= CAP); the tests
        // keep a broken invariant from ever writing past the buffer
        if (n == 1u && pos < (uint32_t)CAP) st64(ubuf + pos, dr::make_key(hv, gb + (uint32_t)hr));
        if (__ballot(n == 1u) != 0ull) vmc += 1;
        // blocks with several survivors (rare): one store per survivor
        uint32_t rest = n > 1u ? mask : 0u;
        while (__ballot(rest != 0u) != 0ull) {
          if (rest != 0u) {
            const int r = __builtin_ctz(rest);
            rest &= rest - 1u;
            const float v = blk_val[ii * 16 + r];
            const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (pos < (uint32_t)CAP) st64(ubuf + pos, dr::make_key(v, gb + (uint32_t)row));
            ++pos;
          }
          vmc += 1;  // one store instruction (some lane had a key)
        }
        } else {
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
      }
      nblk = 0;
      wave_lds_sync();
      DG_ADD(kDgDrain, t_d);
      DG_CNT(kDgNDrain);
    };
    auto stage_hits = [&](int t, f32x16 (&acc)[NG], const uint64_t (&hb)[NG], auto GI) {
      constexpr int g0 = decltype(GI)::value * NG;
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        const uint64_t bal = hb[ut];
        if (bal == 0ull) continue;
        // the lane's hit bit straight from the ballot's SGPR pair (s_and_saveexec
        // on it; no VALU re-materialisation of the compare)
        const bool hit = __builtin_amdgcn_inverse_ballot_w64(bal);
        const int n = __popcll(bal);
        if (nblk + n > SB) resolve(IC<0>{});  // rare (a scan's first stages): few registers
        if (hit) {
          const int i = nblk + lane_prefix(bal);
          float4* dst = reinterpret_cast<float4*>(blk_val + i * 16);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            dst[q] = make_float4(acc[ut][4 * q], acc[ut][4 * q + 1], acc[ut][4 * q + 2],
                                 acc[ut][4 * q + 3]);
          blk_meta[i] = make_uint2((uint32_t)(t - stage_t0) | ((uint32_t)((g0 + ut) * 32 + col) << 8) |
                                       ((uint32_t)h << 16),
                                   __float_as_uint(thr[g0 + ut]));
        }
        nblk += n;
      }
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    // Group-max enqueue (GMAX sample scans): one key per user and tile, the
    // max of the tile's 32 scores of the user (the two half-waves' 16-score
    // maxima merged by v_permlane32_swap). It is the whole epilogue of such a
    // scan (the max is its hot test too). Lane h = 0 of a user appends its
    // key; each user's LDS counter has that one writer, so its slot is a plain
    // read and write (no atomic: one LDS round trip per user-tile group instead
    // of one atomic per hitting half-wave, which also conflicted between the
    // two halves of a user). A partial last tile (rows past the slice end
    // repeat the last row) is skipped: leaving sample rows out only lowers the
    // sample's order statistics, so the guess stays a lower bound.
    auto enqueue_gmax = [&](int t, f32x16 (&acc)[NG], auto GI) {
      constexpr int g0 = decltype(GI)::value * NG;
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      if (a.gmax != 2 && i_end - tile0 < kTileItems) return;
      float m[NG];
      uint64_t bal[NG];
      uint64_t any = 0ull;
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        const float mh = max16(acc[ut]);  // a value (stored): maxNum, NaN scores skipped
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mh), __float_as_uint(mh),
                                                         false, false);
        m[ut] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        if (a.gmax == 2) {  // dense tile maxima
          if (h == 0) dense_tmax(g0 + ut, t)[col] = m[ut];
          vmc += 1;
          continue;
        }
        bal[ut] = __ballot(h == 0 && m[ut] > thr[g0 + ut]);
        any |= bal[ut];
      }
      if (a.gmax == 2) return;
      if (any == 0ull) return;
      uint32_t pos[NG];
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) pos[ut] = bal[ut] ? ucnt[(g0 + ut) * 32 + col] : 0u;
      const uint32_t gkey = (uint32_t)(a.item_base + tile0);
#pragma unroll
      for (int ut = 0; ut < NG; ++ut) {
        if (bal[ut] == 0ull) continue;
        if ((bal[ut] >> lane) & 1ull) {
          const int slot = (g0 + ut) * 32 + col;
          ucnt[slot] = pos[ut] + 1u;
          if (pos[ut] < (uint32_t)CAP) st64(cbase + (size_t)slot * CAP + pos[ut], dr::make_key(m[ut], gkey));
        }
        vmc += 1;  // the store above issued once (some lane had a key)
      }
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    auto epilogue = [&](int t, f32x16 (&acc)[NG], auto GI) {
      // the stage-end work runs after the last group of the tile
      constexpr bool last_group = decltype(GI)::value == NGRP - 1;
      if constexpr (GMAX) {  // sample scan: tile maxima only
        enqueue_gmax(t, acc, GI);
        if (a.gmax != 2 && last_group && ((t + 1) % SR == 0 || t + 1 == ntiles))
          check_compact(flush_at, a.slack);
        return;
      }
      DG_T0(t_h);
      uint64_t hb[NG];
      const uint64_t any = any_hits(acc, hb, GI);
      DG_ADD(kDgHits, t_h);
      if constexpr (STAGED) {
        if (any != 0ull) stage_hits(t, acc, hb, GI);
        // end of a stage: resolve the staged blocks, compact full buffers
        if (last_group && ((t + 1) % SR == 0 || t + 1 == ntiles)) {
          if (nblk > 0) resolve(IC<1>{});
          check_compact(flush_at, a.slack);
        }
      } else {
        if (any != 0ull) enqueue(t, acc, hb, GI);
        // end of a stage: compact the buffers that passed flush_at
        if (last_group && ((t + 1) % SR == 0 || t + 1 == ntiles))
          check_compact(flush_at, a.slack);
      }
    };
    // -------------------------------------------------- per-user-tile pipeline
    // (rows of <= 128 bytes: the main scans and the narrow GMAX sample scans,
    // whose job test is gmax_ut): a job is one (item tile t, user tile u)
    // pair, KS k-steps into ONE accumulator (a single accumulation chain of
    // v_mfma_f32_32x32x16_bf16 issues at full rate). Jobs run t-major; job
    // (t, u) writes accumulator u % 2, and its hot test runs right after job
    // (t, u + 1)'s chain is issued, so the test's max3 chain, compare and
    // ballot issue while this wave's own next MFMAs execute (an MFMA holds the
    // SIMD's vector issue for 8 of its 32 cycles) instead of after the whole
    // group's chain has drained. A hit stages / enqueues the job before its
    // accumulator is reused two jobs later. The tile's A fragments are read
    // once (KS ds_read_b128 at the tile start) for all its NU_T jobs; the first
    // chain retires them one k-step at a time.
    // Rows of <= 128 bytes only: at d = 128 (the headline) it measured +0.4 %
    // (a chain of 8 k-steps already covers the group's hot test), and the fp32
    // d = 128 / bf16 d = 256 instances spill in the loop with it.
    constexpr bool UTP = NU_T % 2 == 0 && W <= 64;
    auto read_a = [&](int t, u32x4 (&af)[KS]) {
      const uint32_t tb = lds_ring + ((t / SR) % kRing) * kStageBytes + (t % SR) * G::TILE_BYTES;
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) af[s2] = ds_read_b128_asm(tb + a_off(s2));
    };
    auto kstep1 = [&](const u32x4& av, const u32x4& bv, f32x16 acc) -> f32x16 {
      if constexpr (F32) {
        const dr::f32x4 a4 = __builtin_bit_cast(dr::f32x4, av), b4 = __builtin_bit_cast(dr::f32x4, bv);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[j], b4[j], acc, 0, 0, 0);
        return acc;
      } else {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                       __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
      }
    };
    // the tile's first chain: fragment s retired (lgkmcnt(KS - 1 - s), the
    // fragment named "+v") right before its k-step
    auto chain_first = [&](u32x4 (&af)[KS], auto UI) -> f32x16 {
      constexpr int u = decltype(UI)::value;
      f32x16 acc = f32x16{};
      static_for<0, KS>([&](auto SI) {
        constexpr int s2 = decltype(SI)::value;
        lds_waitn<KS - 1 - s2>(af[s2]);
        acc = kstep1(af[s2], bfr[u][s2], acc);
        // keep each wait right before its k-step (hipcc would hoist the waits
        // together and wait for all but one fragment before the first MFMA)
        __builtin_amdgcn_sched_barrier(0);
      });
      return acc;
    };
    auto chain = [&](const u32x4 (&af)[KS], auto UI) -> f32x16 {
      constexpr int u = decltype(UI)::value;
      f32x16 acc = f32x16{};
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) acc = kstep1(af[s2], bfr[u][s2], acc);
      return acc;
    };
    // staged survivors of one job (d <= 64): the hitting lanes' 16 scores
    auto stage_ut = [&](int t, const f32x16& ac, uint64_t bal, auto UI) {
      constexpr int u = decltype(UI)::value;
      DG_T0(t_e);
      const bool hit = __builtin_amdgcn_inverse_ballot_w64(bal);
      const int n = __popcll(bal);
      if (nblk + n > SB) resolve(IC<0>{});  // rare (a scan's first stages): few registers
      if (hit) {
        const int i = nblk + lane_prefix(bal);
        float4* dst = reinterpret_cast<float4*>(blk_val + i * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = make_float4(ac[4 * q], ac[4 * q + 1], ac[4 * q + 2], ac[4 * q + 3]);
        blk_meta[i] = make_uint2((uint32_t)(t - stage_t0) | ((uint32_t)(u * 32 + col) << 8) | ((uint32_t)h << 16),
                                 __float_as_uint(thr[u]));
      }
      nblk += n;
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    // direct survivors of one job (d >= 128): one key per lane per round
    auto enqueue_ut = [&](int t, const f32x16& ac, auto UI) {
      constexpr int u = decltype(UI)::value;
      DG_T0(t_e);
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const int valid = (int)((i_end - tile0) < kTileItems ? (i_end - tile0) : kTileItems);
      const uint32_t gbase = (uint32_t)(a.item_base + tile0);
      uint32_t vmask = 0xffffu;  // rows past the slice end (last tile only)
      if (valid < kTileItems) {
        vmask = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) vmask |= ((r & 3) + 8 * (r >> 2) + 4 * h < valid ? 1u : 0u) << r;
      }
      uint32_t mask = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) mask |= (ac[r] > thr[u] ? 1u : 0u) << r;
      mask &= vmask;
      const int slot = u * 32 + col;
      uint64_t* ubuf = cbase + (size_t)slot * CAP;
      // every hitting lane holds ONE survivor (the common case, full tiles):
      // it is the lane's maximum, stored without a value select
      if (vmask == 0xffffu && __ballot((mask & (mask - 1u)) != 0u) == 0ull) {
        if (__ballot(mask != 0u) != 0ull) {
          const float m = max16(ac);
          if (mask != 0u) {
            const int r = __builtin_ctz(mask);
            const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
            if (pos < (uint32_t)CAP)
              st64(ubuf + pos, dr::make_key(m, gbase + (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * h)));
          }
          vmc += 1;
        }
      } else {
        while (__ballot(mask != 0u) != 0ull) {
          const bool has = mask != 0u;
          const int r = has ? __builtin_ctz(mask) : 0;
          mask &= mask - 1u;
          float v = ac[0];
#pragma unroll
          for (int q = 1; q < 16; ++q) v = (r == q) ? ac[q] : v;
          if (has) {
            const uint32_t pos = atomicAdd(&ucnt[slot], 1u);
            if (pos < (uint32_t)CAP)
              st64(ubuf + pos, dr::make_key(v, gbase + (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * h)));
          }
          vmc += 1;
        }
      }
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    // the sample scans' job (GMAX): the user's max of the tile's 32 scores
    // (enqueue_gmax's rule for one user tile)
    auto gmax_ut = [&](int t, const f32x16& ac, auto UI) {
      constexpr int u = decltype(UI)::value;
      const int64_t tile0 = i_beg + (int64_t)t * kTileItems;
      const float mh = max16(ac);  // a value (stored): maxNum, NaN scores skipped
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mh), __float_as_uint(mh),
                                                       false, false);
      const float m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      if (a.gmax == 2) {  // dense tile maxima: one 128-B store, no test
        if (h == 0) dense_tmax(u, t)[col] = m;
        vmc += 1;
        return;
      }
      const uint64_t bal = __ballot(h == 0 && m > thr[u]);
      if (bal == 0ull || i_end - tile0 < kTileItems) return;  // a partial last tile is skipped
      DG_T0(t_e);
      if (__builtin_amdgcn_inverse_ballot_w64(bal)) {
        const int slot = u * 32 + col;
        const uint32_t pos = ucnt[slot];  // one writer per user counter
        ucnt[slot] = pos + 1u;
        if (pos < (uint32_t)CAP)
          st64(cbase + (size_t)slot * CAP + pos, dr::make_key(m, (uint32_t)(a.item_base + tile0)));
      }
      vmc += 1;  // the store above issued once (some lane had a key)
      DG_ADD(kDgEnqueue, t_e);
      DG_CNT(kDgNEnqueue);
    };
    auto test_job = [&](int t, const f32x16& ac, auto UI) {
      constexpr int u = decltype(UI)::value;
      if constexpr (GMAX) {
        gmax_ut(t, ac, UI);
        return;
      }
      DG_T0(t_h);
      const uint64_t bal = __ballot(hot(hot_max16(ac), thr[u]));
      DG_ADD(kDgHits, t_h);
      if (bal == 0ull) return;
      if constexpr (STAGED) stage_ut(t, ac, bal, UI);
      else enqueue_ut(t, ac, UI);
    };
    auto stage_end_utp = [&]() {
      if constexpr (STAGED) {
        if (nblk > 0) resolve(IC<1>{});
      }
      if (GMAX && a.gmax == 2) return;  // dense tile maxima: no buffers
      check_compact(flush_at, a.slack);
    };
    if constexpr (UTP) {
      f32x16 acc0, acc1;  // job (t, u) -> acc(u % 2)
      for (int t = 0; t < ntiles; ++t) {
        DG_CNT(kDgNTiles);
        if (t % SR == 0) {
          // the previous stage's last job, then its stage-end work (every
          // job of the stage tested: at most MARGIN keys per user since the
          // last compaction), then the ring boundary
          if (t > 0) {
            test_job(t - 1, acc1, IC<NU_T - 1>{});
            stage_end_utp();
          }
          boundary(t / SR);
        }
        u32x4 af[KS];
        read_a(t, af);
        DG_T0(t_m);
        acc0 = chain_first(af, IC<0>{});
        DG_ADD(kDgMma, t_m);
        if (t % SR != 0) test_job(t - 1, acc1, IC<NU_T - 1>{});
        static_for<1, NU_T>([&](auto UI) {
          constexpr int u = decltype(UI)::value;
          DG_T0(t_m2);
          if constexpr (u % 2 == 0) acc0 = chain(af, UI);
          else acc1 = chain(af, UI);
          DG_ADD(kDgMma, t_m2);
          if constexpr (u % 2 == 0) test_job(t, acc1, IC<u - 1>{});
          else test_job(t, acc0, IC<u - 1>{});
        });
      }
      if (ntiles > 0) {
        test_job(ntiles - 1, acc1, IC<NU_T - 1>{});
        stage_end_utp();
      }
    } else {
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
    }
    // a chunk of a split tail block ends with at most end_keep keys per user,
    // a whole-catalog unit of a long-list plan with at most head_keep
    if (last_lim < flush_at && ntiles > 0) check_compact(last_lim, last_lim - a.k);
    wait_vmcnt<0>();
    wave_lds_sync();
    for (int s = lane; s < UPW; s += 64) a.cnt[(size_t)brow0 + s] = (int32_t)ucnt[s];
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

// ------------------------------------------------------------------ launch plan
struct Plan {
  int cap;
  int users_per_wg;
  int64_t n_ublocks;
  int64_t n_users_pad;
  int64_t n_head;       // user blocks scanned whole (one unit each)
  int tail_chunks;      // catalog chunks per tail block (1 = no split)
  int64_t chunk_items;  // tail chunk length
  int end_keep;         // keys a tail chunk buffer keeps at its end (0: no end compaction)
  int head_keep;        // keys a whole-catalog buffer keeps at its end (0: no end compaction)
  int slack, gap;       // compaction slack and flush gap (TopkArgs)
  int64_t buf_rows;     // candidate buffers: n_users_pad + the tail's extra chunks
  int keep_all;         // TopkArgs::keep_all: CAP >= n_items, no compaction
  int64_t all_keys;     // keep_all: the keys a buffer ends with (n_items)
  int grid;
  size_t cand_bytes;
  size_t cnt_bytes;
  int64_t head_users() const { return n_head * users_per_wg; }
};

// Launch the scan for rows of width W (bf16 units) on stream s; defined per
// dtype in score_scan_bf16.hip / score_scan_f32.hip. Returns false for a
// (W, cap) pair that has no instantiation.
bool launch_scan_bf16(const Plan& p, const TopkArgs& a, int w, bool seeded, hipStream_t s);
bool launch_scan_f32(const Plan& p, const TopkArgs& a, int w, bool seeded, hipStream_t s);

// Instantiate and launch one dtype's scan over the supported widths.
template <bool F32, int... Ws>
bool launch_scan_widths(const Plan& p, const TopkArgs& a, int w, bool seeded, hipStream_t s) {
  bool done = false;
  auto one = [&](auto WC) {
    constexpr int WW = decltype(WC)::value;
    if (done || w != WW) return;
    done = true;
#define DR_SCAN(CC, SD) \
  hipLaunchKernelGGL((score_scan_kernel<WW, CC, SD, F32>), dim3(p.grid), dim3(waves_for(WW) * 64), \
                     0, s, a)
#define DR_SCAN_GMAX(CC) \
  hipLaunchKernelGGL((score_scan_kernel<WW, CC, false, F32, true>), dim3(p.grid),               \
                     dim3(waves_for(WW) * 64),                                               \
                     0, s, a)
    if (a.gmax && !seeded) {  // sample scans (ks <= ~70 keys: CAP 512, or 1024 at narrow rows)
      if (p.cap == 512) DR_SCAN_GMAX(512);
      else if (p.cap == 1024) DR_SCAN_GMAX(1024);
      else done = false;
    } else if (p.cap == 512) {
      if (seeded) DR_SCAN(512, true); else DR_SCAN(512, false);
    } else if (p.cap == 1024) {
      if (seeded) DR_SCAN(1024, true); else DR_SCAN(1024, false);
    } else if (p.cap == 2048) {
      if (seeded) DR_SCAN(2048, true); else DR_SCAN(2048, false);
    } else {
      done = false;
    }
#undef DR_SCAN
#undef DR_SCAN_GMAX
  };
  (one(IC<Ws>{}), ...);
  return done;
}

}  // namespace dr_topk
