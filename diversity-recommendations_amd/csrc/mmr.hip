// MMR (maximal marginal relevance) diversity re-rank, config 5 of
// BASELINE.json: top-C candidates -> k_out picks per user. There is no
// reference symbol; the spec is the build's own:
//   pick_t = argmax_{i not picked} lambda * s_i - (1 - lambda) * max_{j picked} cos(e_i, e_j)
// (the max term is 0 before the first pick; ties -> lowest candidate position).
//
// Probe-batch design, one 512-thread workgroup per CU
// looping over users (persistent grid):
//   * A user's C <= 1024 candidate rows stay in registers as MFMA B fragments
//     (wave w owns positions w, w+8, ..., 4 tiles of 32): half the register
//     file, so a CU holds one user; the next user's ids, scores and tile-0
//     rows arrive by LDS-DMA while this one runs.
//   * A batch takes 64 PROBES (the 8 best live candidates of every wave by
//     the current MMR value) and BOUND, the best key outside them.
//   * Fast rounds run the greedy over the probes only, on one wave, with the
//     probes' 64 x 64 Gram: a pick is valid while it beats BOUND. Values only
//     fall once a pick exists (the max term grows), so no non-probe can
//     overtake a probe that beats BOUND: the picks are exactly the eager
//     greedy's.
//   * When no probe beats BOUND the batch ends: one MFMA pass of the batch's
//     picks against every candidate folds their cosines into the max terms.
#include <atomic>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kTiles = 4;                          // candidate tiles of 32 per wave
constexpr int kMaxC = kWaves * kTiles * 32;        // 1024

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
using dr::bf16x8;
using dr::f32x16;

// Wave-wide max of a 64-bit key through DPP (VALU lane moves, no LDS round
// trip): quad swaps, half-row and row mirrors, then the row_bcast15/31 steps
// carry the running max into lane 63. The fast rounds are a serial chain of
// these reductions, so their latency is the round time.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
  const int nlo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xF, false);
  const int nhi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xF, false);
  return ((uint64_t)(uint32_t)nhi << 32) | (uint32_t)nlo;
}
__device__ __forceinline__ uint32_t wave_min_u32_64(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xA, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  v = dr::umax64(v, dpp_u64<0xB1>(v));        // quad_perm [1,0,3,2]
  v = dr::umax64(v, dpp_u64<0x4E>(v));        // quad_perm [2,3,0,1]
  v = dr::umax64(v, dpp_u64<0x141>(v));       // row_half_mirror
  v = dr::umax64(v, dpp_u64<0x140>(v));       // row_mirror: every lane holds its row's max
  v = dr::umax64(v, dpp_u64<0x142, 0xA>(v));  // row_bcast15 into rows 1 and 3
  v = dr::umax64(v, dpp_u64<0x143, 0xC>(v));  // row_bcast31 into rows 2 and 3
  return dr::readlane_u64(v, 63);
}


// a[lane] max a[lane ^ 32] (v_permlane32_swap: one VALU, no LDS round trip)
__device__ __forceinline__ float half_swap_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Diagnostic build (-DDR_MMR_DIAG, a measurement variant library only):
// per-wave s_memtime cycles of each phase, summed over users into a device
// array that dr_mmr_diag_read copies out. Never in the product library.
#ifdef DR_MMR_DIAG
__device__ unsigned long long g_mmr_diag[kWaves][16];
#define MG_T0(v) uint64_t v = __builtin_amdgcn_s_memtime()
#define MG_ADD(slot, t0) dg[slot] += __builtin_amdgcn_s_memtime() - (t0)
#else
#define MG_T0(v) ((void)0)
#define MG_ADD(slot, t0) ((void)0)
#endif
enum { kMgLoad, kMgSelect, kMgStage, kMgMma, kMgSync1, kMgRounds, kMgSync2, kMgFold, kMgBatches,
       kMgTotal, kMgStageBar, kMgGt, kMgSlots = 16 };

// Max over the wave's 64 lanes (lanes = 64) or over lanes 0..31 (lanes = 32)
// by fused v_max_u32_dpp steps (one VALU each: the reduction is the latency
// of the serial chains below); the result is read from the last lane.
template <int LANES>
__device__ __forceinline__ uint32_t wmax_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, true));
  if constexpr (LANES == 64) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, true));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  } else {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  }
}

// ---------------------------------------------------------------------------
// Round-3 layout: MFMA work proportional to the PICKS, not to the probes.
//   * 64 probes per batch (8 per wave) instead of 32: the bound (best value
//     outside the probes) is lower, so more picks pass per batch (8 batches
//     instead of 12 for 100 picks of real top-1000 lists, simulated);
//   * the fast rounds need only the probes' pairwise cosines: a 64 x 64 Gram
//     of the staged probe rows (4 MFMA tiles on waves 0-3) instead of 32
//     columns of every candidate;
//   * wave 0 holds its lane's Gram row in registers for the rounds (an SGPR-
//     indexed register read instead of an LDS round trip per round);
//   * after the rounds, ONE MFMA pass of the batch's picks (<= 32 rows per
//     pass) against every candidate folds their columns into the max terms.
// Exactness: the fold computes acc(pick p, candidate c) * inv|c| * inv|p| from
// the same bf16 rows with the same operand roles (A = probe/pick rows from
// LDS, B = candidate row) as the Gram, so the values the rounds see for a
// probe are bit-identical to what the fold leaves in its max term: the picks
// are exactly the eager greedy's on these fp32 cosines, as before.
constexpr int kPP = 64;               // probes per batch

constexpr int kPPW = kPP / kWaves;    // per wave
typedef float f32x32 __attribute__((ext_vector_type(32)));

template <int D>
__global__ __launch_bounds__(kThreads) void mmr_pick_kernel(
    const int32_t* __restrict__ cand_items, const float* __restrict__ cand_scores, int C,
    const __bf16* __restrict__ E, int64_t n_items, int64_t n_users, int k_out, float lambda,
    int32_t* __restrict__ out_items, int32_t* __restrict__ err) {
  constexpr int KS = D / 16;  // MFMA k-steps per row
  constexpr int CPR = D / 8;  // 16-B chunks per row
  constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  constexpr int GS = kPP + 4;  // s_g row stride in floats (16-B rows, 4 banks apart)
  __shared__ uint4 s_prow[kPP * CPR];  // probe rows, chunk c of slot p at p*CPR + (c ^ (p & SWM))
  // s_g[a*GS + p] = cos(probe a, probe p) rounded as a's fold would round it
  __shared__ __attribute__((aligned(16))) float s_g[kPP * GS];
  __shared__ float s_pinv[kPP], s_pscore[kPP], s_ppen[kPP];
  __shared__ int s_pcand[kPP];   // candidate position of each probe slot (-1 = empty)
  __shared__ int s_pitem[kPP];   // its item id
  __shared__ int s_plist[kPP];   // this batch's picks: probe slots in pick order
  __shared__ __attribute__((aligned(16))) float s_lpinv[kPP];  // 1/|e| of pick i
  __shared__ int s_citem[kMaxC];
  __shared__ float s_cscore[kMaxC], s_cinv[kMaxC];  // wave-local index cidx
  __shared__ uint64_t s_wbound[kWaves];
  __shared__ int s_state[5];  // rounds done, picks this batch, picked mask lo / hi, forced pick
  __shared__ int s_out[kMaxC];
  // Prefetch of the workgroup's next user (persistent grid), by LDS-DMA while
  // this user runs: its ids and scores, and the rows of candidate tile 0 of
  // every wave (256 rows; chunk c of row r at r*CPR + (c ^ (r & SWM)))
  __shared__ int s_nitem[kMaxC];
  __shared__ float s_nscore[kMaxC];
  __shared__ uint4 s_pf[kWaves * 32 * CPR];
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto lds_addr = [](const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  };

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float mu = 1.f - lambda;
#ifdef DR_MMR_DIAG
  uint64_t dg[kMgSlots] = {};
  MG_T0(t_kernel);
#endif

  // Persistent grid: workgroup b runs users b, b + G, ...; user b + G's ids,
  // scores and tile-0 rows arrive by LDS-DMA while user b runs.
  const int64_t G = gridDim.x;
  for (int64_t u = blockIdx.x; u < n_users; u += G) {
  // lane coordinates from an opaque copy of the thread id at every user:
  // otherwise hipcc hoists per-lane addresses out of the user loop and spills
  uint32_t tl0 = threadIdx.x;
  asm volatile("" : "+v"(tl0));
  const int tid = (int)tl0, lane = tid & 63, h = lane >> 5, q = lane & 31;
  auto cpos = [&](int j) { return kWaves * (32 * j + q) + w; };
  auto cidx = [&](int j) { return w * 128 + 32 * j + q; };
  // ids and scores of user un: 2 x 16 LDS-DMA blocks of 64 words, 2 + 2 per
  // wave (entries past C repeat entry C - 1: never read)
  auto issue_ids = [&](int64_t un) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int e = (2 * w + b) * 64 + lane;
      const int64_t src = un * C + (e < C ? e : C - 1);
      const uint32_t m0i = lds_addr(s_nitem) + (uint32_t)(2 * w + b) * 256u;
      const uint32_t m0s = lds_addr(s_nscore) + (uint32_t)(2 * w + b) * 256u;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                   : : "v"(cand_items + src), "s"(m0i) : "memory", "m0");
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                   : : "v"(cand_scores + src), "s"(m0s) : "memory", "m0");
#pragma clang diagnostic pop
    }
  };
  // tile-0 rows of the next user (its ids in s_nitem): 256 * CPR 16-B chunks,
  // 64 per DMA instruction; an empty or out-of-range id loads row 0 (never used)
  auto issue_rows = [&]() {
    constexpr int PER = 32 * CPR / 64;  // instructions per wave
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int blk = w * PER + k;
      const int i = blk * 64 + lane;
      const int r = i / CPR, c = (i % CPR) ^ (r & SWM);
      const int32_t it = s_nitem[kWaves * (r & 31) + (r >> 5)];
      const int64_t row = (it >= 0 && (int64_t)it < n_items) ? it : 0;
      const __bf16* src = E + row * D + c * 8;
      const uint32_t m0 = lds_addr(s_pf) + (uint32_t)blk * 1024u;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                   : : "v"(src), "s"(m0) : "memory", "m0");
#pragma clang diagnostic pop
    }
  };
  auto wait_dma = [] { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  const bool pre = u != (int64_t)blockIdx.x;  // ids, scores and tile-0 rows prefetched
  if (pre) {
    wait_dma();
    __syncthreads();
  }
#ifdef DR_MMR_DIAG
  MG_T0(t_user);
#endif

  // ---- candidate rows -> B fragments (tile 0 from the prefetch, if any)
  bf16x8 brow[kTiles][KS];
  float pen[kTiles];
  uint32_t live = 0;
  int nbad = 0;
#pragma unroll
  for (int j = 0; j < kTiles; ++j) {
    const int c = cpos(j);
    int32_t item = c < C ? (pre ? s_nitem[c] : cand_items[u * C + c]) : -1;
    if (item >= 0 && (int64_t)item >= n_items) {
      nbad += h == 0 ? 1 : 0;
      item = -1;
    }
    const bool ok = item >= 0;
    live |= (ok ? 1u : 0u) << j;
    const float sc = ok ? (pre ? s_nscore[c] : cand_scores[u * C + c]) : 0.f;
    if (h == 0) {
      s_citem[c] = item;
      s_cscore[cidx(j)] = sc;
    }
    pen[j] = -INFINITY;
    if (j == 0 && pre) {
      const int r = w * 32 + q;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        brow[0][s] = __builtin_bit_cast(bf16x8, s_pf[r * CPR + ((2 * s + h) ^ (r & SWM))]);
    } else {
      const uint4* src = reinterpret_cast<const uint4*>(E + (int64_t)(ok ? item : 0) * D) + h;
#pragma unroll
      for (int s = 0; s < KS; ++s) brow[j][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
    }
  }
  if (nbad && err) atomicAdd(err, nbad);
#pragma unroll
  for (int j = 0; j < kTiles; ++j) {
    float nsq = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint4 v = __builtin_bit_cast(uint4, brow[j][s]);
      const uint32_t pr[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16x2 a = __builtin_bit_cast(bf16x2, pr[e]);
        nsq = __builtin_amdgcn_fdot2_f32_bf16(a, a, nsq, false);
      }
    }
    nsq += __shfl_xor(nsq, 32);
    if (h == 0) s_cinv[cidx(j)] = 1.f / sqrtf(nsq);
  }
  __syncthreads();
  MG_ADD(kMgLoad, t_user);
  const bool more = u + G < n_users;
  if (more) issue_ids(u + G);  // s_nitem / s_nscore are free from here

  // Fold the np picks of s_plist (their rows staged in s_prow, 1/|e| in
  // s_lpinv) into every candidate's max term: rows of A = the picks in pick
  // order, 32 per pass; register r of tile j holds pick i = 8 (r / 4) + 4 h + r % 4.
  auto fold = [&](int np, int h, int q) {
    auto cidx = [&](int j) { return w * 128 + 32 * j + q; };
    for (int i0 = 0; i0 < np; i0 += 32) {
      const int nrow = np - i0 < 32 ? np - i0 : 32;
      const int sq = q < nrow ? s_plist[i0 + q] : -1;
      f32x16 acc[kTiles];
#pragma unroll
      for (int j = 0; j < kTiles; ++j) acc[j] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const uint4 av = sq >= 0 ? s_prow[sq * CPR + ((2 * s + h) ^ (sq & SWM))] : uint4{0, 0, 0, 0};
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < kTiles; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, brow[j][s], acc[j], 0, 0, 0);
      }
      // 1/|pick| per register pair; NaN for rows past the picks, whose
      // products (NaN) the max ignores: no per-score select. Registers
      // 8-15 (rows 16-31) are skipped when the pass has at most 16 picks
      // (the common case: ~15 picks per batch).
      const bool upper = nrow > 16;
      f32x2 pv2[8];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const float4 v = *reinterpret_cast<const float4*>(&s_lpinv[i0 + 8 * gg + 4 * h]);
        const int r0 = 8 * gg + 4 * h;
        const float nan = __builtin_nanf("");
        pv2[2 * gg] = f32x2{r0 < nrow ? v.x : nan, r0 + 1 < nrow ? v.y : nan};
        pv2[2 * gg + 1] = f32x2{r0 + 2 < nrow ? v.z : nan, r0 + 3 < nrow ? v.w : nan};
      }
      // cos = (acc * 1/|c|) * 1/|p|, the Gram's operand order, two scores per
      // v_pk_mul_f32
#pragma unroll
      for (int j = 0; j < kTiles; ++j) {
        const float ci = s_cinv[cidx(j)];
        const f32x2 c2 = {ci, ci};
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
          const f32x2 cs = (f32x2{acc[j][r], acc[j][r + 1]} * c2) * pv2[r / 2];
          mx = fmaxf(mx, fmaxf(cs.x, cs.y));
        }
        if (upper) {
#pragma unroll
          for (int r = 8; r < 16; r += 2) {
            const f32x2 cs = (f32x2{acc[j][r], acc[j][r + 1]} * c2) * pv2[r / 2];
            mx = fmaxf(mx, fmaxf(cs.x, cs.y));
          }
        }
        pen[j] = fmaxf(pen[j], half_swap_max(mx));
      }
    }
  };

  // ---- first pick: the best live candidate by lambda * score (no max term
  // yet), found by one wave max per wave + a combine; no probes, no rounds.
  int t = 0;
  {
    uint64_t lk = 0ull;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * h + i;
      if ((live >> j) & 1u) {
        const float sc = s_cscore[cidx(j)];
        lk = dr::umax64(lk, dr::make_key(lambda * sc, (uint32_t)cpos(j)));
      }
    }
    const uint64_t wb = wave_max_u64(lk);
    if (lane == 0) s_wbound[w] = wb;
    lds_barrier();
    uint64_t best = 0ull;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) best = dr::umax64(best, s_wbound[i]);
    if (best != 0ull) {
      const int pc = (int)dr::key_item(best);
      const int pj = (pc >> 3) >> 5, pq = (pc >> 3) & 31;
      if (w == (pc & 7) && q == pq) {  // the owner lanes (both halves) stage its row
#pragma unroll
        for (int jj = 0; jj < kTiles; ++jj) {
          if (jj == pj) {
#pragma unroll
            for (int s = 0; s < KS; ++s) s_prow[(2 * s + h)] = __builtin_bit_cast(uint4, brow[jj][s]);
          }
        }
        if (h == 0) {
          s_plist[0] = 0;
          s_lpinv[0] = s_cinv[w * 128 + 32 * pj + q];
          s_out[0] = s_citem[pc];
        }
        live &= ~(1u << pj);
      }
      lds_barrier();
      fold(1, h, q);
      t = 1;
    }
    lds_barrier();  // s_wbound / s_prow are rewritten by the first batch
  }
  if (more) {  // the next user's ids are in (every wave's DMA + a barrier): its tile-0 rows
    wait_dma();
    __syncthreads();
    issue_rows();
  }
  for (int batch = 0; t < k_out && batch <= k_out; ++batch) {
    uint32_t tl = threadIdx.x;  // opaque lane coordinates: else hipcc hoists per-lane LDS offsets and spills them
    asm volatile("" : "+v"(tl));
    const int lane = (int)(tl & 63u), h = lane >> 5, q = lane & 31;
    auto cpos = [&](int j) { return kWaves * (32 * j + q) + w; };
    auto cidx = [&](int j) { return w * 128 + 32 * j + q; };
    MG_T0(t_sel);

    // ---- probes of this wave and its bound. Any probe set is exact as long
    // as the bound is the best key outside it, so the wave takes every live
    // candidate whose value beats the 9th-best value p of its 128 (at most
    // kPPW of them), found by a radix select over the 32-bit value order:
    // one ballot pair per bit, no serial argmax chain. The bound is (p, the
    // lowest position holding p). Lane (q, h) ranks tiles 2h and 2h+1 (both
    // half-waves hold the same candidates; this way each counts once).
    uint32_t v2[2];
    float r_sc[2], r_pen[2];  // the ranked candidates' score and max term (probe state)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float sc = s_cscore[w * 128 + 32 * (2 * h + i) + q];
      uint32_t o = 0u;
      float pn = 0.f;
#pragma unroll
      for (int j = 0; j < kTiles; ++j) {
        if (j == 2 * h + i) {
          pn = pen[j];
          if ((live >> j) & 1u) {
            const float val = t == 0 ? lambda * sc : fmaf(-mu, pen[j], lambda * sc);
            o = dr::f32_to_ord(val);
          }
        }
      }
      v2[i] = o;
      r_sc[i] = sc;
      r_pen[i] = pn;
    }
    // Probe threshold pthr: the wave's probes are its live values > pthr (at
    // most kPPW of them), pthr the (kPPW + 1)-th largest value, found by a
    // radix select bit by bit, both ballots of a step into their own SGPR
    // pairs (hipcc serialises them through VCC). The selection is SALU-bound
    // (the eight waves share the CU's scalar unit); skipping the live values'
    // common prefix and stopping 8 bits short measured slower (64.3 -> 65.7 ms),
    // and so did counting on the VALU (v_bcnt of the ballot halves) on waves
    // 0-3 or on every wave, which balances the waves but lengthens each step
    // (65.6 / 66.5 against 64.4 ms).
    static_assert(kPPW + 1 == 9, "the asm below counts against 8");
    auto radix_step = [&](uint32_t p, uint32_t bit) {
      uint64_t ba_, bb_;
      uint32_t c_, na_, nb_;
      asm volatile(
          "s_or_b32 %[c], %[p], %[bit]\n\t"
          "v_cmp_le_u32_e64 %[ba], %[c], %[v0]\n\t"
          "v_cmp_le_u32_e64 %[bb], %[c], %[v1]\n\t"
          "s_bcnt1_i32_b64 %[na], %[ba]\n\t"
          "s_bcnt1_i32_b64 %[nb], %[bb]\n\t"
          "s_add_u32 %[na], %[na], %[nb]\n\t"
          "s_cmp_gt_u32 %[na], 8\n\t"
          "s_cselect_b32 %[p], %[c], %[p]"
          : [p] "+s"(p), [ba] "=&s"(ba_), [bb] "=&s"(bb_), [c] "=&s"(c_), [na] "=&s"(na_),
            [nb] "=&s"(nb_)
          : [bit] "s"(bit), [v0] "v"(v2[0]), [v1] "v"(v2[1])
          : "scc");
      return p;
    };
    uint32_t pthr;
    {
      uint32_t p = 0u;  // the largest p with at least kPPW + 1 values >= p (0: fewer live)
#pragma unroll
      for (int bit = 31; bit >= 0; --bit) p = radix_step(p, 1u << bit);
      pthr = p;
    }
    const uint32_t p9 = pthr;
    const uint64_t b0 = __ballot(v2[0] > p9), b1 = __ballot(v2[1] > p9);
    const int n0 = __popcll(b0), nprobe = n0 + __popcll(b1);
    uint32_t myslot = 0u;  // per tile j: probe slot + 1 of this lane's candidate (bits 8j..)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint64_t bm = i == 0 ? b0 : b1;
      if ((bm >> lane) & 1ull) {
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0));
        const int slot = w * kPPW + (i == 0 ? 0 : n0) + rank;
        const int j = 2 * h + i;
        const int pos = kWaves * (32 * j + q) + w;
        // the probe's state, written by the lane that ranked it (its row is
        // staged below by the two lanes that hold its halves)
        s_pcand[slot] = pos;
        s_pitem[slot] = s_citem[pos];
        s_pinv[slot] = s_cinv[w * 128 + 32 * j + q];
        s_pscore[slot] = r_sc[i];
        s_ppen[slot] = r_pen[i];
        myslot |= (uint32_t)(slot + 1) << (8 * j);
      }
    }
    myslot |= (uint32_t)__shfl_xor((int)myslot, 32);  // the other half-wave holds the same rows
    if (lane < kPPW && lane >= nprobe) {
      // an empty slot: 1/|e| = 0 (and a zero row, written at staging), so its
      // Gram entries are 0 (finite) and the rounds' max terms stay finite
      // without a select
      const int sl = w * kPPW + lane;
      s_pcand[sl] = -1;
      s_pinv[sl] = 0.f;
      s_ppen[sl] = 0.f;
    }
    // the wave's bound: the best value <= pthr, at its lowest position
    uint64_t wb = 0ull;
    const uint32_t bval = p9;  // p9 itself is a value (0: fewer than kPPW + 1 live)
    if (bval != 0u) {
      uint32_t mp = 0xffffffffu;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (v2[i] == bval) {
          const uint32_t pos = (uint32_t)(kWaves * (32 * (2 * h + i) + q) + w);
          mp = pos < mp ? pos : mp;
        }
      mp = wave_min_u32_64(mp);
      wb = ((uint64_t)bval << 32) | (uint32_t)~mp;
    }
    if (lane == 0) s_wbound[w] = wb;
    MG_ADD(kMgSelect, t_sel);
    MG_T0(t_stage);
    // Staging runs after every wave's fold of the previous batch (each wave
    // folds before it selects, and the stage barrier below waits for all),
    // so probe rows, zero rows of empty slots included, are written here and
    // not during the selection: there is no barrier between a wave's fold and
    // its next selection.
    if (lane < kPPW && lane >= nprobe) {
      const int sl = w * kPPW + lane;
#pragma unroll
      for (int c = 0; c < CPR; ++c) s_prow[sl * CPR + c] = uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      const int sl = (int)((myslot >> (8 * j)) & 255u) - 1;
      if (sl >= 0) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          s_prow[sl * CPR + ((2 * s + h) ^ (sl & SWM))] = __builtin_bit_cast(uint4, brow[j][s]);
      }
    }
    MG_T0(t_sbar);
    lds_barrier();
    MG_ADD(kMgStageBar, t_sbar);
    MG_ADD(kMgStage, t_stage);
    MG_T0(t_mma);
    if (w < 4) {
      // Gram tile of waves 0-3: B columns = probes a = 32 ab + q, A rows =
      // probes p = 32 pb + 8 (r / 4) + 4 h + r % 4 (register r)
      const int pb = w & 1, ab = w >> 1;
      const int ra = 32 * pb + q, rb = 32 * ab + q;
      f32x16 g = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, s_prow[ra * CPR + ((2 * s + h) ^ (ra & SWM))]);
        const bf16x8 b = __builtin_bit_cast(bf16x8, s_prow[rb * CPR + ((2 * s + h) ^ (rb & SWM))]);
        g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, g, 0, 0, 0);
      }
      const float ci = s_pinv[rb];
      float* row = &s_g[rb * GS + 32 * pb + 4 * h];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const float4 v = *reinterpret_cast<const float4*>(&s_pinv[32 * pb + 8 * gg + 4 * h]);
        const float pv[4] = {v.x, v.y, v.z, v.w};
        float4 o;
        o.x = g[4 * gg + 0] * ci * pv[0];
        o.y = g[4 * gg + 1] * ci * pv[1];
        o.z = g[4 * gg + 2] * ci * pv[2];
        o.w = g[4 * gg + 3] * ci * pv[3];
        *reinterpret_cast<float4*>(&row[8 * gg]) = o;
      }
    }
    MG_ADD(kMgGt, t_mma);
    MG_T0(t_sync1);
    lds_barrier();
    MG_ADD(kMgSync1, t_sync1);
    MG_T0(t_rounds);
    uint64_t bound = 0ull;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) bound = dr::umax64(bound, s_wbound[i]);

    // ---- fast rounds over the 64 probes on wave 0 (lane a = probe slot a).
    // The chain of a round: value -> wave max (fused v_max_f32_dpp) -> ballot
    // -> pick -> Gram entry (SGPR-indexed register read) -> max term. The
    // round's outputs are kept in registers (lane i: output i of this batch)
    // and written to LDS once after the rounds, so no LDS access, and no wait
    // on one, sits in the chain.
    if (w == 0) {
      const int pa = s_pcand[lane];
      // +0: lambda * s is never -0, so no value below is -0 either (an fma
      // with a nonzero or +0 addend), and the key order needs no -0 fix-up
      // in the chain. An empty or picked slot has lsa = -inf: its value is
      // -inf, key kDead, below every live value.
      float lsa = pa >= 0 ? lambda * s_pscore[lane] + 0.0f : -INFINITY;
      float pna = s_ppen[lane];
      f32x32 g0, g1;  // this probe's Gram row, indexed by the (uniform) pick slot
      {
        const float4* src = reinterpret_cast<const float4*>(&s_g[lane * GS]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float4 a = src[i], b = src[8 + i];
          g0[4 * i + 0] = a.x; g0[4 * i + 1] = a.y; g0[4 * i + 2] = a.z; g0[4 * i + 3] = a.w;
          g1[4 * i + 0] = b.x; g1[4 * i + 1] = b.y; g1[4 * i + 2] = b.z; g1[4 * i + 3] = b.w;
        }
      }
      // values in the key order's high word
      auto ordv = [](float v) { return __float_as_uint(v) ^ ((uint32_t)((int32_t)__float_as_uint(v) >> 31) | 0x80000000u); };
      constexpr uint32_t kDead = 0x007fffffu;  // ordv(-inf)
      const uint32_t bhi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bound >> 32));
      const uint32_t blo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bound);
      // a real bound's value is finite (bhi > kDead); bhi = 0: no candidate
      // outside the probes. A round stops at m <= bcut, except a tie with a
      // real bound that the probe wins by a lower position.
      const uint32_t bcut = bhi > kDead ? bhi : kDead;
      // t >= 1 here whenever a live candidate exists (the first pick is made
      // before the batches: values only fall from then on, which the bound
      // needs), so every live max term is finite
      uint32_t cur = ordv(fmaf(-mu, pna, lsa));
      int rec_slot = -1;  // lane i: probe slot of pick i of this batch
      const int t0 = t, nr = k_out - t;
      int np = 0;
      uint64_t picked = 0;
      uint32_t m = 0u;
      // The chain of a round: wave max (fused DPP) -> ballot -> pick -> Gram
      // entry (SGPR-indexed register read) -> max term -> key. The stop tests
      // and the tie resolution sit off the common path (one scalar compare).
      const float nmu = -mu, ninf = -INFINITY;
      for (;;) {
        // Common rounds in one asm loop: no tie, no stop test passed, list
        // not full. status 1: the list is full; 2: the slow path below
        // (m <= bcut, or equal values) with m and bal = ballot(cur == m).
        // The Gram row sits in v[2:65] (g0 then g1, contiguous by the operand
        // constraints), read by one SGPR-indexed v_mov (s_set_gpr_idx_on);
        // the pick's and the record's lane masks come from SALU shifts. Wait
        // states as hipcc schedules these pairs: 2 between a DPP source write
        // and the DPP.
        uint64_t bal, vm_, sh_;
        int status, sc_, spk_;
        float vt_, vga_, vpk_;
        asm volatile(
            "L_rt_%=:\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[cur], %[cur] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[t], %[t] quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[t], %[t] row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[t], %[t] row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[t], %[t] row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_max_u32_dpp %[t], %[t], %[t] row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "s_nop 1\n\t"
            "v_readlane_b32 %[m], %[t], 63\n\t"
            "s_cmp_le_u32 %[m], %[bcut]\n\t"
            "s_nop 0\n\t"
            "v_cmp_eq_u32_e64 %[bal], %[m], %[cur]\n\t"
            "s_cbranch_scc1 L_rs_%=\n\t"
            "s_bcnt1_i32_b64 %[c], %[bal]\n\t"
            "s_cmp_gt_u32 %[c], 1\n\t"
            "s_cbranch_scc1 L_rs_%=\n\t"
            "s_ff1_i32_b64 %[pk], %[bal]\n\t"
            "s_set_gpr_idx_on %[pk], gpr_idx(SRC0)\n\t"
            "v_mov_b32 %[ga], v2\n\t"
            "s_set_gpr_idx_off\n\t"
            "s_lshl_b64 %[sh], 1, %[pk]\n\t"
            "s_lshl_b64 %[vm], 1, %[np]\n\t"
            "v_mov_b32 %[pkv], %[pk]\n\t"
            "v_max_f32 %[pna], %[ga], %[pna]\n\t"
            "v_cndmask_b32_e64 %[lsa], %[lsa], %[ninf], %[sh]\n\t"
            "v_fma_f32 %[t], %[nmu], %[pna], %[lsa]\n\t"
            "v_ashrrev_i32 %[ga], 31, %[t]\n\t"
            "v_bitop3_b32 %[cur], %[ga], %[t], %[c80] bitop3:0x36\n\t"
            "s_or_b64 %[pkd], %[pkd], %[sh]\n\t"
            "v_cndmask_b32_e64 %[rec], %[rec], %[pkv], %[vm]\n\t"
            "s_add_u32 %[np], %[np], 1\n\t"
            "s_cmp_lt_u32 %[np], %[nr]\n\t"
            "s_cbranch_scc1 L_rt_%=\n\t"
            "s_mov_b32 %[st], 1\n\t"
            "s_branch L_re_%=\n"
            "L_rs_%=:\n\t"
            "s_mov_b32 %[st], 2\n"
            "L_re_%=:"
            : [cur] "+v"(cur), [pna] "+v"(pna), [lsa] "+v"(lsa), [rec] "+v"(rec_slot),
              [np] "+s"(np), [pkd] "+s"(picked), [st] "=s"(status), [m] "=s"(m), [bal] "=s"(bal),
              [t] "=&v"(vt_), [ga] "=&v"(vga_), [pkv] "=&v"(vpk_), [c] "=&s"(sc_),
              [pk] "=&s"(spk_), [vm] "=&s"(vm_), [sh] "=&s"(sh_)
            : [g0] "{v[2:33]}"(g0), [g1] "{v[34:65]}"(g1), [bcut] "s"(bcut), [nr] "s"(nr),
              [nmu] "v"(nmu), [ninf] "v"(ninf), [c80] "s"(0x80000000u)
            : "scc");
        if (status == 1) break;  // the list is full
        // slow path (rare): a stop test, or equal values at the top
        if (m <= bcut) {
          if (m != bhi) break;  // below a real bound, or no live probe (m = kDead)
          const uint32_t mp = wave_min_u32_64(cur == m ? (uint32_t)pa : 0xffffffffu);
          if (mp >= ~blo) break;  // the bound's candidate has the lower position
          bal = __ballot(cur == m && (uint32_t)pa == mp);
        } else {  // equal values: lowest candidate position wins
          const uint32_t mp = wave_min_u32_64(cur == m ? (uint32_t)pa : 0xffffffffu);
          bal = __ballot(cur == m && (uint32_t)pa == mp);
        }
        const int pk = __builtin_amdgcn_readfirstlane(__builtin_ctzll(bal));
        const float ga = g0[pk & 31], gb = g1[pk & 31];
        const float g = pk < 32 ? ga : gb;
        lsa = lane == pk ? -INFINITY : lsa;
        rec_slot = lane == np ? pk : rec_slot;
        picked |= 1ull << pk;
        float nx;  // max(pna, g): one v_max_f32 (no canonicalizing copies; no NaN here)
        asm("v_max_f32 %0, %1, %2" : "=v"(nx) : "v"(g), "v"(pna));
        pna = nx;
        cur = ordv(fmaf(-mu, pna, lsa));
        if (++np == nr) break;  // the list is full
      }
      t += np;
      if (lane < np) {
        s_out[t0 + lane] = s_pitem[rec_slot];
        s_plist[lane] = rec_slot;
        s_lpinv[lane] = s_pinv[rec_slot];
      }
      if (m == kDead && bhi == 0u) {  // no live candidate left: the rest are -1
        for (int i = t + lane; i < k_out; i += 64) s_out[i] = -1;
        t = k_out;
      }
      // No probe beats the bound (>= kPPW + 1 equal values at the top of
      // every wave that has one): the bound's candidate, the best key outside
      // the probes, is the next pick.
      const int forced = (np == 0 && t < k_out && (bhi | blo) != 0u) ? (int)~blo : -1;
      if (lane == 0) {
        s_state[0] = t;
        s_state[1] = np;
        s_state[2] = (int)(uint32_t)picked;
        s_state[3] = (int)(uint32_t)(picked >> 32);
        s_state[4] = forced;
      }
    }
    MG_ADD(kMgRounds, t_rounds);
    MG_T0(t_sync2);
    lds_barrier();
    t = s_state[0];
    const int np = s_state[1];
    const uint64_t picked = (uint64_t)(uint32_t)s_state[2] | ((uint64_t)(uint32_t)s_state[3] << 32);
    const int forced = s_state[4];
    MG_ADD(kMgSync2, t_sync2);
    MG_T0(t_fold);

    if (t >= k_out) break;  // the list is full: no fold, no further batch
    if (forced >= 0) {
      // the forced pick: its owner lanes stage its row as pick 0, then one fold
      const int fj = (forced >> 3) >> 5, fq = (forced >> 3) & 31;
      if (w == (forced & 7) && q == fq) {
#pragma unroll
        for (int j = 0; j < kTiles; ++j) {
          if (j == fj) {
#pragma unroll
            for (int s = 0; s < KS; ++s) s_prow[2 * s + h] = __builtin_bit_cast(uint4, brow[j][s]);
          }
        }
        if (h == 0) {
          s_plist[0] = 0;
          s_lpinv[0] = s_cinv[w * 128 + 32 * fj + q];
          s_out[t] = s_citem[forced];
        }
        live &= ~(1u << fj);
      }
      t += 1;
      lds_barrier();
      if (t >= k_out) break;
      fold(1, h, q);
    } else {
      // ---- fold: the picks (rows of A, in pick order, 32 per pass) against
      // every candidate
      fold(np, h, q);
      // picked probes of this wave leave the live set
#pragma unroll
      for (int j = 0; j < kTiles; ++j) {
        const int sl = (int)((myslot >> (8 * j)) & 255u) - 1;
        if (sl >= 0 && ((picked >> sl) & 1ull)) live &= ~(1u << j);
      }
    }
    MG_ADD(kMgFold, t_fold);
#ifdef DR_MMR_DIAG
    dg[kMgBatches] += 1;
#endif
  }
  __syncthreads();
  for (int i = tid; i < k_out; i += kThreads) out_items[u * k_out + i] = s_out[i];
  }  // users
#ifdef DR_MMR_DIAG
  MG_ADD(kMgTotal, t_kernel);
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < kMgSlots; ++i) atomicAdd(&g_mmr_diag[w][i], (unsigned long long)dg[i]);
#endif
}

#ifdef DR_MMR_DIAG
}  // namespace
// host: copy (and optionally reset) the per-wave phase totals, [8][16] u64
extern "C" int dr_mmr_diag_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mmr_diag), sizeof(g_mmr_diag)) != hipSuccess) return -1;
  if (reset) {
    static unsigned long long zero[kWaves][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_mmr_diag), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}
namespace {
#endif

// CUs of the current device (cached per device ordinal: a process may drive
// GPUs of different sizes); DR_KNOB_SCAN_SLOTS, the planner's test knob, caps
// the grid so that tests reach many users per workgroup with few users.
int grid_cus() {
  static std::atomic<int> cache[64];
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < 64) n = cache[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (dev < 0 || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                       hipSuccess || n <= 0)
      n = 256;
    if (dev >= 0 && dev < 64) cache[dev].store(n, std::memory_order_relaxed);
  }
  double v;
  if (dr::plan_knob(DR_KNOB_SCAN_SLOTS, &v) && v > 0 && (int)v < n) n = (int)v;
  return n;
}

}  // namespace

extern "C" int dr_mmr_rerank(const int32_t* cand_items, const float* cand_scores, int64_t n_users,
                             int C, const void* item_table, int64_t n_items, int d, int k_out,
                             float lambda, int32_t* out_items, int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(C >= 1 && C <= kMaxC, "C must be in [1, 1024]");
  DR_CHECK_ARG(k_out >= 1 && k_out <= C, "k_out must be in [1, C]");
  DR_CHECK_ARG(lambda >= 0.f && lambda <= 1.f, "lambda must be in [0, 1]");
  DR_CHECK_ARG(n_items >= 0 && n_items < 0x7fffffffLL, "n_items must be in [0, 2^31)");
  if (n_users == 0) return DR_OK;
  if (n_items == 0) {  // no row a candidate could name (the kernel reads row 0 for empty slots)
    dr::set_error("dr_mmr_rerank: empty item table");
    return DR_EINVAL;
  }
  DR_CHECK_ARG(cand_items && cand_scores && item_table && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  // persistent grid: one workgroup per CU (a user's rows take half the
  // register file), each looping over users and prefetching the next one
  const int cus = grid_cus();
  const dim3 grid((unsigned)(n_users < cus ? n_users : cus));
#define DR_MMR(DD)                                                                            \
  hipLaunchKernelGGL(mmr_pick_kernel<DD>, grid, dim3(kThreads), 0, s, cand_items, cand_scores,  \
                     C, (const __bf16*)item_table, n_items, n_users, k_out, lambda, out_items, err)
  switch (d) {
    case 64: DR_MMR(64); break;
    case 128: DR_MMR(128); break;
    default:
      dr::set_error("dr_mmr_rerank: d must be 64 or 128");
      return DR_EUNSUPPORTED;
  }
#undef DR_MMR
  DR_CHECK_LAUNCH();
  return DR_OK;
}
