// MMR (maximal marginal relevance) diversity re-rank, config 5 of
// BASELINE.json: top-C candidates -> k_out picks per user. There is no
// reference symbol; the spec is the build's own:
//   pick_t = argmax_{i not picked} lambda * s_i - (1 - lambda) * max_{j picked} cos(e_i, e_j)
// (the max term is 0 before the first pick; ties -> lowest candidate position).
//
// Probe-batch design. One 512-thread workgroup per user:
//   * The C <= 1024 candidate rows stay in registers as MFMA B fragments for
//     the whole user (wave w owns positions w, w+8, ..., 4 tiles of 32).
//   * A batch picks 32 PROBES: the 4 best live candidates of every wave by the
//     current MMR value, and records BOUND = the best value outside them.
//     One v_mfma_f32_32x32x16_bf16 pass gives the cosine of every candidate
//     with every probe (probe rows staged in LDS): 32 columns of the greedy's
//     similarity matrix for the price of 2 VALU rounds of the eager method.
//   * Fast rounds: the greedy runs over the probes only (their pairwise
//     cosines sit in LDS), on one wave: a pick is the argmax of the probes'
//     values, valid while it beats BOUND. Values only fall once a pick exists
//     (the max term grows), so no non-probe can overtake a probe that beats
//     BOUND: the picks are exactly the eager greedy's. No barrier per round.
//   * When a probe no longer beats BOUND (or after round 0, whose max term is
//     0), the batch ends: every candidate folds the batch's picked columns into
//     its max term and a new batch starts. ~9.6 batches for 100 picks of 1000
//     random candidates (lambda = 0.5), ~12.6 on real top-1000 lists.
// The kernel below is the round-2 layout of this design (mmr_batch_kernel).
#include "common.h"

namespace {

#ifndef DR_MMR_ALLWAVES
#define DR_MMR_ALLWAVES 0  // fast rounds on every wave instead of wave 0 + a barrier (A/B knob)
#endif
constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kTiles = 4;                          // candidate tiles of 32 per wave
constexpr int kMaxC = kWaves * kTiles * 32;        // 1024
constexpr int kProbes = 32;                        // one MFMA M dimension
constexpr int kPerWave = kProbes / kWaves;         // probes chosen by each wave

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
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
// Max / min over lanes 0..31 (rows 0 and 1), result read from lane 31.
__device__ __forceinline__ uint32_t wave_max_u32_32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xA, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
}
__device__ __forceinline__ uint32_t wave_min_u32_32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xA, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
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

// Max of a float over the wave's 64 lanes by fused v_max_f32_dpp steps (one
// VALU each), read from lane 63. -inf is the identity (bound_ctrl lanes read 0
// and are masked by the row masks of the broadcast steps only, so the input
// of every lane takes part; no NaN reaches here).
__device__ __forceinline__ float wmax_f32(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                   __builtin_bit_cast(int, v), __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false)));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

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

// Round-2 layout of the probe-batch kernel: the same probes, bound and exact
// fast rounds as mmr_probe_kernel (identical picks), rebuilt around latency:
//   * the batch's 32 similarity columns stay where the MFMAs leave them
//     (4 accumulators = 64 VGPRs per lane) instead of 128 KB of LDS; the fold
//     reads the picked columns there (constant register pattern per lane
//     half, one v_permlane32_swap per tile);
//   * probe selection ranks by the 32-bit value order (fused-DPP max, one
//     VALU per step), falling back to the exact 64-bit (value, position) key
//     only when two lanes tie on the value; the winner's owners stage its row
//     at once (the winner's tile and lane are uniform), so no probe-slot map
//     is read back from LDS;
//   * per-candidate score, 1/|e| and id live in LDS (registers hold the rows
//     and the columns).
// Out-of-range ids (>= n_items) are counted in *err and never picked.
#ifndef DR_MMR_LEGACY
#define DR_MMR_LEGACY 0  // 1: the round-2 kernel below (A/B of the round-3 rewrite only)
#endif
#if DR_MMR_LEGACY
template <int D>
__global__ __launch_bounds__(kThreads) void mmr_batch_kernel(
    const int32_t* __restrict__ cand_items, const float* __restrict__ cand_scores, int C,
    const __bf16* __restrict__ E, int64_t n_items, int k_out, float lambda,
    int32_t* __restrict__ out_items, int32_t* __restrict__ err) {
  constexpr int KS = D / 16;  // MFMA k-steps per row
  constexpr int CPR = D / 8;  // 16-B chunks per row
  constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;
  constexpr int GTS = 36;  // s_gt row stride in floats: 16-B rows, conflict-free row reads
  __shared__ uint4 s_prow[kProbes * CPR];  // probe rows, chunk c of row p at p*CPR + (c ^ (p & SWM))
  // s_gt[a*GTS + p] = cos(probe a, probe p) as candidate a's accumulator holds
  // it (the same rounding the fold applies to a's max term)
  __shared__ __attribute__((aligned(16))) float s_gt[kProbes * GTS];
  __shared__ float s_pinv[kProbes], s_pscore[kProbes], s_ppen[kProbes];
  __shared__ int s_pcand[kProbes];  // candidate position of each probe slot (-1 = empty)
  __shared__ int s_pitem[kProbes];  // its item id
  __shared__ int s_citem[kMaxC];    // candidate position -> item id
  // per-candidate score and 1/|e|, indexed wave-locally: position c at
  // cidx(c) = (c & 7) * 128 + (c >> 3), i.e. wave w, tile j, lane q at w*128 + 32j + q
  __shared__ float s_cscore[kMaxC], s_cinv[kMaxC];
  __shared__ uint64_t s_wbound[kWaves];
  __shared__ int s_round[2];  // rounds done, picked probe mask (written by wave 0)
  __shared__ int s_out[kMaxC];
  // the picks, stored to HBM once at the end
  // Barriers inside the batch loop order LDS only: a raw s_barrier after
  // lgkmcnt(0), so no wave waits there for its outstanding global stores.
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  const int64_t u = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, q = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index in an SGPR
  const float mu = 1.f - lambda;
  auto cpos = [&](int j) { return kWaves * (32 * j + q) + w; };  // this lane's position in tile j
  auto cidx = [&](int j) { return w * 128 + 32 * j + q; };      // = (cpos & 7) * 128 + (cpos >> 3)
#ifdef DR_MMR_DIAG
  uint64_t dg[kMgSlots] = {};
#endif
  MG_T0(t_kernel);

  // ---- candidate rows -> B fragments (lane: position cpos(j), k = 16s + 8h .. +7)
  bf16x8 brow[kTiles][KS];
  float pen[kTiles];  // max cosine to the picks so far (-inf before the first)
  uint32_t live = 0;
  int nbad = 0;
#pragma unroll
  for (int j = 0; j < kTiles; ++j) {
    const int c = cpos(j);
    int32_t item = c < C ? cand_items[u * C + c] : -1;
    if (item >= 0 && (int64_t)item >= n_items) {  // out of range: counted, never picked
      nbad += h == 0 ? 1 : 0;
      item = -1;
    }
    const bool ok = item >= 0;
    live |= (ok ? 1u : 0u) << j;
    const float sc = ok ? cand_scores[u * C + c] : 0.f;
    if (h == 0) {
      s_citem[c] = item;
      s_cscore[cidx(j)] = sc;
    }
    pen[j] = -INFINITY;
    const uint4* src = reinterpret_cast<const uint4*>(E + (int64_t)(ok ? item : 0) * D) + h;
#pragma unroll
    for (int s = 0; s < KS; ++s) brow[j][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
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
    nsq += __shfl_xor(nsq, 32);  // the two half-rows of the candidate
    if (h == 0) s_cinv[cidx(j)] = 1.f / sqrtf(nsq);
  }
  __syncthreads();
  MG_ADD(kMgLoad, t_kernel);

  int t = 0;
  // every batch picks at least once (its best probe beats BOUND by
  // construction), so k_out batches always suffice; the cap only bounds the
  // loop should that invariant ever break
  for (int batch = 0; t < k_out && batch <= k_out; ++batch) {
    // Lane coordinates re-derived from an opaque copy of the thread id every
    // batch: otherwise hipcc hoists dozens of per-lane LDS offsets out of the
    // loop, and with 192 VGPRs of rows + columns resident they spill (and the
    // reloads land inside the MFMA chain).
    uint32_t tl = threadIdx.x;
    asm volatile("" : "+v"(tl));
    const int lane = (int)(tl & 63u), h = lane >> 5, q = lane & 31;
    auto cpos = [&](int j) { return kWaves * (32 * j + q) + w; };
    auto cidx = [&](int j) { return w * 128 + 32 * j + q; };
    MG_T0(t_sel);

    // ---- probes: the kPerWave best live candidates of this wave + its bound.
    // Lane (q, h) ranks tiles 2h and 2h+1 (the two half-waves hold the same
    // candidates; this way each is counted once). Key = ord(value) << 32 |
    // ~position: (value desc, position asc), exact.
    uint64_t kk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float sc = s_cscore[w * 128 + 32 * (2 * h + i) + q];
      uint64_t key = 0ull;
#pragma unroll
      for (int j = 0; j < kTiles; ++j) {
        if (j == 2 * h + i && ((live >> j) & 1u)) {
          // the value every phase computes: lambda*s before the first pick,
          // then fma(-mu, pen, lambda*s)
          const float val = t == 0 ? lambda * sc : fmaf(-mu, pen[j], lambda * sc);
          key = dr::make_key(val, (uint32_t)cpos(j));
        }
      }
      kk[i] = key;
      (void)sc;
    }
    int pc[kPerWave];  // positions of this wave's probes (uniform; -1 = none)
    // per lane: probe slot + 1 of its candidate in tile j at bits 8j .. 8j+7
    uint32_t myslot = 0u;
#pragma unroll
    for (int m = 0; m <= kPerWave; ++m) {
      const uint64_t lb = dr::umax64(kk[0], kk[1]);  // this lane's best key
      const uint32_t hi = (uint32_t)(lb >> 32);
      const uint32_t mh = wmax_u32<64>(hi);  // best value (ord); 0 = no live key left
      uint64_t best = 0ull;
      if (mh != 0u) {
        const uint64_t bal = __ballot(hi == mh);
        if (__popcll(bal) == 1) best = dr::readlane_u64(lb, __builtin_ctzll(bal));
        else best = wave_max_u64(hi == mh ? lb : 0ull);  // equal values: lowest position
      }
      if (m == kPerWave) {
        if (lane == 0) s_wbound[w] = best;
        break;
      }
      const int slot = w * kPerWave + m;
      pc[m] = __builtin_amdgcn_readfirstlane(best != 0ull ? (int)dr::key_item(best) : -1);
      if (best != 0ull) {
        kk[0] = kk[0] == best ? 0ull : kk[0];
        kk[1] = kk[1] == best ? 0ull : kk[1];
        const int pj = (pc[m] >> 3) >> 5, pq = (pc[m] >> 3) & 31;
        if (q == pq) myslot |= (uint32_t)(slot + 1) << (8 * pj);
      }
      if (lane == 0) s_pcand[slot] = pc[m];
    }
    MG_ADD(kMgSelect, t_sel);
    MG_T0(t_stage);
    // the owners of each probe (lanes of its tile column, both halves) stage
    // its row and state
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      const int sl = (int)((myslot >> (8 * j)) & 255u) - 1;
      if (sl >= 0) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          s_prow[sl * CPR + ((2 * s + h) ^ (sl & SWM))] = __builtin_bit_cast(uint4, brow[j][s]);
        if (h == 0) {
          s_pitem[sl] = s_citem[cpos(j)];
          s_pinv[sl] = s_cinv[cidx(j)];
          s_pscore[sl] = s_cscore[cidx(j)];
          s_ppen[sl] = pen[j];
        }
      }
    }
    MG_T0(t_sbar);
    lds_barrier();
    MG_ADD(kMgStageBar, t_sbar);
    uint64_t bound = 0ull;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) bound = dr::umax64(bound, s_wbound[i]);
    MG_ADD(kMgStage, t_stage);
    MG_T0(t_mma);

    // ---- MFMA: dot(probe p, candidate) for the 32 probes x this wave's 128
    // candidates, four independent accumulator chains; the columns stay here
    // until the fold. Register r of tile j holds probe p(r) = 8*(r/4) + 4h + r%4.
    f32x16 acc[kTiles];
#pragma unroll
    for (int j = 0; j < kTiles; ++j) acc[j] = f32x16{};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, s_prow[q * CPR + ((2 * s + h) ^ (q & SWM))]);
#pragma unroll
      for (int j = 0; j < kTiles; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, brow[j][s], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      const float ci = s_cinv[cidx(j)];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 v = *reinterpret_cast<const float4*>(&s_pinv[8 * g + 4 * h]);
        const float pv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j][4 * g + e] = acc[j][4 * g + e] * ci * pv[e];
      }
    }
    MG_T0(t_gt);
    // the owners of probe b write row b of s_gt (their column of the batch)
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      const int sl = (int)((myslot >> (8 * j)) & 255u) - 1;
      if (sl >= 0) {
        float* row = &s_gt[sl * GTS + 4 * h];
#pragma unroll
        for (int r = 0; r < 16; ++r) row[8 * (r >> 2) + (r & 3)] = acc[j][r];
      }
    }
    MG_ADD(kMgGt, t_gt);
    MG_ADD(kMgMma, t_mma);
    MG_T0(t_sync1);
    lds_barrier();
    MG_ADD(kMgSync1, t_sync1);
    MG_T0(t_rounds);

    // ---- fast rounds over the probes: wave 0 alone (the other waves wait at
    // the batch-end barrier). Lane a < 32 holds probe a. The argmax is a 32-bit
    // max of ord(value) (fused DPP); an exact tie of values falls back to the
    // lowest candidate position, so the pick is the (value desc, position asc) max.
#if DR_MMR_ALLWAVES
    // every wave runs the (identical) rounds: t and the picked mask stay in
    // registers, so no post-round barrier or LDS broadcast is needed
    uint32_t picked = 0;
    {
#else
    if (w == 0) {
#endif
      const int pa = lane < kProbes ? s_pcand[lane] : -1;
      const int pitem = lane < kProbes ? s_pitem[lane] : -1;
      const float lsa = lambda * (lane < kProbes ? s_pscore[lane] : 0.f);
      float pna = lane < kProbes ? s_ppen[lane] : 0.f;
      const int gbase = (lane & 31) * GTS;
      const uint32_t bhi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bound >> 32));
      const uint32_t blo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bound);
      const bool first = t == 0;  // round 0 ranks without the max term: one pick, then a new batch
      bool alive = pa >= 0;
#if !DR_MMR_ALLWAVES
      uint32_t picked = 0;
#endif
      while (t < k_out) {
        const float val = first ? lsa : fmaf(-mu, pna, lsa);
        const uint32_t ov = alive ? dr::f32_to_ord(val) : 0u;  // live ords are > 0
        const uint32_t m = wmax_u32<32>(ov);
        if (m == 0u) {  // no live probe
          if ((bhi | blo) != 0u) break;
          if (w == 0 && lane == 0) s_out[t] = -1;  // no live candidate left
          ++t;
          continue;
        }
        uint64_t bal = __ballot(ov == m);
        if (__popcll(bal) > 1) {  // equal values: lowest candidate position wins
          const uint32_t mp = wave_min_u32_32(ov == m ? (uint32_t)pa : 0xffffffffu);
          bal = __ballot(ov == m && (uint32_t)pa == mp);
        }
        const int pk = __builtin_ctzll(bal);
        const uint32_t npos = ~(uint32_t)__builtin_amdgcn_readlane(pa, pk);
        if (m < bhi || (m == bhi && npos <= blo)) break;  // a non-probe may be better
        const float g = s_gt[gbase + pk];  // issued ahead of the bookkeeping
        if (w == 0 && lane == pk) s_out[t] = pitem;
        picked |= 1u << pk;
        alive = alive && lane != pk;
        ++t;
        if (first) break;
        pna = fmaxf(pna, g);
      }
#if !DR_MMR_ALLWAVES
      if (lane == 0) {
        s_round[0] = t;
        s_round[1] = (int)picked;
      }
#endif
    }
    MG_ADD(kMgRounds, t_rounds);
    MG_T0(t_sync2);
#if DR_MMR_ALLWAVES
    t = __builtin_amdgcn_readfirstlane(t);
    picked = (uint32_t)__builtin_amdgcn_readfirstlane((int)picked);
#else
    lds_barrier();
    t = s_round[0];
    const uint32_t picked = (uint32_t)s_round[1];
#endif
    MG_ADD(kMgSync2, t_sync2);
    MG_T0(t_fold);

    // ---- batch end: fold the picked columns into every candidate's max term,
    // straight from the accumulators (lane half h holds probes 8i + 4h + e)
    const uint32_t pm = picked >> (4 * h);
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if ((pm >> (8 * (r >> 2) + (r & 3))) & 1u) mx = fmaxf(mx, acc[j][r]);
      pen[j] = fmaxf(pen[j], half_swap_max(mx));
    }
    // picked probes of this wave leave the live set
#pragma unroll
    for (int j = 0; j < kTiles; ++j) {
      const int sl = (int)((myslot >> (8 * j)) & 255u) - 1;
      if (sl >= 0 && ((picked >> sl) & 1u)) live &= ~(1u << j);
    }
    lds_barrier();  // s_prow / s_gt / s_wbound / s_pcand are rewritten by the next batch
    MG_ADD(kMgFold, t_fold);
#ifdef DR_MMR_DIAG
    dg[kMgBatches] += 1;
#endif
  }
  __syncthreads();
  for (int i = tid; i < k_out; i += kThreads) out_items[u * k_out + i] = s_out[i];
#ifdef DR_MMR_DIAG
  MG_ADD(kMgTotal, t_kernel);
  if (lane == 0)
    for (int i = 0; i < kMgSlots; ++i) atomicAdd(&g_mmr_diag[w][i], (unsigned long long)dg[i]);
#endif
}
#endif  // DR_MMR_LEGACY

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
    const __bf16* __restrict__ E, int64_t n_items, int k_out, float lambda,
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
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  const int64_t u = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, q = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float mu = 1.f - lambda;
  auto cpos = [&](int j) { return kWaves * (32 * j + q) + w; };
  auto cidx = [&](int j) { return w * 128 + 32 * j + q; };
#ifdef DR_MMR_DIAG
  uint64_t dg[kMgSlots] = {};
#endif
  MG_T0(t_kernel);

  // ---- candidate rows -> B fragments (as in the round-2 kernel)
  bf16x8 brow[kTiles][KS];
  float pen[kTiles];
  uint32_t live = 0;
  int nbad = 0;
#pragma unroll
  for (int j = 0; j < kTiles; ++j) {
    const int c = cpos(j);
    int32_t item = c < C ? cand_items[u * C + c] : -1;
    if (item >= 0 && (int64_t)item >= n_items) {
      nbad += h == 0 ? 1 : 0;
      item = -1;
    }
    const bool ok = item >= 0;
    live |= (ok ? 1u : 0u) << j;
    const float sc = ok ? cand_scores[u * C + c] : 0.f;
    if (h == 0) {
      s_citem[c] = item;
      s_cscore[cidx(j)] = sc;
    }
    pen[j] = -INFINITY;
    const uint4* src = reinterpret_cast<const uint4*>(E + (int64_t)(ok ? item : 0) * D) + h;
#pragma unroll
    for (int s = 0; s < KS; ++s) brow[j][s] = __builtin_bit_cast(bf16x8, src[2 * s]);
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
  MG_ADD(kMgLoad, t_kernel);

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
      float pv[16];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const float4 v = *reinterpret_cast<const float4*>(&s_lpinv[i0 + 8 * gg + 4 * h]);
        pv[4 * gg + 0] = v.x; pv[4 * gg + 1] = v.y; pv[4 * gg + 2] = v.z; pv[4 * gg + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < kTiles; ++j) {
        const float ci = s_cinv[cidx(j)];
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (8 * (r >> 2) + 4 * h + (r & 3) < nrow) mx = fmaxf(mx, acc[j][r] * ci * pv[r]);
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
  for (int batch = 0; t < k_out && batch <= k_out; ++batch) {
    uint32_t tl = threadIdx.x;  // opaque lane coordinates (see mmr_batch_kernel)
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
    uint32_t p9 = 0u;  // largest p with at least kPPW + 1 values >= p (0: fewer live)
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t c = p9 | (1u << bit);
      const int n = __popcll(__ballot(v2[0] >= c)) + __popcll(__ballot(v2[1] >= c));
      p9 = n >= kPPW + 1 ? c : p9;
    }
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
    if (lane < kPPW && lane >= nprobe) s_pcand[w * kPPW + lane] = -1;
    uint64_t wb = 0ull;  // the wave's bound: value p9 at its lowest position among the rest
    if (p9 != 0u) {
      uint32_t mp = 0xffffffffu;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (v2[i] == p9) {
          const uint32_t pos = (uint32_t)(kWaves * (32 * (2 * h + i) + q) + w);
          mp = pos < mp ? pos : mp;
        }
      mp = wave_min_u32_64(mp);
      wb = ((uint64_t)p9 << 32) | (uint32_t)~mp;
    }
    if (lane == 0) s_wbound[w] = wb;
    MG_ADD(kMgSelect, t_sel);
    MG_T0(t_stage);
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
      const float lsa = lambda * s_pscore[lane];
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
      // values in the key order's high word: ord(v) (0 = not live)
      auto ordv = [](float v) {
        const uint32_t u = __float_as_uint(v + 0.0f);  // -0 -> +0
        return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
      };
      const uint32_t bhi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bound >> 32));
      const uint32_t blo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bound);
      // t >= 1 here whenever a live candidate exists (the first pick is made
      // before the batches: values only fall from then on, which the bound
      // needs), so every live max term is finite
      bool alive = pa >= 0;
      uint32_t cur = alive ? ordv(fmaf(-mu, pna, lsa)) : 0u;
      int rec_slot = -1;  // lane i: probe slot of pick i of this batch
      const int t0 = t, nr = k_out - t;
      int np = 0;
      uint64_t picked = 0;
      uint32_t m = 0u;
      for (;;) {
        m = wmax_u32<64>(cur);
        if (m == 0u) break;  // no live probe: a non-probe is next, or nothing is left
        uint64_t bal = __ballot(cur == m);
        if (bal & (bal - 1)) {  // equal values: lowest candidate position wins
          const uint32_t mp = wave_min_u32_64(cur == m ? (uint32_t)pa : 0xffffffffu);
          bal = __ballot(cur == m && (uint32_t)pa == mp);
        }
        const int pk = __builtin_amdgcn_readfirstlane(__builtin_ctzll(bal));
        const uint32_t npos = ~(uint32_t)__builtin_amdgcn_readlane(pa, pk);
        // stop when a non-probe may be better, or the list is full
        if (m < bhi || (m == bhi && npos <= blo) || np == nr) break;
        const float ga = g0[pk & 31], gb = g1[pk & 31];
        const float g = pk < 32 ? ga : gb;
        rec_slot = lane == np ? pk : rec_slot;
        picked |= 1ull << pk;
        ++np;
        alive = alive && lane != pk;
        pna = g > pna ? g : pna;  // a select: fmaxf would canonicalize both inputs first
        cur = alive ? ordv(fmaf(-mu, pna, lsa)) : 0u;
      }
      t += np;
      if (lane < np) {
        s_out[t0 + lane] = s_pitem[rec_slot];
        s_plist[lane] = rec_slot;
        s_lpinv[lane] = s_pinv[rec_slot];
      }
      if (m == 0u && (bhi | blo) == 0u) {  // no live candidate left: the rest are -1
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
    lds_barrier();  // LDS probe state is rewritten by the next batch
    MG_ADD(kMgFold, t_fold);
#ifdef DR_MMR_DIAG
    dg[kMgBatches] += 1;
#endif
  }
  __syncthreads();
  for (int i = tid; i < k_out; i += kThreads) out_items[u * k_out + i] = s_out[i];
#ifdef DR_MMR_DIAG
  MG_ADD(kMgTotal, t_kernel);
  if (lane == 0)
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

}  // namespace

extern "C" int dr_mmr_rerank(const int32_t* cand_items, const float* cand_scores, int64_t n_users,
                             int C, const void* item_table, int64_t n_items, int d, int k_out,
                             float lambda, int32_t* out_items, int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(C >= 1 && C <= kMaxC, "C must be in [1, 1024]");
  DR_CHECK_ARG(k_out >= 1 && k_out <= C, "k_out must be in [1, C]");
  DR_CHECK_ARG(lambda >= 0.f && lambda <= 1.f, "lambda must be in [0, 1]");
  DR_CHECK_ARG(n_items >= 0 && n_items < 0x7fffffffLL, "n_items must be in [0, 2^31)");
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(cand_items && cand_scores && item_table && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)n_users);
#if DR_MMR_LEGACY
#define DR_MMR_KERNEL mmr_batch_kernel
#else
#define DR_MMR_KERNEL mmr_pick_kernel
#endif
#define DR_MMR(DD)                                                                            \
  hipLaunchKernelGGL(DR_MMR_KERNEL<DD>, grid, dim3(kThreads), 0, s, cand_items, cand_scores,    \
                     C, (const __bf16*)item_table, n_items, k_out, lambda, out_items, err)
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
