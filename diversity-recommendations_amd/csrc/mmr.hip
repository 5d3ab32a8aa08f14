// MMR (maximal marginal relevance) diversity re-rank, config 5 of
// BASELINE.json: top-C candidates -> k_out picks per user. There is no
// reference symbol; the spec is the build's own:
//   pick_t = argmax_{i not picked} lambda * s_i - (1 - lambda) * max_{j picked} cos(e_i, e_j)
// (the max term is 0 before the first pick; ties -> lowest candidate position).
//
// One 512-thread workgroup per user. Each thread keeps two candidate slots
// (C <= 1024) resident in registers as packed bf16 pairs, so the candidate
// rows are read from HBM exactly once per user; each greedy step is a block
// argmax plus one broadcast row (LDS) and 2*d/2 v_dot2_f32_bf16 per thread.
#include "common.h"

namespace {

constexpr int kThreads = 512;
constexpr int kSlots = 2;  // candidate slots per thread: C <= 1024

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int D>
__global__ __launch_bounds__(kThreads) void mmr_kernel(const int32_t* __restrict__ cand_items,
                                                      const float* __restrict__ cand_scores,
                                                      int C, const __bf16* __restrict__ E,
                                                      int k_out, float lambda,
                                                      int32_t* __restrict__ out_items) {
  constexpr int W = D / 2;  // packed bf16 pairs per row
  __shared__ uint32_t s_row[W];
  __shared__ float s_inv;
  __shared__ uint64_t s_best[kThreads / 64];
  __shared__ int s_pick;
  const int64_t u = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;

  uint32_t row[kSlots][W];
  float inv[kSlots], score[kSlots], maxsim[kSlots];
  bool live[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const int c = tid + s * kThreads;
    int32_t item = c < C ? cand_items[u * C + c] : -1;
    live[s] = item >= 0;
    score[s] = live[s] ? cand_scores[u * C + c] : 0.f;
    maxsim[s] = -INFINITY;
    const uint4* src = reinterpret_cast<const uint4*>(E + (int64_t)(live[s] ? item : 0) * D);
    float nsq = 0.f;
#pragma unroll
    for (int w4 = 0; w4 < W / 4; ++w4) {
      const uint4 v = src[w4];
      row[s][4 * w4 + 0] = v.x; row[s][4 * w4 + 1] = v.y;
      row[s][4 * w4 + 2] = v.z; row[s][4 * w4 + 3] = v.w;
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const bf16x2 a = __builtin_bit_cast(bf16x2, row[s][w]);
      nsq = __builtin_amdgcn_fdot2_f32_bf16(a, a, nsq, false);
    }
    inv[s] = 1.f / sqrtf(nsq);
  }

  for (int t = 0; t < k_out; ++t) {
    // Local best key: (ordered value, ~position) -> max = best value, lowest position.
    uint64_t best = 0ull;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      if (live[s]) {
        const float pen = t == 0 ? 0.f : maxsim[s];
        const float val = lambda * score[s] - (1.f - lambda) * pen;
        const uint32_t c = (uint32_t)(tid + s * kThreads);
        const uint64_t key = dr::make_key(val, c);
        best = key > best ? key : best;
      }
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      const uint64_t o = dr::shfl_xor_u64(best, m);
      best = o > best ? o : best;
    }
    if (lane == 0) s_best[wave] = best;
    __syncthreads();
    if (tid == 0) {
      uint64_t b = s_best[0];
#pragma unroll
      for (int w = 1; w < kThreads / 64; ++w) b = s_best[w] > b ? s_best[w] : b;
      const int pick = b == 0ull ? -1 : (int)dr::key_item(b);
      s_pick = pick;
      out_items[u * k_out + t] = pick < 0 ? -1 : cand_items[u * C + pick];
    }
    __syncthreads();
    const int pick = s_pick;
    if (pick < 0) continue;  // fewer live candidates than k_out (uniform)
    const int owner = pick % kThreads, oslot = pick / kThreads;
    if (tid == owner) {
#pragma unroll
      for (int s = 0; s < kSlots; ++s) {
        if (s == oslot) {
#pragma unroll
          for (int w = 0; w < W; ++w) s_row[w] = row[s][w];
          s_inv = inv[s];
          live[s] = false;
        }
      }
    }
    __syncthreads();
    const float pinv = s_inv;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      if (live[s]) {
        float dot = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w)
          dot = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, row[s][w]),
                                               __builtin_bit_cast(bf16x2, s_row[w]), dot, false);
        maxsim[s] = fmaxf(maxsim[s], dot * inv[s] * pinv);
      }
    }
    __syncthreads();  // s_row / s_best are rewritten next step
  }
}

}  // namespace

extern "C" int dr_mmr_rerank(const int32_t* cand_items, const float* cand_scores, int64_t n_users,
                             int C, const void* item_table, int64_t n_items, int d, int k_out,
                             float lambda, int32_t* out_items, dr_stream_t stream) {
  DR_CHECK_ARG(C >= 1 && C <= kThreads * kSlots, "C must be in [1, 1024]");
  DR_CHECK_ARG(k_out >= 1 && k_out <= C, "k_out must be in [1, C]");
  DR_CHECK_ARG(lambda >= 0.f && lambda <= 1.f, "lambda must be in [0, 1]");
  (void)n_items;
  if (n_users == 0) return DR_OK;
  DR_CHECK_ARG(cand_items && cand_scores && item_table && out_items, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)n_users);
  switch (d) {
    case 64:
      hipLaunchKernelGGL(mmr_kernel<64>, grid, dim3(kThreads), 0, s, cand_items, cand_scores, C,
                         (const __bf16*)item_table, k_out, lambda, out_items);
      break;
    case 128:
      hipLaunchKernelGGL(mmr_kernel<128>, grid, dim3(kThreads), 0, s, cand_items, cand_scores, C,
                         (const __bf16*)item_table, k_out, lambda, out_items);
      break;
    default:
      dr::set_error("dr_mmr_rerank: d must be 64 or 128");
      return DR_EUNSUPPORTED;
  }
  DR_CHECK_LAUNCH();
  return DR_OK;
}
