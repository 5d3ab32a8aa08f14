// BPR training step pieces: the fused triple gather + pairwise loss + embedding
// gradient scatter of pair_wise_train_loop (reference divrec/train/utils.py:144-152)
// with LogSigmoidDifferenceLoss (divrec/losses/log_sigmoid_difference_loss.py:11-14)
// and AUCScore (divrec/metrics/auc_score.py:6-10), plus the dense Adam update
// that torch.optim.Adam applies at utils.py:151.
//
// bpr_fwd_bwd is HBM/atomic-bound: per triple it reads three fp32 rows
// (3*d*4 B), 24 B of ids, writes loss/hit, and adds 3*d*4 B of gradient with
// fp32 atomics. A group of 32 lanes owns one triple and lane l handles row
// elements l, l+32, l+64, ...: every load and every atomic wave-instruction
// then covers two contiguous 128-B row segments, the shape at which
// global_atomic_add_f32 runs at its full rate (MI355X_MICROARCH.md, Global
// float atomics); 16-B-per-lane chunks would scatter each atomic instruction
// over 16-B strides. Any d <= 512. Out-of-range ids are range-checked
// (include/divrec_hip.h): such a triple reads and adds nothing.
#include <algorithm>
#include <cmath>

#include "common.h"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// -logsigmoid(x) in torch's stable form: max(-x, 0) + log1p(exp(-|x|)).
__device__ __forceinline__ float neg_log_sigmoid(float x) {
  return fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x)));
}
// d/dx of -logsigmoid(x) = -(1 - sigmoid(x)) = -sigmoid(-x)
__device__ __forceinline__ float neg_log_sigmoid_grad(float x) {
  const float e = expf(-fabsf(x));  // in (0, 1]
  // sigmoid(-x) = x >= 0 ? e / (1 + e) : 1 / (1 + e)
  return -(x >= 0.f ? e / (1.f + e) : 1.f / (1.f + e));
}

__device__ __forceinline__ bool in_rows(int64_t r, int64_t n) { return r >= 0 && r < n; }

template <int E>  // row elements per lane: ceil(d / 32)
__global__ __launch_bounds__(kBlock) void bpr_kernel(
    const float* __restrict__ U, int64_t nu, const float* __restrict__ I, int64_t ni, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ pid,
    const int64_t* __restrict__ nid, int64_t batch, int64_t span, float grad_scale,
    float* __restrict__ loss, int32_t* __restrict__ hit, float* __restrict__ gU,
    float* __restrict__ gI, int32_t* __restrict__ err) {
  // Each 32-lane group walks a CONTIGUOUS span of triples and keeps one run
  // per table side: the current user, positive and negative rows are read
  // once per run of equal ids, and their gradient contributions are summed in
  // registers and added with ONE row of atomics when the run ends. The
  // reference's own batches are such runs (PairWiseDataset's m x m product:
  // one user for m*m triples, each positive repeated m times in a row,
  // base_datasets.py:94-107), so the atomics per triple drop from 3 rows to
  // ~1 there; uniform random triples (runs of 1) cost what they did.
  const int gl = threadIdx.x & 31;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 5;
  const int64_t b0 = group * span;
  const int64_t b1 = b0 + span < batch ? b0 + span : batch;
  int bad = 0;
  int64_t cu = -1, cp = -1, cn = -1;  // ids of the current runs (-1 = none)
  float uv[E], pv[E], nv[E];          // their rows
  float gu[E], gp[E], gn[E];          // their summed gradient contributions
#pragma unroll
  for (int e = 0; e < E; ++e) gu[e] = gp[e] = gn[e] = 0.f;
  auto load = [&](const float* tab, int64_t r, float (&v)[E]) {
    const float* row = tab + r * d;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t x = e * 32 + gl;
      v[e] = x < d ? row[x] : 0.f;
    }
  };
  auto flush = [&](float* g, int64_t r, float (&acc)[E]) {  // one row of atomics
    if (g && r >= 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t x = e * 32 + gl;
        if (x < d) atomicAdd(g + r * d + x, acc[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
  };
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t u = uid[b], p = pid[b], n = nid[b];
    if (!in_rows(u, nu) || !in_rows(p, ni) || !in_rows(n, ni)) {  // uniform in the group
      if (gl == 0) {
        if (loss) loss[b] = __builtin_nanf("");
        if (hit) hit[b] = 0;
        bad += 1;
      }
      continue;
    }
    if (u != cu) {
      flush(gU, cu, gu);
      cu = u;
      load(U, u, uv);
    }
    if (p != cp) {
      flush(gI, cp, gp);
      cp = p;
      load(I, p, pv);
    }
    if (n != cn) {
      flush(gI, cn, gn);
      cn = n;
      load(I, n, nv);
    }
    float sp = 0.f, sn = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      sp = fmaf(uv[e], pv[e], sp);
      sn = fmaf(uv[e], nv[e], sn);
    }
#pragma unroll
    for (int m = 16; m > 0; m >>= 1) {  // xor < 32 stays inside the 32-lane group
      sp += __shfl_xor(sp, m);
      sn += __shfl_xor(sn, m);
    }
    const float x = sp - sn;
    if (gl == 0) {
      if (loss) loss[b] = neg_log_sigmoid(x);
      if (hit) hit[b] = sp >= sn ? 1 : 0;
    }
    const float g = neg_log_sigmoid_grad(x) * grad_scale;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      gu[e] += g * pv[e] - g * nv[e];
      gp[e] += g * uv[e];
      gn[e] += -g * uv[e];
    }
  }
  flush(gU, cu, gu);
  flush(gI, cp, gp);
  flush(gI, cn, gn);
  if (bad && err) atomicAdd(err, bad);
}

// Dense Adam, elementwise, 4 floats per lane. Written as the same sequence of
// fp32 roundings as torch's single-tensor Adam (lerp_, mul_, addcmul_, sqrt,
// div, add_, addcdiv_), with contraction disabled so no FMA changes them.
__global__ __launch_bounds__(kBlock) void adam_kernel(float* __restrict__ param,
                                                     const float* __restrict__ grad,
                                                     float* __restrict__ m,
                                                     float* __restrict__ v, int64_t n, float w1,
                                                     float b2, float w2, float bc2_sqrt,
                                                     float neg_step, float eps, float wd) {
#pragma clang fp contract(off)
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const float p = param[i];
    float g = grad[i];
    if (wd != 0.f) g = g + wd * p;
    float mi = m[i];
    // torch lerp: weight < 0.5 ? self + weight * (end - self) : end - (end - self) * (1 - weight)
    mi = (w1 < 0.5f) ? mi + w1 * (g - mi) : g - (g - mi) * (1.f - w1);
    float vi = v[i] * b2;
    vi = vi + w2 * g * g;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    param[i] = p + neg_step * mi / denom;
    m[i] = mi;
    v[i] = vi;
  }
}

// Row-sparse ("lazy") Adam over the listed rows only: the update
// torch.optim.SparseAdam applies (torch/optim/_functional.py sparse_adam) to a
// coalesced sparse gradient whose indices are `rows`, with the values read
// from the dense gradient table the BPR kernel accumulated. Same fp32 rounding
// sequence as torch's sequence of tensor ops:
//   u1 = (g - m) * w1;  m' = m + u1
//   u2 = (g * g - v) * w2;  v' = v + u2
//   p' = p + neg_step * ((u1 + m) / (sqrt(u2 + v) + eps))
// The touched gradient entries are zeroed afterwards (zero_grad of the rows),
// so the dense gradient table never needs a full memset. One thread per
// element: rows are contiguous, so a wave covers 64 consecutive floats.
__global__ __launch_bounds__(kBlock) void adam_rows_kernel(
    float* __restrict__ param, float* __restrict__ grad, float* __restrict__ m,
    float* __restrict__ v, int64_t d, const int64_t* __restrict__ rows, int64_t n,
    float w1, float w2, float neg_step, float eps, int zero_grad) {
#pragma clang fp contract(off)
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / d;
    const int64_t e = rows[r] * d + (i - r * d);
    const float g = grad[e];
    const float mo = m[e], vo = v[e];
    const float u1 = (g - mo) * w1;
    const float u2 = (g * g - vo) * w2;
    m[e] = mo + u1;
    v[e] = vo + u2;
    const float q = (u1 + mo) / (sqrtf(u2 + vo) + eps);
    param[e] = param[e] + neg_step * q;
    if (zero_grad) grad[e] = 0.f;
  }
}

}  // namespace

extern "C" int dr_adam_rows(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                            int64_t d, const int64_t* rows, int64_t n_rows, double lr,
                            double beta1, double beta2, double eps, int64_t step, int zero_grad,
                            dr_stream_t stream) {
  DR_CHECK_ARG(n_rows >= 0 && d >= 1 && step >= 1, "n_rows must be >= 0, d >= 1, step >= 1");
  if (n_rows == 0) return DR_OK;
  DR_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && rows, "null pointer");
  // Python-float arithmetic of sparse_adam, in double, cast once:
  // step_size = lr * sqrt(1 - beta2^step) / (1 - beta1^step); mul by -step_size.
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const double step_size = lr * std::sqrt(bc2) / bc1;
  const int64_t n = n_rows * d;
  int64_t grid = dr::ceil_div(n, kBlock);
  if (grid > 256 * 16) grid = 256 * 16;
  hipLaunchKernelGGL(adam_rows_kernel, dim3((unsigned)grid), dim3(kBlock), 0,
                     (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq, d, rows, n,
                     (float)(1.0 - beta1), (float)(1.0 - beta2), (float)(-step_size), (float)eps,
                     zero_grad);
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_bpr_fwd_bwd(const float* user_table, int64_t n_user_rows,
                              const float* item_table, int64_t n_item_rows, int64_t d,
                              const int64_t* user_id, const int64_t* pos_id,
                              const int64_t* neg_id, int64_t batch, float grad_scale,
                              float* loss, int32_t* hit, float* grad_user, float* grad_item,
                              int32_t* err, dr_stream_t stream) {
  DR_CHECK_ARG(batch >= 0 && n_user_rows >= 0 && n_item_rows >= 0, "sizes must be >= 0");
  if (batch == 0) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && pos_id && neg_id, "null pointer");
  DR_CHECK_ARG(d >= 1 && d <= 512, "d must be in [1, 512]");
  hipStream_t s = (hipStream_t)stream;
  // contiguous spans of triples per 32-lane group, up to 8 workgroups per CU
  constexpr int64_t kGroups = 256 * 8 * (kBlock / 32);
  // (at least 16 per span, so runs are summed in small batches too)
  const int64_t span = std::max<int64_t>(16, dr::ceil_div(batch, kGroups));
  const int64_t grid = dr::ceil_div(dr::ceil_div(batch, span), kBlock / 32);
#define DR_BPR(EE)                                                                          \
  hipLaunchKernelGGL(bpr_kernel<EE>, dim3((unsigned)grid), dim3(kBlock), 0, s, user_table,  \
                     n_user_rows, item_table, n_item_rows, d, user_id, pos_id, neg_id, batch, \
                     span, grad_scale, loss, hit, grad_user, grad_item, err)
  switch ((int)dr::ceil_div(d, 32)) {
    case 1: DR_BPR(1); break;
    case 2: DR_BPR(2); break;
    case 3: DR_BPR(3); break;
    case 4: DR_BPR(4); break;
    case 5: DR_BPR(5); break;
    case 6: DR_BPR(6); break;
    case 7: DR_BPR(7); break;
    case 8: DR_BPR(8); break;
    case 9: case 10: case 11: case 12: DR_BPR(12); break;
    default: DR_BPR(16); break;
  }
#undef DR_BPR
  DR_CHECK_LAUNCH();
  return DR_OK;
}

extern "C" int dr_adam_dense(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t n, double lr, double beta1, double beta2, double eps,
                             double weight_decay, int64_t step, dr_stream_t stream) {
  DR_CHECK_ARG(n >= 0 && step >= 1, "n must be >= 0 and step >= 1");
  if (n == 0) return DR_OK;
  DR_CHECK_ARG(param && grad && exp_avg && exp_avg_sq, "null pointer");
  // Host-side scalars in double, then cast once, as torch does with Python floats.
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float neg_step = (float)(-(lr / bc1));
  const float bc2_sqrt = (float)std::pow(bc2, 0.5);  // Python: bias_correction2 ** 0.5
  const float w1 = (float)(1.0 - beta1);
  const float w2 = (float)(1.0 - beta2);
  int64_t grid = dr::ceil_div(n, kBlock);
  if (grid > 256 * 16) grid = 256 * 16;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)grid), dim3(kBlock), 0, (hipStream_t)stream,
                     param, grad, exp_avg, exp_avg_sq, n, w1, (float)beta2, w2, bc2_sqrt, neg_step,
                     (float)eps, (float)weight_decay);
  DR_CHECK_LAUNCH();
  return DR_OK;
}
