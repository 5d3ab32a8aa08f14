// BPR training step pieces: the fused triple gather + pairwise loss + embedding
// gradient scatter of pair_wise_train_loop (reference divrec/train/utils.py:144-152)
// with LogSigmoidDifferenceLoss (divrec/losses/log_sigmoid_difference_loss.py:11-14)
// and AUCScore (divrec/metrics/auc_score.py:6-10), plus the dense Adam update
// that torch.optim.Adam applies at utils.py:151.
//
// bpr_fwd_bwd is HBM/atomic-bound: per triple it reads three fp32 rows
// (3*d*4 B), 24 B of ids, writes loss/hit, and adds 3*d*4 B of gradient with
// fp32 atomics. A group of G lanes (16 B per lane) owns one triple.
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

template <int G, int CH>
__global__ __launch_bounds__(kBlock) void bpr_kernel(
    const float* __restrict__ U, const float* __restrict__ I, int64_t d,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ pid,
    const int64_t* __restrict__ nid, int64_t batch, float grad_scale, float* __restrict__ loss,
    int32_t* __restrict__ hit, float* __restrict__ gU, float* __restrict__ gI) {
  const int gl = threadIdx.x % G;
  const int64_t group = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  const int64_t ngroups = (int64_t)gridDim.x * kBlock / G;
  for (int64_t b = group; b < batch; b += ngroups) {
    const int64_t u = uid[b], p = pid[b], n = nid[b];
    float4 uv[CH], pv[CH], nv[CH];
    float sp = 0.f, sn = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t off = (int64_t)(c * G + gl) * 4;
      uv[c] = ld4(U + u * d + off);
      pv[c] = ld4(I + p * d + off);
      nv[c] = ld4(I + n * d + off);
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      sp = fmaf(uv[c].x, pv[c].x, sp); sp = fmaf(uv[c].y, pv[c].y, sp);
      sp = fmaf(uv[c].z, pv[c].z, sp); sp = fmaf(uv[c].w, pv[c].w, sp);
      sn = fmaf(uv[c].x, nv[c].x, sn); sn = fmaf(uv[c].y, nv[c].y, sn);
      sn = fmaf(uv[c].z, nv[c].z, sn); sn = fmaf(uv[c].w, nv[c].w, sn);
    }
#pragma unroll
    for (int m = G / 2; m > 0; m >>= 1) {
      sp += __shfl_xor(sp, m);
      sn += __shfl_xor(sn, m);
    }
    const float x = sp - sn;
    if (gl == 0) {
      if (loss) loss[b] = neg_log_sigmoid(x);
      if (hit) hit[b] = sp >= sn ? 1 : 0;
    }
    const float g = neg_log_sigmoid_grad(x) * grad_scale;
    if (gU || gI) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int64_t off = (int64_t)(c * G + gl) * 4;
        if (gU) {
          float* o = gU + u * d + off;
          atomicAdd(o + 0, g * pv[c].x - g * nv[c].x);
          atomicAdd(o + 1, g * pv[c].y - g * nv[c].y);
          atomicAdd(o + 2, g * pv[c].z - g * nv[c].z);
          atomicAdd(o + 3, g * pv[c].w - g * nv[c].w);
        }
        if (gI) {
          float* op = gI + p * d + off;
          float* on = gI + n * d + off;
          atomicAdd(op + 0, g * uv[c].x); atomicAdd(op + 1, g * uv[c].y);
          atomicAdd(op + 2, g * uv[c].z); atomicAdd(op + 3, g * uv[c].w);
          atomicAdd(on + 0, -g * uv[c].x); atomicAdd(on + 1, -g * uv[c].y);
          atomicAdd(on + 2, -g * uv[c].z); atomicAdd(on + 3, -g * uv[c].w);
        }
      }
    }
  }
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

}  // namespace

extern "C" int dr_bpr_fwd_bwd(const float* user_table, const float* item_table, int64_t d,
                              const int64_t* user_id, const int64_t* pos_id,
                              const int64_t* neg_id, int64_t batch, float grad_scale,
                              float* loss, int32_t* hit, float* grad_user, float* grad_item,
                              dr_stream_t stream) {
  DR_CHECK_ARG(batch >= 0, "batch must be >= 0");
  if (batch == 0) return DR_OK;
  DR_CHECK_ARG(user_table && item_table && user_id && pos_id && neg_id, "null pointer");
  DR_CHECK_ARG(d % 4 == 0 && d >= 16 && d <= 512, "d must be a multiple of 4 in [16, 512]");
  hipStream_t s = (hipStream_t)stream;
  const int64_t chunks = d / 4;  // 16-B chunks per row
  auto go = [&](auto kern, int G) {
    int64_t grid = dr::ceil_div(batch, kBlock / G);
    if (grid > 256 * 8) grid = 256 * 8;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), 0, s, user_table, item_table,
                       d, user_id, pos_id, neg_id, batch, grad_scale, loss, hit, grad_user,
                       grad_item);
  };
  switch (chunks) {
    case 4: go(bpr_kernel<4, 1>, 4); break;
    case 8: go(bpr_kernel<8, 1>, 8); break;
    case 16: go(bpr_kernel<16, 1>, 16); break;
    case 32: go(bpr_kernel<32, 1>, 32); break;
    case 64: go(bpr_kernel<64, 1>, 64); break;
    case 128: go(bpr_kernel<64, 2>, 64); break;
    default:
      dr::set_error("dr_bpr_fwd_bwd: d/4 must be a power of two in [4, 128]");
      return DR_EUNSUPPORTED;
  }
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
