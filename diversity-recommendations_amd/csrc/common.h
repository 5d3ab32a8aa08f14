// Shared device/host helpers for libdivrec_hip (gfx950 / CDNA4 only).
//
// Everything here is written for 64-lane wavefronts: lane = threadIdx.x & 63,
// ballots are 64-bit, cross-lane moves go through ds_bpermute (__shfl_xor).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/divrec_hip.h"

namespace dr {

// ---------------------------------------------------------------- errors
// Thread-local last-error string behind dr_last_error() (include/divrec_hip.h).
void set_error(const std::string& msg);

// Planner knobs (dr_set_plan_knob, include/divrec_hip.h): true and *v set when
// knob `id` holds a value (not NaN).
bool plan_knob(int id, double* v);

// Compute units of the current device (cached per device ordinal; 256 if the
// query fails): the grid of the persistent kernels.
int device_cus();

#define DR_CHECK_ARG(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) {                                                \
      ::dr::set_error(std::string(__func__) + ": " + (msg));      \
      return DR_EINVAL;                                           \
    }                                                             \
  } while (0)

#define DR_CHECK_HIP(expr)                                                        \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::dr::set_error(std::string(__func__) + ": " #expr " -> " +                 \
                      hipGetErrorString(e_));                                     \
      return DR_EHIP;                                                             \
    }                                                                             \
  } while (0)

#define DR_CHECK_LAUNCH() DR_CHECK_HIP(hipGetLastError())

// ---------------------------------------------------------------- types
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ float bf16_bits_to_f32(uint32_t b16) {
  return __uint_as_float(b16 << 16);
}

// ---------------------------------------------------------------- top-K keys
// A (score, item) pair is packed into one 64-bit key whose unsigned order is
// the ranking order of the reference path with its tie-break made explicit:
// score descending, then item id ascending (divrec/train/utils.py:73 ranks with
// an unstable argsort; SURVEY.md §8 quirk 3 fixes ties to "id asc").
//   key = ord(score) << 32 | ~item
// ord() maps fp32 to an order-preserving uint32 after canonicalising -0 to +0
// (so -0 and +0 tie, as they do under float comparison). Key 0 = empty slot.
__device__ __forceinline__ uint32_t f32_to_ord(float f) {
  f = f + 0.0f;  // -0.0 -> +0.0 (round-to-nearest); not folded without fast-math
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_to_f32(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t make_key(float score, uint32_t item) {
  return ((uint64_t)f32_to_ord(score) << 32) | (uint64_t)(~item);
}
__device__ __forceinline__ uint32_t key_item(uint64_t key) { return ~(uint32_t)key; }
__device__ __forceinline__ float key_score(uint64_t key) {
  return ord_to_f32((uint32_t)(key >> 32));
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int mask) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, mask);
  hi = __shfl_xor(hi, mask);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// Wave-wide bitonic sort, DESCENDING, of N = 64*P keys held in registers.
// Element e lives in lane e / P, register e % P. Every loop bound is a
// compile-time constant, so the network unrolls and all register indices are
// static (no scratch). Strides < P are register swaps inside a lane; strides
// >= P exchange with lane ^ (stride / P).
template <int P>
__device__ __forceinline__ void wave_sort_desc(uint64_t (&key)[P]) {
  constexpr int N = 64 * P;
  const int lane = lane_id();
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j < P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
          if ((i & j) == 0) {
            const int e = lane * P + i;
            const bool desc = (e & k) == 0;
            uint64_t a = key[i], b = key[i | j];
            uint64_t mx = umax64(a, b), mn = umin64(a, b);
            key[i] = desc ? mx : mn;
            key[i | j] = desc ? mn : mx;
          }
        }
      } else {
        const int lm = j / P;
        const bool lower = (lane & lm) == 0;
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const int e = lane * P + i;
          const bool desc = (e & k) == 0;
          uint64_t o = shfl_xor_u64(key[i], lm);
          const bool keep_max = (lower == desc);
          key[i] = keep_max ? umax64(key[i], o) : umin64(key[i], o);
        }
      }
    }
  }
}

// Select register i of a lane-local array with a runtime index without
// dynamic register indexing (which would spill to scratch).
template <int P, typename T>
__device__ __forceinline__ T select_reg(const T (&v)[P], int idx) {
  T r = v[0];
#pragma unroll
  for (int i = 1; i < P; ++i) r = (idx == i) ? v[i] : r;
  return r;
}
// The same for 64-bit keys as a masked OR: at P >= 16 hipcc turns the select
// chain above back into an indexed access of a stack copy (scratch).
template <int P>
__device__ __forceinline__ uint64_t select_key(const uint64_t (&v)[P], int idx) {
  uint64_t r = 0ull;
#pragma unroll
  for (int i = 0; i < P; ++i) r |= v[i] & (0ull - (uint64_t)(idx == i));
  return r;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace dr
