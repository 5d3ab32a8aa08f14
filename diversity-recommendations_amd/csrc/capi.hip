// Library-level C ABI pieces: version, build id, the thread-local error string
// and the planner knobs.
#include <atomic>
#include <cmath>

#include "common.h"

namespace dr {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// Knob values, NaN = the default plan. Set only through dr_set_plan_knob: the
// library reads no environment variable.
static std::atomic<double> g_knobs[DR_KNOB_COUNT] = {
    {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}};
static_assert(DR_KNOB_COUNT == 11, "initialise every knob");

// The range of each knob (include/divrec_hip.h): the planner casts integer
// knobs with (int), so a value outside them would be undefined behaviour.
static const char* knob_range_error(int knob, double v) {
  const bool integral = v == std::floor(v);
  switch (knob) {
    case DR_KNOB_SCAN_SLOTS:
    case DR_KNOB_SCAN_SPLIT:
    case DR_KNOB_TAIL_KEYS:
    case DR_KNOB_GUESS_STRIDE:
      return (integral && v >= 1.0 && v <= 1073741824.0) ? nullptr : "an integer in [1, 2^30]";
    case DR_KNOB_SCAN_SEED:
    case DR_KNOB_GUESS_TIGHT:
    case DR_KNOB_ILD_STREAM:
      return (v == 0.0 || v == 1.0) ? nullptr : "0 or 1";
    case DR_KNOB_GUESS_Z1:
    case DR_KNOB_GUESS_C1:
      return (v >= -64.0 && v <= 64.0) ? nullptr : "a value in [-64, 64]";
    case DR_KNOB_SAMPLE_DENSE:
      return (v == 0.0 || v == 1.0 || (v > 1.0 && v <= 1048576.0))
                 ? nullptr
                 : "0 (off), 1 (on, the default budget) or a budget in GiB in (1, 2^20]";
    case DR_KNOB_ILD_BUFS:
      return (integral && v >= 1.0 && v <= 64.0) ? nullptr : "an integer in [1, 64]";
    default:
      return "a known knob";
  }
}
bool plan_knob(int id, double* v) {
  if (id < 0 || id >= DR_KNOB_COUNT) return false;
  const double x = g_knobs[id].load(std::memory_order_relaxed);
  if (std::isnan(x)) return false;
  *v = x;
  return true;
}

int device_cus() {
  static std::atomic<int> cache[64];
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < 64) n = cache[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (dev < 0 ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    if (dev >= 0 && dev < 64) cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}
}  // namespace dr

extern "C" int dr_set_plan_knob(int knob, double value) {
  if (knob < 0 || knob >= DR_KNOB_COUNT) {
    dr::set_error("dr_set_plan_knob: unknown knob " + std::to_string(knob));
    return DR_EINVAL;
  }
  if (!std::isnan(value)) {
    const char* want = std::isfinite(value) ? dr::knob_range_error(knob, value) : "finite";
    if (want) {
      dr::set_error("dr_set_plan_knob: knob " + std::to_string(knob) + " must be " + want +
                    ", got " + std::to_string(value));
      return DR_EINVAL;
    }
  }
  dr::g_knobs[knob].store(value, std::memory_order_relaxed);
  return DR_OK;
}

extern "C" double dr_get_plan_knob(int knob) {
  double v = NAN;
  return dr::plan_knob(knob, &v) ? v : NAN;
}

extern "C" int dr_version(void) { return 100; /* 0.1.0 */ }

// Source hash of the tree this library was compiled from (build_native.py
// source_hash), passed in by the build as -DDR_BUILD_ID="...".
#ifndef DR_BUILD_ID
#define DR_BUILD_ID "unknown"
#endif
extern "C" const char* dr_build_id(void) { return DR_BUILD_ID; }

extern "C" const char* dr_last_error(void) { return dr::g_last_error.c_str(); }
