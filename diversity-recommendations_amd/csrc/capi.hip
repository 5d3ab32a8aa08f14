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
    {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}, {NAN}};
static_assert(DR_KNOB_COUNT == 9, "initialise every knob");
bool plan_knob(int id, double* v) {
  if (id < 0 || id >= DR_KNOB_COUNT) return false;
  const double x = g_knobs[id].load(std::memory_order_relaxed);
  if (std::isnan(x)) return false;
  *v = x;
  return true;
}
}  // namespace dr

extern "C" int dr_set_plan_knob(int knob, double value) {
  if (knob < 0 || knob >= DR_KNOB_COUNT) {
    dr::set_error("dr_set_plan_knob: unknown knob " + std::to_string(knob));
    return DR_EINVAL;
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
