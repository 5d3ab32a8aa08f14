// Library-level C ABI pieces: version, build id and the thread-local error string.
#include "common.h"

namespace dr {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace dr

extern "C" int dr_version(void) { return 100; /* 0.1.0 */ }

// Source hash of the tree this library was compiled from (build_native.py
// source_hash), passed in by the build as -DDR_BUILD_ID="...".
#ifndef DR_BUILD_ID
#define DR_BUILD_ID "unknown"
#endif
extern "C" const char* dr_build_id(void) { return DR_BUILD_ID; }

extern "C" const char* dr_last_error(void) { return dr::g_last_error.c_str(); }
