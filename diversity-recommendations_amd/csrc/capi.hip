// Library-level C ABI pieces: version and the thread-local error string.
#include "common.h"

namespace dr {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace dr

extern "C" int dr_version(void) { return 100; /* 0.1.0 */ }

extern "C" const char* dr_last_error(void) { return dr::g_last_error.c_str(); }
