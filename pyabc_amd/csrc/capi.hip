// Library-wide C-ABI plumbing: error reporting and version.
#include <cstdarg>
#include "common.hpp"

namespace abc {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace abc

extern "C" {
const char* abc_last_error(void) { return abc::g_err; }
int abc_version(void) { return 10000; }  // 0.1.0
}
