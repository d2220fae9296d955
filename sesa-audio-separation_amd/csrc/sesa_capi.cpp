// Version / error-string entry points of the libsesa C ABI.
#include <cstdarg>
#include <cstdio>

#include "sesa_common.hpp"

namespace sesa {
namespace {
thread_local char g_err[1024] = {0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace sesa

extern "C" int sesa_version(void) { return 100; }  // 0.1.0

extern "C" const char* sesa_last_error(void) { return sesa::g_err; }
