// librpt's error plumbing: a thread-local last error set by every failing entry point and read
// through rpt_last_error() (include/rpt.h); plus the library version.  Host-only (see
// host_common.h).
#include <cstdarg>
#include <cstdio>
#include <string>

#include "host_common.h"

namespace rpt {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
}
void clear_error() { g_last_error.clear(); }
const char* last_error_cstr() { return g_last_error.c_str(); }

}  // namespace rpt

extern "C" {
const char* rpt_last_error(void) { return rpt::last_error_cstr(); }
int32_t rpt_version(void) { return 100; }  // 0.1.0
}
