// roctx ranges for rocprofv3 (see include/msbfs/trace.hpp).
#include "msbfs/trace.hpp"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#ifdef MSBFS_HAVE_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

namespace msbfs {
namespace trace {

bool enabled() {
#ifdef MSBFS_HAVE_ROCTX
  static const bool on = [] {
    const char* e = getenv("MSBFS_ROCTX");
    return !(e && !strcmp(e, "0"));
  }();
  return on;
#else
  return false;
#endif
}

void push(const char* fmt, ...) {
  if (!enabled()) return;
  char buf[128];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
#ifdef MSBFS_HAVE_ROCTX
  roctxRangePushA(buf);
#endif
}

void pop() {
  if (!enabled()) return;
#ifdef MSBFS_HAVE_ROCTX
  roctxRangePop();
#endif
}

void mark(const char* msg) {
  if (!enabled()) return;
#ifdef MSBFS_HAVE_ROCTX
  roctxMarkA(msg);
#else
  (void)msg;
#endif
}

}  // namespace trace
}  // namespace msbfs
