// common.hip - thread-local error state and library-level entry points of libmqhip.so.
#include "common.hpp"

namespace mq {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

void clear_error() { g_last_error.clear(); }

}  // namespace mq

extern "C" {

const char* mq_last_error(void) { return mq::g_last_error.c_str(); }

const char* mq_version(void) { return "libmqhip 0.1 (gfx950, HIP " MQ_STR(HIP_VERSION_MAJOR) "." MQ_STR(HIP_VERSION_MINOR) ")"; }

int mq_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
