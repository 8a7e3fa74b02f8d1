// common.hpp - status plumbing, device guard and small device helpers shared by the
// index (index.hip) and encoder (encoder.hip) halves of libmqhip.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>

#include "mq.h"

#define MQ_STR2(x) #x
#define MQ_STR(x) MQ_STR2(x)

namespace mq {

// ------------------------------------------------------------------ status ----
void set_error(const char* fmt, ...);
void clear_error();

struct Status {
  int code = MQ_OK;
};

#define MQ_FAIL(code, ...)        \
  do {                            \
    ::mq::set_error(__VA_ARGS__); \
    return (code);                \
  } while (0)

#define MQ_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ::mq::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                       \
      return MQ_EHIP;                                                                  \
    }                                                                                  \
  } while (0)

#define MQ_CHECK_ARG(cond, ...)              \
  do {                                       \
    if (!(cond)) MQ_FAIL(MQ_EINVAL, __VA_ARGS__); \
  } while (0)

// Run `fn` with `device` current, restoring the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(device) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// ------------------------------------------------------------ device side ----
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

// Ordering used everywhere for retrieval results: higher score first, then lower id.
// Padding entries carry (-inf, -1) and lose to every real entry.
__device__ __forceinline__ bool better(float sa, int64_t ia, float sb, int64_t ib) {
  return sa > sb || (sa == sb && (unsigned long long)ia < (unsigned long long)ib);
}

}  // namespace mq
