// common.hpp - status plumbing, device guard and small device helpers shared by the
// index (index.hip) and encoder (encoder.hip) halves of libmqhip.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

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

// Grow-only pinned host staging for the host-pointer entry points: a pageable 3-KB copy
// is staged by the runtime and synchronous (~10-20 us each way on the single-query path);
// from pinned memory it is one DMA on the stream.
struct PinBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return MQ_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    if (hipHostMalloc(&p, need, hipHostMallocDefault) != hipSuccess)
      MQ_FAIL(MQ_ENOMEM, "hipHostMalloc(%zu bytes) failed", need);
    bytes = need;
    return MQ_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

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

// Optional per-kernel-class device timeline: one HIP event per launch boundary on the
// launch stream; interval i (event i -> i+1) is charged to stage[i].  Off by default;
// drain() folds the intervals into acc[] (it synchronises on the last event).
struct Timeline {
  static constexpr int kMaxStages = 16;
  bool on = false;
  std::vector<hipEvent_t> pool;
  std::vector<int> stage;
  size_t used = 0;
  float acc[kMaxStages] = {};

  void mark(hipStream_t st, int next_stage) {
    if (!on) return;
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      pool.push_back(e);
    }
    (void)hipEventRecord(pool[used], st);
    stage.resize(used + 1);
    stage[used] = next_stage;
    ++used;
  }
  void close(hipStream_t st) { mark(st, -1); }
  void drain() {
    if (used >= 2) {
      (void)hipEventSynchronize(pool[used - 1]);
      for (size_t i = 0; i + 1 < used; ++i) {
        if (stage[i] < 0 || stage[i] >= kMaxStages) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pool[i], pool[i + 1]) == hipSuccess) acc[stage[i]] += ms;
      }
    }
    used = 0;
  }
  // copy out and reset the accumulated milliseconds
  void read(float* out, int n) {
    drain();
    for (int i = 0; i < n && i < kMaxStages; ++i) out[i] = acc[i];
    for (float& a : acc) a = 0.f;
  }
  ~Timeline() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace mq
