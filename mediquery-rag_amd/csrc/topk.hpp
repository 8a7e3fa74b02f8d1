// topk.hpp - register-resident sorted candidate list shared by the scan kernels of
// index.hip (K9, K9s) and thresh.hip (K9t).
#pragma once

#include "common.hpp"

namespace mq {

// Register-resident running top-KC list per lane, kept sorted by (score desc, id asc).
template <int KC>
struct TopList {
  float s[KC];
  int id[KC];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      s[i] = -INFINITY;
      id[i] = -1;
    }
  }
  __device__ __forceinline__ bool beats_tail(float x, int xi) const {
    return better(x, xi, s[KC - 1], id[KC - 1]);
  }
  // Branch-free bubble insertion with static indices (stays in VGPRs).
  __device__ __forceinline__ void insert(float x, int xi) {
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const bool sw = better(x, xi, s[i], id[i]);
      const float ts = s[i];
      const int ti = id[i];
      s[i] = sw ? x : ts;
      id[i] = sw ? xi : ti;
      x = sw ? ts : x;
      xi = sw ? ti : xi;
    }
  }
  __device__ __forceinline__ void pop_front() {
#pragma unroll
    for (int i = 0; i + 1 < KC; ++i) {
      s[i] = s[i + 1];
      id[i] = id[i + 1];
    }
    s[KC - 1] = -INFINITY;
    id[KC - 1] = -1;
  }
};

}  // namespace mq
