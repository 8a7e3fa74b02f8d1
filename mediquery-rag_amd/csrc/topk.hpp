// topk.hpp - register-resident sorted candidate list shared by the scan kernels of
// index.hip (K9, K9s) and thresh.hip (K9t).
#pragma once

#include "common.hpp"

namespace mq {

// Lane exchanges without the LDS crossbar: xor 1 / 2 / 8 by DPP, xor 4 by a swizzle
// (bit mode, within 32 lanes), wider by ds_bpermute.
__device__ __forceinline__ float xor_move(float v, int m) {
  const int b = __float_as_int(v);
  switch (m) {
    case 8: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x128, 0xf, 0xf, false));  // row_ror:8
    case 4: return __int_as_float(__builtin_amdgcn_ds_swizzle(b, 0x101f));  // xor 4 (bit mode)
    case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0x4e, 0xf, 0xf, false));   // quad [2,3,0,1]
    case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(b, 0xb1, 0xf, 0xf, false));   // quad [1,0,3,2]
    default: return __shfl_xor(v, m);
  }
}

// max over the wave, every lane gets it: DPP / swizzle within 16 lanes, then the two swaps
__device__ __forceinline__ unsigned wave_max_u32(unsigned m) {
#pragma unroll
  for (int off = 1; off <= 8; off <<= 1) m = max(m, (unsigned)__float_as_int(xor_move(__int_as_float((int)m), off)));
  auto r = __builtin_amdgcn_permlane16_swap(m, m, false, false);
  m = max((unsigned)r[0], (unsigned)r[1]);
  r = __builtin_amdgcn_permlane32_swap(m, m, false, false);
  return max((unsigned)r[0], (unsigned)r[1]);
}

// Sum each of U = 8 per-lane values over the 64 lanes of a wave.  Lane l ends holding
// value rerank_slot(l) (the 8 lanes with (l & 7) == 0 hold all eight).  Each sum is the
// same pairwise tree as `for (off = 32; off; off >>= 1) v += shfl_xor(v, off)` (each lane
// adds its own and its xor-partner's partial sum at every level; addition commutes), so
// the result is bit-identical to that butterfly.  Halving steps: v_permlane32_swap /
// v_permlane16_swap of the pair (x, y) then x' + y', a DPP row_ror:8 for xor 8.
__device__ __forceinline__ int rerank_slot(int lane) {
  return (((lane >> 5) & 1) << 2) | (((lane >> 4) & 1) << 1) | ((lane >> 3) & 1);
}
__device__ __forceinline__ float transpose_sum8(float (&v)[8], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 4]), false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 2]), false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool hi = (lane & 8) != 0;
  float x = (hi ? v[1] : v[0]) + xor_move(hi ? v[0] : v[1], 8);
  x += xor_move(x, 4);
  x += xor_move(x, 2);
  return x + xor_move(x, 1);
}

// fp32 dots of query q4 with U = 8 gathered rows (ids < 0: row 0, ignored by the caller):
// lane l accumulates float4 columns l, l + 64, ... in that order with one fma chain per
// float4 (w, z, y, x innermost first), every row load of the round issued before the first
// fma (the rows are scattered in HBM: one round trip instead of one per 64 columns).
// Returns the wave-summed dot of candidate rerank_slot(lane).
__device__ __forceinline__ float rerank_dots8(const floatx4* __restrict__ q4, const float* __restrict__ rows,
                                              int dim, const long long (&id)[8], int lane) {
  const int n4 = dim >> 2;
  floatx4 b[4][8];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (lane + 64 * t < n4)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        b[t][u] = reinterpret_cast<const floatx4*>(rows + (id[u] >= 0 ? id[u] : 0) * dim)[lane + 64 * t];
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (lane + 64 * t < n4) {
      const floatx4 a = q4[lane + 64 * t];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        acc[u] = fmaf(a.x, b[t][u].x, fmaf(a.y, b[t][u].y, fmaf(a.z, b[t][u].z, fmaf(a.w, b[t][u].w, acc[u]))));
    }
  for (int i = lane + 256; i < n4; i += 64) {  // dim > 1024 (plain bf16 mode): a round trip per 64
    const floatx4 a = q4[i];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const floatx4 c = reinterpret_cast<const floatx4*>(rows + (id[u] >= 0 ? id[u] : 0) * dim)[i];
      acc[u] = fmaf(a.x, c.x, fmaf(a.y, c.y, fmaf(a.z, c.z, fmaf(a.w, c.w, acc[u]))));
    }
  }
  return transpose_sum8(acc, lane);
}

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
