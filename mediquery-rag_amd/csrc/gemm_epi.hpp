// gemm_epi.hpp - epilogue pieces shared by the encoder GEMMs (encoder.hip) and the
// pre-split split-f32 GEMM (gemm_x6p.hip): the epilogue kinds, the branch-free GELU
// forms, and a wave-tile store of 32x32 MFMA accumulators with bias / GELU / residual.
#pragma once

#include "gemm_f32.hpp"

namespace mq {

// EPI_RESID_STATS: EPI_RESID that also leaves per-row LayerNorm partials of its output
// (encoder.hip, LnArgs: the LayerNorm is then applied by the consuming GEMM).
enum Epi { EPI_BIAS = 0, EPI_GELU_ERF = 1, EPI_GELU_TANH = 2, EPI_RESID = 3, EPI_RESID_STATS = 4 };

// GELU, branch-free (it runs 64 times per lane in every FFN-up tile epilogue; ocml's erff
// is ~50 VALU + a divergent branch per element and measured as the FFN-up epilogue's cost).
// erf form: x * Phi(x), Phi(x) = 0.5 erfc(-x / sqrt 2), with erfc(z) for z = |x| / sqrt 2 from
// the Chebyshev fit t * exp(-z^2 + P(t)), t = 1 / (1 + z / 2) (Numerical Recipes erfcc,
// |relative error| < 1.2e-7 for all z >= 0): Phi = 1 - e / 2 for x >= 0, e / 2 below.  No
// 1 + erf cancellation for negative x: max |error| vs float64 3.8e-7 over [-12, 12], relative
// 1.7e-6 where |gelu| > 1e-3 (0.5 x (1 + erff) in fp32: 4.5e-7 and 5.1e-5).  v_rcp / v_exp
// are the hardware 1-ulp forms.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = t * __builtin_amdgcn_exp2f(fmaf(-z, z, p) * 1.4426950408889634f);  // erfc(z)
  return x * (x >= 0.f ? fmaf(-0.5f, e, 1.0f) : 0.5f * e);
}
// tanh form (llama.cpp's): 0.5 x (1 + tanh u) = x / (1 + exp(-2u)), u = sqrt(2/pi)(x + 0.044715 x^3)
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u * -2.8853900817779268f));
}

template <int EPI>
__device__ __forceinline__ float epi_apply(float v) {
  if constexpr (EPI == EPI_GELU_ERF) return gelu_erf(v);
  if constexpr (EPI == EPI_GELU_TANH) return gelu_tanh(v);
  return v;
}

// Store one wave's TM x TN grid of 32x32 accumulators whose origin is (wr0, wc0):
// out = epi(acc + bias[col]) (+ resid for EPI_RESID).  A wave tile inside [M, N] takes
// buffer loads / stores off its origin (one lane offset in a VGPR, each register's row
// offset a scalar soffset: no per-element address arithmetic) with every bias / residual
// load issued before the first use; a ragged edge tile takes guarded plain accesses.
template <int EPI, int TM, int TN>
__device__ __forceinline__ void store_wave_tile(floatx16 (&acc)[TM][TN], int wr0, int wc0, int M, int N,
                                                const float* __restrict__ bias, const float* __restrict__ resid,
                                                int ldr, float* __restrict__ out, int ldo, int lane) {
  if (wr0 + TM * 32 <= M && wc0 + TN * 32 <= N) {
    float bv[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bv[tn] = bias[wc0 + tn * 32 + (lane & 31)];
    float rv[TM][TN][16];
    if constexpr (EPI == EPI_RESID) {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(resid + (int64_t)wr0 * ldr + wc0), (short)0, 0x7fffffff, 0x00020000);
      const int rl = (4 * (lane >> 5) * ldr + (lane & 31)) * 4;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            rv[tm][tn][e] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(rr, rl, (acc_row(tm, e, 0) * ldr + tn * 32) * 4, 0));
    }
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(out + (int64_t)wr0 * ldo + wc0), (short)0, 0x7fffffff, 0x00020000);
    const int ol = (4 * (lane >> 5) * ldo + (lane & 31)) * 4;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = epi_apply<EPI>(acc[tm][tn][e] + bv[tn]);
          if constexpr (EPI == EPI_RESID) v += rv[tm][tn][e];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ro, ol, (acc_row(tm, e, 0) * ldo + tn * 32) * 4, 0);
        }
    return;
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = wc0 + tn * 32 + (lane & 31);
    if (col >= N) continue;
    const float b = bias[col];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr0 + acc_row(tm, e, lane);
        if (row >= M) continue;
        float v = epi_apply<EPI>(acc[tm][tn][e] + b);
        if constexpr (EPI == EPI_RESID) v += resid[(int64_t)row * ldr + col];
        out[(int64_t)row * ldo + col] = v;
      }
  }
}

}  // namespace mq
