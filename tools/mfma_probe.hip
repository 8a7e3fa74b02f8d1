// mfma_probe.hip - calibration kernels for the fp32 MFMA GEMM core (not part of the product).
//  probe_regs: back-to-back v_mfma_f32_32x32x2_f32 on registers (4 accumulators / wave)
//  probe_lds : the gemm_f32.hpp mma_slice loop over one resident LDS stage, no global
//              loads and no barriers -> ceiling of the LDS-read + MFMA part of the core
#include <hip/hip_runtime.h>
#include "../mediquery-rag_amd/csrc/gemm_f32.hpp"
using namespace mq;

extern "C" __global__ __launch_bounds__(256, 2) void probe_regs(float* out, int iters) {
  floatx16 acc[4];
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
  }
  float s = 0.f;
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 16; ++e) s += acc[t][e];
  if (s == 12345.f) out[threadIdx.x] = s;
}

__device__ float hashf(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (float)(x & 0xffffff) / 16777216.0f - 0.5f;
}

// MODE 0: LDS + MFMA only; 1: + __syncthreads per slice; 2: + ds_write of a staged
// slice + barrier; 3: + global loads (L2-resident buffer) into the stager, i.e. the full
// gemm_f32 pipeline on a resident operand
template <class T, int MODE>
__device__ void probe_lds_t(float* out, int iters, const float* gsrc) {
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  for (int i = threadIdx.x; i < 2 * T::STAGE_FLOATS; i += 256) lds[i] = hashf(i + 977 * blockIdx.x);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  floatx16 acc[T::TM][T::TN];
  zero_acc<T>(acc);
  Stager<T> st;
  for (int j = 0; j < T::LOADS; ++j) st.r[j] = floatx4{hashf(tid + j), 0.1f, 0.2f, 0.3f};
  for (int i = 0; i < iters; ++i) {
    if (MODE >= 3) st.load(gsrc, 768, 8192, (blockIdx.x % 64) * T::BM, gsrc, 768, 8192, 4096 + (blockIdx.x % 32) * T::BN, (i % 24) * 32, tid);
    mma_slice<T>(lds + (i & 1) * T::STAGE_FLOATS, acc, wave / T::WAVES_N, wave % T::WAVES_N, lane);
    if (MODE >= 2) st.store(lds + ((i + 1) & 1) * T::STAGE_FLOATS, tid);
    if (MODE >= 1) __syncthreads();
  }
  float s = 0.f;
  for (int tm = 0; tm < T::TM; ++tm)
    for (int tn = 0; tn < T::TN; ++tn)
      for (int e = 0; e < 16; ++e) s += acc[tm][tn][e];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void probe_lds_128x96(float* out, int iters, const float* g) {
  probe_lds_t<F32Tile<4, 1, 1, 3>, MODE>(out, iters, g);
}

extern "C" int probe_run(int which, int blocks, int iters, float* out, const float* g, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (which == 0) hipLaunchKernelGGL(probe_regs, dim3(blocks), dim3(256), 0, s, out, iters);
  if (which == 1) hipLaunchKernelGGL(probe_lds_128x96<0>, dim3(blocks), dim3(256), 0, s, out, iters, g);
  if (which == 2) hipLaunchKernelGGL(probe_lds_128x96<1>, dim3(blocks), dim3(256), 0, s, out, iters, g);
  if (which == 3) hipLaunchKernelGGL(probe_lds_128x96<2>, dim3(blocks), dim3(256), 0, s, out, iters, g);
  if (which == 4) hipLaunchKernelGGL(probe_lds_128x96<3>, dim3(blocks), dim3(256), 0, s, out, iters, g);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
