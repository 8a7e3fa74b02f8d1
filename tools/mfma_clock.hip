// mfma_clock.hip - calibration (not part of the product): the f32 MFMA ceiling with the
// shader clock measured in the same run.  Each wave runs `iters` x 4 independent
// v_mfma_f32_32x32x2_f32 on register operands (constant or per-lane random values);
// thread 0 of each workgroup stamps clock64() (shader clock) and wall_clock64() (100 MHz)
// before and after, so TFLOP/s and the clock the chip held come from one launch.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_clock.hip -o tools/mfma_clock
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ float hashf(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return (float)(x & 0xffffff) / 16777216.0f - 0.5f;
}

template <bool RANDOM>
__global__ __launch_bounds__(256) void mfma_loop(long long* stamps, float* out, int iters) {
  floatx16 acc[4];
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float a[4], b[4];
  for (int t = 0; t < 4; ++t) {
    a[t] = RANDOM ? hashf(threadIdx.x * 7 + blockIdx.x * 977 + t) : 1e-3f * t;
    b[t] = RANDOM ? hashf(threadIdx.x * 13 + blockIdx.x * 331 + t + 100) : 2e-3f;
  }
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc[t], 0, 0, 0);
  }
  __syncthreads();
  const long long c1 = clock64(), w1 = wall_clock64();
  float s = 0.f;
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 16; ++e) s += acc[t][e];
  if (s == 12345.f) out[threadIdx.x] = s;
  if (threadIdx.x == 0) {
    stamps[blockIdx.x * 4 + 0] = c1 - c0;
    stamps[blockIdx.x * 4 + 1] = w1 - w0;
  }
}

template <bool RANDOM>
void run(const char* name, int blocks, int iters, long long* d_st, float* d_out) {
  hipLaunchKernelGGL(mfma_loop<RANDOM>, dim3(blocks), dim3(256), 0, 0, d_st, d_out, 100);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<RANDOM>, dim3(blocks), dim3(256), 0, 0, d_st, d_out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> st(blocks * 4);
  hipMemcpy(st.data(), d_st, st.size() * sizeof(long long), hipMemcpyDeviceToHost);
  double ghz = 0.0;
  for (int b = 0; b < blocks; ++b) ghz += (double)st[b * 4] / ((double)st[b * 4 + 1] * 10.0);  // cycles per ns
  ghz /= blocks;
  const double flops = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * 32 * 32 * 2 * 2;
  const double tf = flops / (ms * 1e-3) / 1e12;
  // peak at the measured clock: 256 CUs x 4 SIMDs x 64 FLOP/clk
  const double peak_at_clock = 256.0 * 4 * 64 * ghz * 1e9 / 1e12;
  printf("%-22s blocks %4d: %.1f TFLOP/s at %.3f GHz held -> %.1f%% of the peak at that clock (%.1f TF); "
         "%.1f%% of 157.3 spec\n",
         name, blocks, tf, ghz, 100.0 * tf / peak_at_clock, peak_at_clock, 100.0 * tf / 157.3);
}

int main() {
  long long* d_st;
  float* d_out;
  hipMalloc(&d_st, 4096 * 4 * sizeof(long long));
  hipMalloc(&d_out, 4096 * sizeof(float));
  const int iters = 40000;
  run<false>("constant, 1 wave/SIMD", 256, iters, d_st, d_out);
  run<true>("random,   1 wave/SIMD", 256, iters, d_st, d_out);
  run<false>("constant, 2 waves/SIMD", 512, iters, d_st, d_out);
  run<true>("random,   2 waves/SIMD", 512, iters, d_st, d_out);
  run<true>("random,   1 wave/SIMD", 256, iters / 8, d_st, d_out);
  return 0;
}
