// launch_probe.hip - calibration (not part of the product): the per-launch floor of
// dependent kernel chains in the shapes the few-row encoder uses, so the single-query
// encoder's 61 launches can be priced.  Each kernel reads one float per thread from a
// small L2-resident buffer (or nothing), optionally allocates LDS and crosses one
// barrier, and writes one float per workgroup.  60 launches per chain, HIP events.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o /tmp/launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int LDS_FLOATS, bool LOAD, bool BAR>
__global__ void probe(const float* __restrict__ in, float* __restrict__ out, int n) {
  __shared__ float s[LDS_FLOATS > 0 ? LDS_FLOATS : 1];
  float v = LOAD ? in[(blockIdx.x * blockDim.x + threadIdx.x) % n] : (float)threadIdx.x;
  if (LDS_FLOATS > 0) s[threadIdx.x % (LDS_FLOATS > 0 ? LDS_FLOATS : 1)] = v;
  if (BAR) __syncthreads();
  if (LDS_FLOATS > 0) v += s[(threadIdx.x + 1) % (LDS_FLOATS > 0 ? LDS_FLOATS : 1)];
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// per-launch time of a dependent chain captured as ONE hipGraph of `reps` launches (the
// device-side floor: no host enqueue cost inside the replay)
template <class K>
float chain(K kern, int grid, int block, const float* in, float* out, int n, int reps) {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, s, in, out, n);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int r = 0; r < 5; ++r) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  hipStreamDestroy(s);
  return ms * 1e3f / (5 * reps);
}

int main() {
  const int n = 1 << 20;
  float *in, *out;
  hipMalloc(&in, n * sizeof(float));
  hipMalloc(&out, 1 << 16);
  hipMemset(in, 0, n * sizeof(float));
  const int reps = 200;
  struct Cfg {
    int grid, block;
  };
  const Cfg cfgs[] = {{96, 1024}, {288, 1024}, {384, 1024}, {96, 256}, {384, 256}, {1536, 256}, {256, 512}, {12, 512}};
  for (const Cfg& c : cfgs) {
    printf("grid %5d x %4d: empty %.2f us | load %.2f | load+bar %.2f | load+bar+16KB LDS %.2f | +64KB LDS %.2f\n",
           c.grid, c.block, chain(probe<0, false, false>, c.grid, c.block, in, out, n, reps),
           chain(probe<0, true, false>, c.grid, c.block, in, out, n, reps),
           chain(probe<0, true, true>, c.grid, c.block, in, out, n, reps),
           chain(probe<4096, true, true>, c.grid, c.block, in, out, n, reps),
           chain(probe<16384, true, true>, c.grid, c.block, in, out, n, reps));
  }
  return 0;
}
