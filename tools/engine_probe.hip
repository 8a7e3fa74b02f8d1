// engine_probe.hip - what a persistent single-query engine could save.
//
// The few-row forward (csrc/encoder.hip forward_rows) is a chain of ~49 launches, ~8.7 us
// each; in every launch each workgroup first streams its weight slice (48-96 KB) AND the
// full activation rows of the query (98-196 KB: every output column needs every K), and
// the trace (profiles/r4/ktrace_L32.txt) shows the operands landing 3.2-4.0 us after the
// workgroup starts.  A persistent engine can issue the weight loads before it waits for
// the previous phase, but the activation rows can only be loaded after it, through a
// grid-wide hand-off.  This probe times that critical path with the compute left out:
//   chain:      P dependent launches; launch p: every workgroup loads W bytes of its own
//               weight slice and the A bytes of activation phase p - 1 wrote, reduces them
//               to one value per thread and writes its 2 KB share of phase p's activation
//               (the launch boundary is the hand-off);
//   persistent: ONE launch of P phases, one workgroup per CU: the weight loads of phase p
//               issued BEFORE the grid barrier that ends phase p - 1 (off the critical path),
//               then an agent-scope acquire and the activation loads, the same reduction and
//               store, and the barrier arrive (release fence; MI355X_MICROARCH.md's
//               barrier-xcd form: per-group counters of 32 workgroups, a top counter and a
//               generation word; every spin bounded by a 50 ms timeout word).
// Both write identical activations (checked).  Prints us per phase for each (A, W).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/engine_probe tools/engine_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int kThreads = 1024;
constexpr int kShare = 512;  // floats each workgroup writes per phase (2 KB)

struct Sync {
  unsigned cnt[8][32];  // per-group arrival counters, one 128-B line each
  unsigned top[32];
  unsigned gen[32];
  unsigned tmo[32];
};

__device__ __forceinline__ unsigned ld_rlx(unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded spin of ONE lane on gen >= want (s_sleep between polls); false on timeout
__device__ bool spin_until(Sync* sy, unsigned want) {
  const long long t0 = wall_clock64();
  while (ld_rlx(&sy->gen[0]) < want) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > 5000000ll) {  // 50 ms at 100 MHz
      __hip_atomic_store((gu32*)&sy->tmo[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

// grid barrier episode `e` (1, 2, ...), split so the next phase's weight loads issue
// between the two halves: arrive = every storing wave drains its stores, one lane's
// agent release, the group / top counters; wait = one lane's bounded relaxed poll of the
// generation word, one agent acquire, then the workgroup barrier
__device__ void barrier_arrive(Sync* sy, unsigned e, int nwg) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int g = blockIdx.x & 7;
    const unsigned members = (unsigned)((nwg - g + 7) / 8);
    const unsigned v = __hip_atomic_fetch_add((gu32*)&sy->cnt[g][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v + 1 == members * e) {
      const unsigned u = __hip_atomic_fetch_add((gu32*)&sy->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned groups = (unsigned)(nwg < 8 ? nwg : 8);
      if (u + 1 == groups * e) __hip_atomic_store((gu32*)&sy->gen[0], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ void barrier_wait(Sync* sy, unsigned e) {
  if (threadIdx.x == 0) {
    spin_until(sy, e);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// one phase's body: W-slice values (already loaded) + the activation bytes -> a value
// per thread; workgroup b writes floats [b * kShare, (b + 1) * kShare) of `out`
template <int NA, int NW>
__device__ __forceinline__ void body(const floatx4 (&w)[NW > 0 ? NW : 1], const float* __restrict__ act,
                                     float* __restrict__ out, int phase) {
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  floatx4 a[NA > 0 ? NA : 1];
#pragma unroll
  for (int i = 0; i < NA; ++i) a[i] = reinterpret_cast<const floatx4*>(act)[i * kThreads + threadIdx.x];
#pragma unroll
  for (int i = 0; i < NA; ++i) s += a[i];
#pragma unroll
  for (int i = 0; i < NW; ++i) s += w[i] * 1e-3f;
  if (threadIdx.x < kShare) out[blockIdx.x * kShare + threadIdx.x] = s.x + s.y + s.z + s.w + (float)phase;
}

template <int NA, int NW>
__device__ __forceinline__ void load_w(floatx4 (&w)[NW > 0 ? NW : 1], const float* __restrict__ W, int phase) {
  const floatx4* src = reinterpret_cast<const floatx4*>(W) + ((size_t)phase * gridDim.x + blockIdx.x) * NW * kThreads;
#pragma unroll
  for (int i = 0; i < NW; ++i) w[i] = src[i * kThreads + threadIdx.x];
}

template <int NA, int NW>
__global__ __launch_bounds__(kThreads, 1) void chain_kernel(const float* W, float* act, int phase, int act_floats) {
  floatx4 w[NW > 0 ? NW : 1];
  load_w<NA, NW>(w, W, phase);
  body<NA, NW>(w, act + (size_t)(phase & 1) * act_floats, act + (size_t)((phase + 1) & 1) * act_floats, phase);
}

// The few-row kernels' own operand pattern (rows_gemm_kernel, FFN-down shape: 32 rows x
// 1536 of A and 16 rows x 1536 of W per workgroup, wave w = K range [96 w, 96 w + 96)):
// lane (c = lane & 15, kq = lane >> 4) loads 16 B at row c (+ 16 rt) of A / row c of W,
// k = 96 w + 16 j + 4 kq - each wave instruction touches 16 rows x 64 B, not 1 KB of
// whole lines.  FULL = 1: the same bytes read lane-linear (whole lines per instruction).
template <bool FULL>
__global__ __launch_bounds__(kThreads, 1) void rows_pattern_kernel(const float* W, float* act, int phase, int act_floats) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, kq = lane >> 4;
  const float* A = act + (size_t)(phase & 1) * act_floats;
  const float* Wp = W + ((size_t)phase * gridDim.x + blockIdx.x) * 16 * 1536;
  floatx4 s = {0.f, 0.f, 0.f, 0.f}, a[12], w[6];
  if (FULL) {
#pragma unroll
    for (int i = 0; i < 12; ++i) a[i] = reinterpret_cast<const floatx4*>(A)[i * kThreads + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 6; ++i) w[i] = reinterpret_cast<const floatx4*>(Wp)[i * kThreads + threadIdx.x];
  } else {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int j = 0; j < 6; ++j)
        a[rt * 6 + j] = *reinterpret_cast<const floatx4*>(A + (rt * 16 + c) * 1536 + wave * 96 + 16 * j + 4 * kq);
#pragma unroll
    for (int j = 0; j < 6; ++j) w[j] = *reinterpret_cast<const floatx4*>(Wp + c * 1536 + wave * 96 + 16 * j + 4 * kq);
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) s += a[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) s += w[i] * 1e-3f;
  float* out = act + (size_t)((phase + 1) & 1) * act_floats;
  if (threadIdx.x < kShare) out[blockIdx.x * kShare + threadIdx.x] = s.x + s.y + s.z + s.w + (float)phase;
}

template <bool FULL>
void run_pattern(int nwg, int phases, const float* W, float* act, int act_floats) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CHECK(hipEventRecord(e0));
    for (int p = 0; p < phases; ++p)
      hipLaunchKernelGGL((rows_pattern_kernel<FULL>), dim3(nwg), dim3(kThreads), 0, 0, W, act, p, act_floats);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best = ms < best ? ms : best;
  }
  std::printf("{\"pattern\": \"%s\", \"act_kb_per_wg\": 192, \"w_kb_per_wg\": 96, \"wgs\": %d, \"chain_us_per_phase\": %.3f}\n",
              FULL ? "lane-linear (whole lines)" : "rows_gemm (16 rows x 64 B per instruction)", nwg, best * 1e3f / phases);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

template <int NA, int NW>
__global__ __launch_bounds__(kThreads, 1) void persistent_kernel(const float* W, float* act, int phases, int act_floats,
                                                                 Sync* sy) {
  floatx4 w[NW > 0 ? NW : 1];
  for (int p = 0; p < phases; ++p) {
    if (p > 0) barrier_arrive(sy, (unsigned)p, (int)gridDim.x);
    load_w<NA, NW>(w, W, p);             // this phase's weights: issued before the hand-off wait
    if (p > 0) barrier_wait(sy, (unsigned)p);
    if (ld_rlx(&sy->tmo[0])) return;     // a timed-out barrier: every workgroup leaves
    body<NA, NW>(w, act + (size_t)(p & 1) * act_floats, act + (size_t)((p + 1) & 1) * act_floats, p);
  }
}

template <int NA, int NW>
void run(int nwg, int phases, const float* W, float* act, Sync* sy, int act_floats) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const size_t abytes = (size_t)2 * act_floats * 4;
  std::vector<float> r1(act_floats * 2), r2(act_floats * 2);
  float best_c = 1e30f, best_p = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CHECK(hipMemset(act, 0, abytes));
    CHECK(hipEventRecord(e0));
    for (int p = 0; p < phases; ++p) hipLaunchKernelGGL((chain_kernel<NA, NW>), dim3(nwg), dim3(kThreads), 0, 0, W, act, p, act_floats);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best_c = ms < best_c ? ms : best_c;
    if (rep == 5) CHECK(hipMemcpy(r1.data(), act, abytes, hipMemcpyDeviceToHost));
    CHECK(hipMemset(act, 0, abytes));
    CHECK(hipMemset(sy, 0, sizeof(Sync)));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((persistent_kernel<NA, NW>), dim3(nwg), dim3(kThreads), 0, 0, W, act, phases, act_floats, sy);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned tmo = 0;
    CHECK(hipMemcpy(&tmo, &sy->tmo[0], 4, hipMemcpyDeviceToHost));
    if (tmo) {
      std::printf("TIMEOUT in the persistent barrier (A=%d W=%d)\n", NA, NW);
      return;
    }
    if (rep) best_p = ms < best_p ? ms : best_p;
    if (rep == 5) CHECK(hipMemcpy(r2.data(), act, abytes, hipMemcpyDeviceToHost));
  }
  bool same = true;
  for (size_t i = 0; i < r1.size(); ++i) same &= r1[i] == r2[i];
  std::printf("{\"act_kb_per_wg\": %d, \"w_kb_per_wg\": %d, \"wgs\": %d, \"phases\": %d, \"chain_us_per_phase\": %.3f, "
              "\"persistent_us_per_phase\": %.3f, \"ratio\": %.3f, \"same_output\": %s}\n",
              NA * kThreads * 16 / 1024, NW * kThreads * 16 / 1024, nwg, phases, best_c * 1e3f / phases,
              best_p * 1e3f / phases, best_p / best_c, same ? "true" : "false");
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent_kernel<12, 3>, kThreads, 0));
  const int nwg = cus;  // one workgroup per CU: every one resident (checked below)
  std::printf("{\"cus\": %d, \"blocks_per_cu\": %d}\n", cus, occ);
  if (occ < 1) return 1;
  const int phases = 48;
  const int act_floats = 128 * 1024;  // >= 12 x 1024 x 4 floats read and nwg x kShare written
  if (nwg * kShare > act_floats) return 1;
  const size_t wfloats = (size_t)phases * nwg * 6 * kThreads * 4;  // 6 float4 per thread per phase max
  float *W, *act;
  Sync* sy;
  CHECK(hipMalloc(&W, wfloats * 4));
  CHECK(hipMemset(W, 0, wfloats * 4));
  CHECK(hipMalloc(&act, (size_t)2 * act_floats * 4));
  CHECK(hipMalloc(&sy, sizeof(Sync)));
  // activation 0 / 98 / 196 KB per workgroup x weights 0 / 48 / 96 KB (the few-row launches'
  // per-CU bytes: QKV and FFN-up read 196 KB of rows + 48 KB of weights)
  run<0, 0>(nwg, phases, W, act, sy, act_floats);
  run<6, 0>(nwg, phases, W, act, sy, act_floats);
  run<12, 0>(nwg, phases, W, act, sy, act_floats);
  run<0, 3>(nwg, phases, W, act, sy, act_floats);
  run<6, 3>(nwg, phases, W, act, sy, act_floats);
  run<12, 3>(nwg, phases, W, act, sy, act_floats);
  run<12, 6>(nwg, phases, W, act, sy, act_floats);
  for (int g : {96, 256}) {  // FFN-down's 96 workgroups, and a full chip
    run_pattern<true>(g, phases, W, act, act_floats);
    run_pattern<false>(g, phases, W, act, act_floats);
  }
  CHECK(hipFree(W));
  CHECK(hipFree(act));
  CHECK(hipFree(sy));
  return 0;
}
