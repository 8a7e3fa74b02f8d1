// thresh.hip - K9t: the bf16 threshold scan that produces the candidates of batched
// bf16 searches (the certified screen's first tier, MQ_DTYPE_F32_SCREEN, and BASELINE
// config 5's coarse scan, MQ_DTYPE_BF16) - the top-k half of Chroma's similarity_search
// (reference src/agents/nodes.py:93) at batch scale.  See DESIGN.md §4.
#include "gemm_f32.hpp"

#ifndef MQ_TS_DBG  // measurement builds only (wrong results): 1 = stream only, 2 = multiply
                   // only, 4 = no fragment reads, 8 = no barrier
#define MQ_TS_DBG 0
#endif
#include "thresh.hpp"
#include "topk.hpp"

namespace mq {

// ===================================== K9t: bf16 threshold scan (batched screens) ==
// The batched bf16 screen needs, per query, every row whose bf16 score clears a
// threshold tau_q chosen so that ~128 rows do (the 64 candidates come from those).
// With a fixed threshold the epilogue is one compare per score - no per-lane sorted
// lists, no LDS round trip of the score tile - and the kernel is a pure row stream:
//  * one 512-thread workgroup per CU (8 waves, 2 per SIMD); wave w owns 32 queries whose
//    bf16 fragments stay in registers for the whole launch (dim/4 VGPRs: 192 at 768), so
//    the query panel is never re-staged (the 128x128 tile kernel re-staged it for every
//    row tile: half of its LDS and L2 traffic);
//  * rows stream HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) in 32-row blocks through
//    a 3-buffer ring: two blocks (2 x 48 KB at dim 768) in flight while one is multiplied,
//    a counted vmcnt and one raw s_barrier per block;
//  * each wave-instruction fills 8 rows x 128 B (whole lines); within a row the eight
//    16-B slots are XOR-swizzled by (row >> 1) & 7 through the SOURCE addresses, which
//    makes the A-fragment ds_read_b128 of every MFMA step conflict-free;
//  * A = 32 rows, B = 32 queries: v_mfma_f32_32x32x16_bf16, one 48-MFMA chain per block
//    (k = 64c + 16s + 8h + j for chunk c, step s, lane half h - the same order in both
//    operands); lane (col, h) then holds 16 scores of ONE query.
// Two modes share the loop: TS_MAX (sample pass over every `period`-th block: per-lane
// running max -> lmax[list][q]) and TS_APPEND (every block: score >= tau[q] appended to
// the query's survivor list by one atomicAdd; rare by construction).
constexpr int kTsWaves = 8;      // waves per workgroup (32 queries each)
constexpr int kTsQ = kTsWaves * 32;  // queries per workgroup
constexpr int kTsBufs = 3;       // LDS ring depth
constexpr int kTsPeriod = 16;    // sample pass: every 16th block
constexpr int kTsRank = 8;       // tau = 8th largest list maximum of the sample (~128 survivors)

enum { TS_MAX = 0, TS_APPEND = 1 };

constexpr int kTsWaveSurv = 160;  // LDS survivor slots per wave (TS_APPEND; fills the 160 KB with NCH 12)
struct Survivor {
  float s;
  int row;
  int q;
};

typedef __attribute__((address_space(3))) void lds_void_t;

// One LDS-DMA wave-instruction: 16 B from base + voff (per lane) to LDS[lds_dst + 16 lane].
// Issued as inline asm: hipcc tracks a compiler-visible LDS-DMA as a pending LDS write
// and waits vmcnt(0) before every later ds_read of the same array, which would drain the
// ring's prefetch each block.  Completion is counted by hand (s_waitcnt vmcnt(N)).  The
// SGPR-base form keeps one 32-bit VGPR per address (the kernel runs at ~240 VGPRs: a
// spill reload inside the loop would wait vmcnt(0) and serialise the ring).
__device__ __forceinline__ void glds16(const void* base, unsigned voff, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

template <int NCH, int MODE>
__global__ __launch_bounds__(512, 2) void bf16_thresh_kernel(
    const uint4* __restrict__ Qb, int nq, const unsigned char* __restrict__ C, int64_t n_rows,
    int64_t n_blocks, int period, const float* __restrict__ tau, float* __restrict__ lmax,
    int* __restrict__ count, float* __restrict__ cs, int* __restrict__ ci) {
  constexpr int ROW_B = NCH * 128;             // bf16 row bytes
  constexpr int BLK_B = kTsRows * ROW_B;       // one staged block (the shadow is padded to
                                               // whole blocks: no row clamping)
  constexpr int DMA_PER_WAVE = NCH * 4 / kTsWaves;
  static_assert(NCH % 2 == 0 && DMA_PER_WAVE * kTsWaves == NCH * 4, "8 waves share a block's DMAs");
  // one LDS array: the row ring, then each wave's survivor list (TS_APPEND)
  constexpr int SURV_B = MODE == TS_APPEND ? kTsWaves * kTsWaveSurv * (int)sizeof(Survivor) : 0;
  __shared__ __attribute__((aligned(1024))) unsigned char ring[kTsBufs * BLK_B + SURV_B];
  Survivor* surv = reinterpret_cast<Survivor*>(ring + kTsBufs * BLK_B) + (threadIdx.x >> 6) * kTsWaveSurv;
  int n_surv = 0;  // wave-uniform
  const unsigned ring_lds = (unsigned)(uintptr_t)(lds_void_t*)ring;  // LDS byte address
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, h = lane >> 5;
  const int qw0 = blockIdx.y * kTsQ + wave * 32;  // this wave's first query
  const int q = min(qw0 + col, nq - 1);           // lanes past nq compute a duplicate column
  const bool qvalid = qw0 + col < nq;

  // query fragments: step (c, s), lane half h -> k = 64c + 16s + 8h .. +7
  bf16x8 qf[NCH * 4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[c * 4 + s] = __builtin_bit_cast(bf16x8, Qb[(int64_t)q * (NCH * 8) + c * 8 + 2 * s + h]);
  float t = MODE == TS_APPEND ? tau[q] : 0.f;
  // Retire the fragment loads here, visibly to the compiler: every later use reads the
  // asm's outputs, so no wait for these loads lands in the loop, where the (invisible)
  // DMAs of the ring would make any counted vmcnt drain the prefetch.
#pragma unroll
  for (int i = 0; i < NCH * 4; ++i) asm volatile("" : "+v"(qf[i]));
  asm volatile("" : "+v"(t));

  // this workgroup's blocks: j_i = (blockIdx.x + i * gridDim.x) * period
  const int64_t stride = (int64_t)gridDim.x * period;
  const int64_t first = (int64_t)blockIdx.x * period;
  const int nb = first < n_blocks ? (int)((n_blocks - 1 - first) / stride + 1) : 0;

  // DMA lane map: instruction d (chunk d >> 2, rows 8(d & 3) .. +7), lane p -> row
  // rl = 8(d & 3) + (p >> 3), 16-B slot u = (p & 7) ^ ((rl >> 1) & 7) of the chunk's 128 B.
  // (rl >> 1) & 7 = (4(d & 3) + (p >> 4)) & 7, so the per-lane part takes two values.
  unsigned dofs[2];
#pragma unroll
  for (int v = 0; v < 2; ++v)
    dofs[v] = (lane >> 3) * ROW_B + (((lane & 7) ^ ((4 * v + (lane >> 4)) & 7)) * 16);
  auto issue_one = [&](int i, int buf, int tt) __attribute__((always_inline)) {
    const int64_t j = first + (int64_t)min(i, nb - 1) * stride;  // past the end: re-read the last
    const int d = wave * DMA_PER_WAVE + tt;
    glds16(C + j * BLK_B, dofs[d & 1] + (unsigned)((d & 3) * 8 * ROW_B + (d >> 2) * 128),
           ring_lds + buf * BLK_B + d * 1024);
  };
  auto issue = [&](int i, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int tt = 0; tt < DMA_PER_WAVE; ++tt) issue_one(i, buf, tt);
  };
  // A-fragment read offsets: row `col` of the block, slot (2s + h) ^ ((col >> 1) & 7)
  const int rbase = (col >> 3) * 1024 + (col & 7) * 128;
  const int rx = (col >> 1) & 7;

  float mx = -INFINITY;
  if (nb > 0) {
    issue(0, 0);
    issue(1, 1);
  }
  const bool active = qw0 < nq;
  for (int i = 0; i < nb; ++i) {
    // own DMAs of block i landed (block i+1's may still fly), then everyone's, and every
    // wave is done reading block i-1, whose buffer this iteration refills
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_WAVE) : "memory");
    if (!(MQ_TS_DBG & 8)) __builtin_amdgcn_s_barrier();
    if (!active || (MQ_TS_DBG & 1)) {
      issue(i + 2, (i + 2) % kTsBufs);
      continue;
    }
    const unsigned char* blk = ring + (i % kTsBufs) * BLK_B + rbase;
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    // Hand-scheduled chain: fragment reads run three MFMA steps ahead (the compiler's own
    // order reads one step ahead and waits out the LDS latency before every other MFMA),
    // and block i+2's DMAs are spread over the chain, one every 8 steps, instead of
    // delaying its start.
    bf16x8 a[4];
    auto frag = [&](int st) __attribute__((always_inline)) {
      const int c = st >> 2, s = st & 3;
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(blk + c * 4096 + (((2 * s + h) ^ rx) * 16)));
    };
    a[0] = frag(0);
    a[1] = frag(1);
    a[2] = frag(2);
    static_for<NCH * 4>([&](auto sc) {
      constexpr int st = decltype(sc)::value;
      if constexpr (st % 8 == 0 && st / 8 < DMA_PER_WAVE && !(MQ_TS_DBG & 2))
        issue_one(i + 2, (i + 2) % kTsBufs, st / 8);
      if constexpr (st + 3 < NCH * 4) a[(st + 3) & 3] = (MQ_TS_DBG & 4) ? qf[(st + 5) % (NCH * 4)] : frag(st + 3);
      __builtin_amdgcn_sched_barrier(0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[st & 3], qf[st], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    const int64_t row0 = (first + (int64_t)i * stride) * kTsRows;
    const bool full = row0 + kTsRows <= n_rows;
    if constexpr (MODE == TS_MAX) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = row0 + acc_row(0, e, lane);
        if (full || row < n_rows) mx = fmaxf(mx, acc[e]);
      }
    } else {
      // survivors go to this wave's LDS list (a ballot + lane prefix picks the slots);
      // global slots are claimed only after the loop, so no returning atomic - whose
      // vmcnt(0) would drain the ring - ever runs inside it
      bool any = false;
#pragma unroll
      for (int e = 0; e < 16; ++e) any |= acc[e] >= t;
      if (__builtin_amdgcn_ballot_w64(any && qvalid)) {  // rare: ~128 survivors per query
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t row = row0 + acc_row(0, e, lane);
          const bool hit = acc[e] >= t && row < n_rows && qvalid;
          const unsigned long long m = __builtin_amdgcn_ballot_w64(hit);
          if (m) {
            const int pos = n_surv + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
            if (hit) {
              if (pos < kTsWaveSurv) {
                surv[pos] = Survivor{acc[e], (int)row, q};
              } else {  // list full: straight to global (drains the ring; rarer still)
                const int slot = atomicAdd(count + q, 1);
                if (slot < kTsCap) {
                  cs[(int64_t)q * kTsCap + slot] = acc[e];
                  ci[(int64_t)q * kTsCap + slot] = (int)row;
                }
              }
            }
            n_surv += __builtin_popcountll(m);
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-read DMAs
  if constexpr (MODE == TS_MAX) {
    if (qvalid) lmax[(int64_t)q * (2 * gridDim.x) + blockIdx.x * 2 + h] = mx;  // [q][list]
  } else {
    for (int j = lane; j < min(n_surv, kTsWaveSurv); j += 64) {  // flush the wave's list
      const Survivor v = surv[j];
      const int slot = atomicAdd(count + v.q, 1);
      if (slot < kTsCap) {
        cs[(int64_t)v.q * kTsCap + slot] = v.s;
        ci[(int64_t)v.q * kTsCap + slot] = v.row;
      }
    }
  }
}

// tau[q] = the kTsRank-th largest of the sample pass's per-list maxima (-inf when fewer
// lists saw a row), and the survivor count reset.  One wave per query.  The kTsRank-th
// largest list maximum is <= the kTsRank-th best sampled score (each of the top lists
// holds a distinct sampled row), so at least kTsRank rows survive.
__global__ __launch_bounds__(256) void bf16_tau_kernel(const float* __restrict__ lmax, int n_lists,
                                                       int nq, float* __restrict__ tau,
                                                       int* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  TopList<kTsRank> t;
  t.init();
  for (int l = lane; l < n_lists; l += 64) {
    const float x = lmax[(int64_t)q * n_lists + l];
    if (t.beats_tail(x, l)) t.insert(x, l);
  }
  float kth = -INFINITY;
  for (int r = 0; r < kTsRank; ++r) {
    float bs = t.s[0];
    int bi = t.id[0], bt = lane;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off);
      const int oi = __shfl_xor(bi, off), ot = __shfl_xor(bt, off);
      if (better(os, oi, bs, bi)) {
        bs = os;
        bi = oi;
        bt = ot;
      }
    }
    kth = bs;
    if (lane == bt && bi >= 0) t.pop_front();
  }
  if (lane == 0) {
    tau[q] = kth;
    count[q] = 0;
  }
}

// Survivors -> the query's top-kc candidates by (score desc, id asc), one block per
// query; slots past the survivor count hold (tau, -1), so the certificate's bound on a
// non-candidate is max(kc-th survivor, tau).  More than kTsCap survivors: the kept set
// is incomplete and the bound is set to +inf (the certificate then fails, the query is
// re-run one tier down).
__global__ __launch_bounds__(256) void bf16_select_kernel(const float* __restrict__ cs,
                                                          const int* __restrict__ ci,
                                                          const int* __restrict__ count,
                                                          const float* __restrict__ tau, int kc,
                                                          float* __restrict__ out_s,
                                                          int64_t* __restrict__ out_i) {
  __shared__ float ls[kTsCap];
  __shared__ int li[kTsCap];
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x;
  const int total = count[q];
  const int cnt = min(total, kTsCap);
  for (int i = tid; i < cnt; i += 256) {
    ls[i] = cs[q * kTsCap + i];
    li[i] = ci[q * kTsCap + i];
  }
  __syncthreads();
  for (int i = tid; i < cnt; i += 256) {
    const float x = ls[i];
    const int xi = li[i];
    int rank = 0;
    for (int j = 0; j < cnt; ++j) rank += better(ls[j], li[j], x, xi) ? 1 : 0;
    if (rank < kc) {
      out_s[q * kc + rank] = rank == kc - 1 && total > kTsCap ? INFINITY : x;
      out_i[q * kc + rank] = xi;
    }
  }
  for (int i = cnt + tid; i < kc; i += 256) {  // (never on overflow: kTsCap > kc)
    out_s[q * kc + i] = tau[q];
    out_i[q * kc + i] = -1;
  }
}

template <int NCH>
void launch_nch(const ThreshArgs& a, hipStream_t s, Timeline* tl) {
  // One workgroup per CU in total (LDS and VGPRs allow one): several query groups split
  // the CUs instead of running in rounds.  G is a multiple of the 8 XCDs, so (x, y) and
  // (x, y') sit on one XCD and stream the same blocks at about the same time through its
  // L2 - one HBM read serves every group.
  const int gy = (a.nq + kTsQ - 1) / kTsQ;
  const int G = gy == 1 ? a.num_cus : std::max(8, a.num_cus / gy / 8 * 8);
  const int64_t n_blocks = (a.n + kTsRows - 1) / kTsRows;
  const uint4* qb = reinterpret_cast<const uint4*>(a.q16);
  tl->mark(s, 0);
  hipLaunchKernelGGL((bf16_thresh_kernel<NCH, TS_MAX>), dim3(G, gy), dim3(512), 0, s, qb, a.nq, a.rows,
                     a.n, n_blocks, kTsPeriod, a.tau, a.lmax, a.count, a.cs, a.ci);
  tl->mark(s, 1);
  hipLaunchKernelGGL(bf16_tau_kernel, dim3((a.nq + 3) / 4), dim3(256), 0, s, a.lmax, 2 * G, a.nq, a.tau,
                     a.count);
  tl->mark(s, 0);
  hipLaunchKernelGGL((bf16_thresh_kernel<NCH, TS_APPEND>), dim3(G, gy), dim3(512), 0, s, qb, a.nq,
                     a.rows, a.n, n_blocks, 1, a.tau, a.lmax, a.count, a.cs, a.ci);
  tl->mark(s, 1);
  hipLaunchKernelGGL(bf16_select_kernel, dim3(a.nq), dim3(256), 0, s, a.cs, a.ci, a.count, a.tau, a.kc,
                     a.out_s, a.out_i);
}

void launch_thresh(const ThreshArgs& a, hipStream_t s, Timeline* tl) {
  switch (a.dim / 64) {
    case 4: launch_nch<4>(a, s, tl); break;
    case 8: launch_nch<8>(a, s, tl); break;
    default: launch_nch<12>(a, s, tl); break;
  }
}

}  // namespace mq
