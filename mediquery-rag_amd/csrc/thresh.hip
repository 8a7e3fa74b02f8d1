// thresh.hip - K9t: the bf16 threshold scan that produces the candidates of batched
// bf16 searches (the certified screen's first tier, MQ_DTYPE_F32_SCREEN, and BASELINE
// config 5's coarse scan, MQ_DTYPE_BF16) - the top-k half of Chroma's similarity_search
// (reference src/agents/nodes.py:93) at batch scale.  See DESIGN.md §4.
#include "gemm_f32.hpp"

#ifndef MQ_TS_DBG  // measurement builds only (wrong results): 1 = stream only, 2 = multiply
                   // only, 4 = no fragment reads, 8 = no barrier
#define MQ_TS_DBG 0
#endif
#if MQ_TS_DBG != 0 && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_TS_DBG computes wrong results: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
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
// Waves that issue the ring's DMAs.  4 = waves 0-3, one per SIMD: the other wave of every
// SIMD runs its MFMA chain without DMA issues.  Measured (profiles/r6/k9t_dma_waves.txt, one
// box, 1M rows): K9t append 453 us at 8 waves, 398 at 4, 543 at 2, 577 at 1 (B = 256).
#ifndef MQ_TS_DMAW
#define MQ_TS_DMAW 4
#endif
constexpr int kTsDmaWaves = MQ_TS_DMAW;
static_assert(kTsDmaWaves == 8 || kTsDmaWaves == 4 || kTsDmaWaves == 2 || kTsDmaWaves == 1, "DMA waves");
constexpr int kTsQ = kTsWaves * 32;  // queries per workgroup
constexpr int kTsBufs = 3;       // LDS ring depth
constexpr int kTsPeriod = 16;    // sample pass: every 16th block
#ifndef MQ_TS_BF_PERIOD
#define MQ_TS_BF_PERIOD 16
#endif
constexpr int kTsBfPeriod = MQ_TS_BF_PERIOD;  // ... of the bf16 scan

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
#ifndef MQ_TS_NT  // 1: the ring's row stream is non-temporal.  Measured (r4): -2% at one query group
#define MQ_TS_NT 0    // (B <= 256), +4% at four (B = 1024: the groups re-read the rows), so off
#endif
__device__ __forceinline__ void glds16(const void* base, unsigned voff, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
#if MQ_TS_NT
      " nt"
#endif
      "\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

// MASKED (batched filtered search): a 32-row block's rows are bits 0..31 of mask word j
// (block j); a masked row is absent from both passes.  The word is read by a scalar load
// waited at once at the top of the block (asm: a compiler-visible SMEM load outstanding
// across the chain would turn its counted LDS waits into lgkmcnt(0)).
template <int NCH, int MODE, bool MASKED = false>
__global__ __launch_bounds__(512, 2) void bf16_thresh_kernel(
    const uint4* __restrict__ Qb, int nq, const unsigned char* __restrict__ C, int64_t n_rows,
    int64_t n_blocks, int period, const float* __restrict__ tau, float* __restrict__ lmax,
    int* __restrict__ count, float* __restrict__ cs, int* __restrict__ ci,
    const unsigned* __restrict__ mask) {
  constexpr int ROW_B = NCH * 128;             // bf16 row bytes
  constexpr int BLK_B = kTsRows * ROW_B;       // one staged block (the shadow is padded to
                                               // whole blocks: no row clamping)
  constexpr int DMA_PER_WAVE = NCH * 4 / kTsDmaWaves;  // (waves past kTsDmaWaves issue none)
  constexpr int DSTEP = NCH * 4 / DMA_PER_WAVE;         // chain steps between a wave's DMAs
  static_assert(NCH % 2 == 0 && DMA_PER_WAVE * kTsDmaWaves == NCH * 4, "the DMA waves share a block's DMAs");
  // one LDS array: the row ring, then each wave's survivor list (TS_APPEND)
  constexpr int SURV_B = MODE == TS_APPEND ? kTsWaves * kTsWaveSurv * (int)sizeof(Survivor) : 0;
  __shared__ __attribute__((aligned(1024))) unsigned char ring[kTsBufs * BLK_B + SURV_B];
  Survivor* surv = reinterpret_cast<Survivor*>(ring + kTsBufs * BLK_B) + (threadIdx.x >> 6) * kTsWaveSurv;
  int n_surv = 0;  // wave-uniform
  const unsigned ring_lds = (unsigned)(uintptr_t)(lds_void_t*)ring;  // LDS byte address
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dma_wave = wave < kTsDmaWaves;
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
  // (measurement builds that replace operands score garbage: no row may clear tau there)
  float t = MODE == TS_APPEND ? (MQ_TS_DBG & 6 ? INFINITY : tau[q]) : 0.f;
  // Retire the fragment loads here, visibly to the compiler: every later use reads the
  // asm's outputs, so no wait for these loads lands in the loop, where the (invisible)
  // DMAs of the ring would make any counted vmcnt drain the prefetch.
#pragma unroll
  for (int i = 0; i < NCH * 4; ++i) asm volatile("" : "+v"(qf[i]));
  asm volatile("" : "+v"(t));

  const int n_rows_i = (int)min(n_rows, (int64_t)INT_MAX);
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
    if (!dma_wave) return;
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
    // (MASKED) block i's row bits: a scalar load, here for the sample pass; the append
    // pass loads them in its rare survivor path only
    auto mask_word = [&]() __attribute__((always_inline)) {
      unsigned w;
      const unsigned* mp = mask + (first + (int64_t)i * stride);
      asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w) : "s"(mp) : "memory");
      return w;
    };
    unsigned mw = ~0u;
    if constexpr (MASKED && MODE == TS_MAX) mw = mask_word();
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
    // and block i+2's DMAs (DMA waves only) are spread over the chain, one every DSTEP
    // steps, instead of delaying its start.
    bf16x8 a[4];
    auto frag = [&](int st) __attribute__((always_inline)) {
      const int c = st >> 2, s = st & 3;
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(blk + c * 4096 + (((2 * s + h) ^ rx) * 16)));
    };
    a[0] = frag(0);
    a[1] = frag(1);
    a[2] = frag(2);
    // block i+2's source and ring slot, once per block (not per DMA slot)
    const unsigned char* nsrc = C + (first + (int64_t)min(i + 2, nb - 1) * stride) * BLK_B;
    const unsigned nlds = ring_lds + ((i + 2) % kTsBufs) * BLK_B;
    static_for<NCH * 4>([&](auto sc) {
      constexpr int st = decltype(sc)::value;
      if constexpr (st % DSTEP == 0 && st / DSTEP < DMA_PER_WAVE && !(MQ_TS_DBG & 2)) {
        if (dma_wave) {
          const int d = wave * DMA_PER_WAVE + st / DSTEP;
          glds16(nsrc, dofs[d & 1] + (unsigned)((d & 3) * 8 * ROW_B + (d >> 2) * 128), nlds + d * 1024);
        }
      }
      if constexpr (st + 3 < NCH * 4) a[(st + 3) & 3] = (MQ_TS_DBG & 4) ? qf[(st + 5) % (NCH * 4)] : frag(st + 3);
      __builtin_amdgcn_sched_barrier(0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[st & 3], qf[st], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    const int64_t row0 = (first + (int64_t)i * stride) * kTsRows;
    const bool full = row0 + kTsRows <= n_rows;
    if constexpr (MASKED && MODE == TS_MAX) {
      // rows outside the mask score -inf, in place.  The lane's mask word and the fill
      // value are made here, by asm the compiler cannot hoist above the chain, where
      // every VGPR is taken (acc element e is row (e & 3) + 8 (e >> 2) + 4 h)
      unsigned mwl;
      float off;
      asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(mwl) : "v"(4 * h), "s"(mw));
      asm volatile("v_mov_b32 %0, %1" : "=v"(off) : "i"(0xff800000u));
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (!((mwl >> ((e & 3) + 8 * (e >> 2))) & 1u)) acc[e] = off;
    }
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
        // (MASKED: the lane's mask word, by asm so that it is not hoisted out of the loop)
        unsigned mwl = 0;
        if constexpr (MASKED) asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(mwl) : "v"(4 * h), "s"(mask_word()));
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = (int)row0 + acc_row(0, e, lane);  // (ids are 32-bit: Survivor, ci)
          // (MASKED: the mask is applied here only - a masked row that clears tau enters
          // this rare path and is dropped; any mask term in the every-block test above cost
          // the append kernel a spilled query fragment, reloaded per block)
          const bool hit = acc[e] >= t && row < n_rows_i && qvalid &&
                           (!MASKED || ((mwl >> ((e & 3) + 8 * (e >> 2))) & 1u));
          const unsigned long long m = __builtin_amdgcn_ballot_w64(hit);
          if (m) {
            const int pos = n_surv + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
            if (hit) {
              if (pos < kTsWaveSurv) {
                surv[pos] = Survivor{acc[e], row, q};
              } else {  // list full: straight to global (drains the ring; rarer still)
                const int slot = atomicAdd(count + q, 1);
                if (slot < kTsCap) {
                  cs[(int64_t)q * kTsCap + slot] = acc[e];
                  ci[(int64_t)q * kTsCap + slot] = row;
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
// rank <= 64: each lane keeps its best kTsRank lists (all of them when n_lists <= 512 =
// 2 x 256 CUs; with more, dropping a lane's lower maxima can only lower tau).
__global__ __launch_bounds__(256) void bf16_tau_kernel(const float* __restrict__ lmax, int n_lists,
                                                       int nq, int rank, float* __restrict__ tau,
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
  for (int r = 0; r < rank; ++r) {
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
// re-run one tier down).  With `fail` set (the approximate bf16 mode, no certificate), a
// query with more than kTsCap or fewer than kc survivors is appended to fail[] instead,
// for the caller to re-run on the tiled scan.
//
// Past 256 survivors (a block-uniform branch) ranks are counted only among the survivors
// that can still place: T = the kc-th best of the 256 threads' own best survivors bounds
// the kc-th best overall from below (the thread maxima are distinct survivors), so every
// survivor worse than T has rank >= kc, and every survivor better than one at or above T
// is at or above T too - ranks counted in the filtered set are the exact ranks (the same
// output as counting over all survivors, at O(n + 256^2 + m^2) instead of O(n^2): a query
// with thousands of survivors held the whole launch for 30-500 us).
__global__ __launch_bounds__(256) void bf16_select_kernel(const float* __restrict__ cs,
                                                          const int* __restrict__ ci,
                                                          const int* __restrict__ count,
                                                          const float* __restrict__ tau, int kc,
                                                          float* __restrict__ out_s,
                                                          int64_t* __restrict__ out_i,
                                                          int* __restrict__ fail_count,
                                                          int64_t* __restrict__ fail) {
  __shared__ float ls[kTsCap], fs[kTsCap], ts[256];
  __shared__ int li[kTsCap], fi[kTsCap], ti[256];
  __shared__ float cut_s;
  __shared__ int cut_i, nf;
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x;
  const int total = count[q];
  if (fail && tid == 0 && (total > kTsCap || total < kc)) fail[atomicAdd(fail_count, 1)] = q;
  const int cnt = min(total, kTsCap);
  float bs = -INFINITY;
  int bi = -1;  // no survivor (as unsigned: after every real id)
  for (int i = tid; i < cnt; i += 256) {
    const float x = cs[q * kTsCap + i];
    const int xi = ci[q * kTsCap + i];
    ls[i] = x;
    li[i] = xi;
    if (bi == -1 || better(x, (unsigned)xi, bs, (unsigned)bi)) {
      bs = x;
      bi = xi;
    }
  }
  // exact rank of each of the m survivors in (rs, ri) among them; the top kc go out
  auto rank_out = [&](const float* rs, const int* ri, int m) __attribute__((always_inline)) {
    for (int i = tid; i < m; i += 256) {
      const float x = rs[i];
      const int xi = ri[i];
      int rank = 0;
      for (int j = 0; j < m; ++j) rank += better(rs[j], (unsigned)ri[j], x, (unsigned)xi) ? 1 : 0;
      if (rank < kc) {
        out_s[q * kc + rank] = rank == kc - 1 && total > kTsCap ? INFINITY : x;
        out_i[q * kc + rank] = xi;
      }
    }
  };
  if (cnt <= 256) {
    __syncthreads();
    rank_out(ls, li, cnt);
  } else {
    ts[tid] = bs;
    ti[tid] = bi;
    if (tid == 0) {
      cut_s = -INFINITY;  // (kc > 256: no cut)
      cut_i = -1;
      nf = 0;
    }
    __syncthreads();
    int rank = 0;  // every thread holds a survivor here
    for (int j = 0; j < 256; ++j) rank += better(ts[j], (unsigned)ti[j], bs, (unsigned)bi) ? 1 : 0;
    if (rank == kc - 1) {
      cut_s = bs;
      cut_i = bi;
    }
    __syncthreads();
    const float Ts = cut_s;
    const unsigned Ti = (unsigned)cut_i;
    // the survivors at or above T to fs / fi: a ballot and lane prefix per wave, one LDS
    // slot claim per wave and round
    const int lane = tid & 63;
    for (int base = 0; base < cnt; base += 256) {
      const int i = base + tid;
      const bool keep = i < cnt && !better(Ts, Ti, ls[i], (unsigned)li[i]);
      const unsigned long long bal = __ballot(keep);
      int slot0 = 0;
      if (lane == 0 && bal) slot0 = atomicAdd(&nf, __popcll(bal));
      slot0 = __shfl(slot0, 0);
      if (keep) {
        const int slot = slot0 + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
        fs[slot] = ls[i];
        fi[slot] = li[i];
      }
    }
    __syncthreads();
    rank_out(fs, fi, nf);
  }
  for (int i = cnt + tid; i < kc; i += 256) {  // (never on overflow: kTsCap > kc)
    out_s[q * kc + i] = tau[q];
    out_i[q * kc + i] = -1;
  }
}

template <int NCH, bool MASKED>
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
  hipLaunchKernelGGL((bf16_thresh_kernel<NCH, TS_MAX, MASKED>), dim3(G, gy), dim3(512), 0, s, qb, a.nq, a.rows,
                     a.n, n_blocks, kTsBfPeriod, a.tau, a.lmax, a.count, a.cs, a.ci, a.mask);
  tl->mark(s, 1);
  hipLaunchKernelGGL(bf16_tau_kernel, dim3((a.nq + 3) / 4), dim3(256), 0, s, a.lmax, 2 * G, a.nq,
                     a.tau_rank, a.tau, a.count);
  tl->mark(s, 0);
  hipLaunchKernelGGL((bf16_thresh_kernel<NCH, TS_APPEND, MASKED>), dim3(G, gy), dim3(512), 0, s, qb, a.nq,
                     a.rows, a.n, n_blocks, 1, a.tau, a.lmax, a.count, a.cs, a.ci, a.mask);
  tl->mark(s, 1);
  hipLaunchKernelGGL(bf16_select_kernel, dim3(a.nq), dim3(256), 0, s, a.cs, a.ci, a.count, a.tau, a.kc,
                     a.out_s, a.out_i, a.fail_count, a.fail);
}

template <bool MASKED>
void launch_dim(const ThreshArgs& a, hipStream_t s, Timeline* tl) {
  switch (a.dim / 64) {
    case 4: launch_nch<4, MASKED>(a, s, tl); break;
    case 8: launch_nch<8, MASKED>(a, s, tl); break;
    default: launch_nch<12, MASKED>(a, s, tl); break;
  }
}

void launch_thresh(const ThreshArgs& a, hipStream_t s, Timeline* tl) {
  if (a.mask)
    launch_dim<true>(a, s, tl);
  else
    launch_dim<false>(a, s, tl);
}

// ============================ K9q: int8 threshold scan (few-query screens) ==========
// A single query (or up to 4) over the int8 shadow: a row is stored as int8 r8 with one
// fp32 scale (absmax / 127), 1 byte per element - half the bytes of the bf16 shadow that
// bounds the few-query screen (HBM-bound: ~0.13 instead of ~0.24 ms at 1M x 768).  The
// screen score of row c is fl(scale_c * fl(sum_j q_j r8_cj)) with the fp32 query; its
// error against the exact dot is bounded as in VERIFY_BF16_Q32 with the int8 shadow's own
// maxima (dmax = max ||c - scale_c r8_c||, cmax = max ||scale_c r8_c||).  Same threshold
// scheme as K9t (sample pass -> tau -> appending pass -> select; tau is found inside the
// appending pass, the select fused with the re-rank in index.hip), on the VALU: lane l
// holds elements [l E, l E + E) of every row (E = dim / 64) and of the query, in
// registers; a wave takes 8 rows per step (8 x dim bytes, contiguous), converts and
// multiplies, and one transposed butterfly (xor 32 / 16 / 8 halving the values, then
// xor 4 / 2 / 1) leaves lane l with row 4 b5 + 2 b4 + b3 of the 8.

// int8 shadow of rows [0, n) + scales + per-row errors + the screen statistics (float bits,
// atomicMax).  One wave per row, rows strided over a grid of a few waves per SIMD; lane l
// quantises elements [l E, l E + E), E = 4 * E4.  Each wave keeps its running maxima and
// issues one atomicMax pair at the end (one pair per row serialised ~1M same-address
// atomics: 22.7 ms per 1M rows).
template <int E4>
__global__ __launch_bounds__(256) void i8_shadow_kernel(const float* __restrict__ src, int64_t n,
                                                        unsigned* __restrict__ r8,
                                                        float* __restrict__ scale,
                                                        float* __restrict__ err,
                                                        unsigned* __restrict__ stats) {
  constexpr int E = 4 * E4, DIM = 64 * E;
  const int lane = threadIdx.x & 63;
  float emax = 0.f, cmax = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    floatx4 x[E4];
    float amax = 0.f;
#pragma unroll
    for (int d = 0; d < E4; ++d) {
      x[d] = *reinterpret_cast<const floatx4*>(src + row * DIM + lane * E + 4 * d);
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(x[d].x), fabsf(x[d].y)), fmaxf(fabsf(x[d].z), fabsf(x[d].w))));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    const float sc = amax / 127.f, inv = amax > 0.f ? 127.f / amax : 0.f;
    float se = 0.f, sd = 0.f;
#pragma unroll
    for (int d = 0; d < E4; ++d) {
      unsigned w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float v = x[d][b];
        const float r = fminf(fmaxf(rintf(v * inv), -127.f), 127.f);
        const float deq = sc * r;
        se += (v - deq) * (v - deq);
        sd += deq * deq;
        w |= ((unsigned)(int)r & 0xffu) << (8 * b);
      }
      r8[row * (DIM / 4) + lane * E4 + d] = w;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      se += __shfl_xor(se, off);
      sd += __shfl_xor(sd, off);
    }
    const float e = sqrtf(se);
    if (lane == 0) {
      scale[row] = sc;
      err[row] = e;
    }
    emax = fmaxf(emax, e);
    cmax = fmaxf(cmax, sqrtf(sd));
  }
  if (lane == 0 && cmax > 0.f) {
    atomicMax(stats, __float_as_uint(emax));
    atomicMax(stats + 1, __float_as_uint(cmax));
  }
}

// order-preserving float <-> unsigned (key 0 is below every float)
__device__ __forceinline__ unsigned ord_key(float x) {
  const unsigned b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_ord(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

#ifndef MQ_I8_CERT_DBG  // measurement builds only: 1 = tau without the certificate term (r4's tau),
                        // 2 = the certificate term computed, r4's tau kept
#define MQ_I8_CERT_DBG 0
#endif
#if MQ_I8_CERT_DBG != 0 && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_I8_CERT_DBG breaks the int8 certificate: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
#endif
#ifndef MQ_I8_ROWS
#define MQ_I8_ROWS 8
#endif
#ifndef MQ_I8_NT  // 1: the int8 shadow streams with non-temporal loads (read once per search)
#define MQ_I8_NT 1
#endif
constexpr int kI8Rows = MQ_I8_ROWS;  // rows per wave step (8 or 16)
#ifndef MQ_I8_STAGES
#define MQ_I8_STAGES 3
#endif
#ifndef MQ_I8_TAU_POP
#define MQ_I8_TAU_POP 1  // in-kernel tau: per-lane top-k + wave pops (1) or bitwise ballot search (0)
#endif
constexpr int kI8Stages = MQ_I8_STAGES;  // register stages of the row stream (2 or 3: 3 measured
                                         // 2-3 us faster per search, 158 VGPRs, no spills)
static_assert(kI8Stages == 2 || kI8Stages == 3, "2 or 3 register stages");
constexpr int kI8Lg = kI8Rows == 16 ? 4 : 3;
static_assert(kI8Rows == 1 << kI8Lg, "8 or 16 rows per step");

// values v[0 .. R NQ) indexed r * NQ + q -> lane l holds v[0 .. NQ) of row i8_row(l),
// summed over the 64 lanes: log2 R halving exchanges (xor 32, 16, ...), then a plain
// butterfly over the remaining lane bits.  A halving step pairs x = v[i] with
// y = v[i + c/2]: lanes with bit m clear keep x and add their partner's x, the others
// keep y and add their partner's y.  For m = 32 / 16 that is exactly one gfx950
// v_permlane{32,16}_swap of (x, y) followed by x' + y' (no lane selects); for m = 8 / 4 a
// select of the two values and one DPP row_ror:8 / swizzle xor-4 move.  Written as
// `hi ? v[i + c/2] : v[i]` the compiler turned the selects into dynamically indexed
// register chains (7 v_cmp + 7 v_cndmask per value, ~200 VALU per 8-row step).
__device__ __forceinline__ int i8_row(int lane) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < kI8Lg; ++i) r |= ((lane >> (5 - i)) & 1) << (kI8Lg - 1 - i);
  return r;
}

template <int NQ>
__device__ __forceinline__ void transpose_reduce(float (&v)[kI8Rows * NQ], int lane) {
#pragma unroll
  for (int m = 32, c = kI8Rows * NQ; m >= 64 / kI8Rows; m >>= 1, c >>= 1) {
#pragma unroll
    for (int i = 0; i < c / 2; ++i) {
      const float x = v[i], y = v[i + c / 2];
      if (m == 32 || m == 16) {
        const auto r = m == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false)
                               : __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      } else {
        const bool hi = (lane & m) != 0;
        const float keep = hi ? y : x, give = hi ? x : y;
        v[i] = keep + xor_move(give, m);
      }
    }
  }
#pragma unroll
  for (int m = 32 / kI8Rows; m > 0; m >>= 1)
#pragma unroll
    for (int i = 0; i < NQ; ++i) v[i] += xor_move(v[i], m);
}

template <int E4>
__device__ __forceinline__ void i8_load(const unsigned* __restrict__ r8, int64_t unit, int lane,
                                        unsigned (&a)[kI8Rows][E4]) {
  constexpr int DIM4 = 64 * E4;  // dwords per row (dim = 256 E4 one-byte elements)
#pragma unroll
  for (int r = 0; r < kI8Rows; ++r) {
    const unsigned* p = r8 + (unit * kI8Rows + r) * DIM4 + lane * E4;
#pragma unroll
    for (int d = 0; d < E4; ++d) a[r][d] = MQ_I8_NT ? __builtin_nontemporal_load(p + d) : p[d];
  }
}

template <int E4, int NQ>
__device__ __forceinline__ void i8_dot(const unsigned (&a)[kI8Rows][E4], const float (&qv)[NQ][4 * E4],
                                       float (&v)[kI8Rows * NQ]) {
  // two rows per packed FMA (v_pk_fma_f32: one instruction for both rows' products,
  // each row's chain in the same element order as a scalar fma chain)
  typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int r = 0; r < kI8Rows; r += 2) {
    f2 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = f2{0.f, 0.f};
#pragma unroll
    for (int d = 0; d < E4; ++d)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const f2 x = {(float)((int)(a[r][d] << (24 - 8 * b)) >> 24),  // signed byte b
                      (float)((int)(a[r + 1][d] << (24 - 8 * b)) >> 24)};
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const f2 qq = {qv[q][4 * d + b], qv[q][4 * d + b]};
          acc[q] = __builtin_elementwise_fma(qq, x, acc[q]);
        }
      }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      v[r * NQ + q] = acc[q].x;
      v[(r + 1) * NQ + q] = acc[q].y;
    }
  }
}

// MODE TS_MAX: every `period`-th unit, per-workgroup maxima -> lmax[q][workgroup];
// TS_APPEND: every unit, score >= tau[q] appended to the query's survivors.
template <int E4, int NQ, int MODE>
__global__ __launch_bounds__(256, kI8WgPerCu) void i8_thresh_kernel(
    const float* __restrict__ Q, int nq, const unsigned* __restrict__ r8, const float* __restrict__ scale,
    int64_t n_rows, int64_t n_units, int period, float* __restrict__ tau, const float* __restrict__ lmax_in,
    int* __restrict__ count, float* __restrict__ cs, int* __restrict__ ci, int* __restrict__ zero,
    const unsigned* __restrict__ stats, int kcert, const unsigned* __restrict__ mask) {
  constexpr int E = 4 * E4, DIM = 64 * E;
  if (MQ_I8_CERT_DBG & 1) kcert = 0;
  float* lmax = const_cast<float*>(lmax_in);  // written by TS_MAX, read by TS_APPEND
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int W = gridDim.x * 4;
  float qv[NQ][E];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float* src = Q + (int64_t)min(q, nq - 1) * DIM + lane * E;
#pragma unroll
    for (int d = 0; d < E4; ++d) {
      const floatx4 t = *reinterpret_cast<const floatx4*>(src + 4 * d);
      qv[q][4 * d] = t.x;
      qv[q][4 * d + 1] = t.y;
      qv[q][4 * d + 2] = t.z;
      qv[q][4 * d + 3] = t.w;
    }
  }
  float th[NQ], mx[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    th[q] = 0.f;
    mx[q] = -INFINITY;
  }
  if (MODE == TS_MAX && blockIdx.x == 0 && threadIdx.x == 0 && zero) *zero = 0;  // caller's flag
  const int my_r = i8_row(lane);
  __shared__ int seg_n[NQ];  // TS_APPEND: this workgroup's survivors per query
  const int64_t stride = (int64_t)W * period;
  unsigned a[kI8Stages][kI8Rows][E4];
  float sc[kI8Stages];
  unsigned mw[kI8Stages];  // (mask) the word holding this lane's row's bit
  int64_t u = (int64_t)gw * period;
  auto fetch = [&](int buf, int64_t unit) {
    const int64_t uu = min(unit, n_units - 1);  // past the end: re-read the last unit
    i8_load<E4>(r8, uu, lane, a[buf]);
    sc[buf] = scale[uu * kI8Rows + my_r];  // (padding rows: allocated, unused)
    mw[buf] = mask ? mask[(uu * kI8Rows + my_r) >> 5] : ~0u;  // (rows < 8 n_units <= 32 ceil(n / 32))
  };
  auto consume = [&](int buf, int64_t unit) {
    float v[kI8Rows * NQ];
    i8_dot<E4, NQ>(a[buf], qv, v);
    transpose_reduce<NQ>(v, lane);
    const int64_t row = unit * kI8Rows + my_r;
    const bool valid = row < n_rows && ((mw[buf] >> (row & 31)) & 1u);  // masked rows do not exist
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float score = v[q] * sc[buf];
      if (MODE == TS_MAX) {
        mx[q] = valid ? fmaxf(mx[q], score) : mx[q];
      } else if ((lane & (64 / kI8Rows - 1)) == 0 && valid && q < nq && score >= th[q]) {
        const int slot = atomicAdd(&seg_n[q], 1);  // LDS
        if (slot < kI8Seg) {
          const int64_t at = ((int64_t)q * gridDim.x + blockIdx.x) * kI8Seg + slot;
          cs[at] = score;
          ci[at] = (int)row;
        }
      }
    }
  };
  // kI8Stages register stages: the next kI8Stages - 1 units' loads are in flight while
  // one is multiplied (stage indices are compile-time: no register indexing)
  // tau per query from the sample pass's n_lists = gridDim.x workgroup maxima, computed
  // in every workgroup by wave 0 (same inputs, same steps: the same tau everywhere)
  // instead of a separate launch: the kTsRank-th largest maximum by a bitwise search on
  // order-preserving keys with ballot counts; workgroup 0 stores it for the select.  The
  // maxima are loaded before the first rows, so the search runs under their latency.
  constexpr int kPer = kI8MaxLists / 64;  // lists per lane
  __shared__ float th_sh[NQ];
  const bool tau_wave = MODE == TS_APPEND && (threadIdx.x >> 6) == 0;
  unsigned key[NQ][kPer];
  float st_d = 0.f, st_c = 0.f;  // the shadow's maxima (kcert > 0), loaded with the keys
  if (tau_wave) {
    if (kcert > 0 && stats) {
      st_d = __uint_as_float(stats[0]);
      st_c = __uint_as_float(stats[1]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int l = lane + 64 * j;
        key[q][j] = l < (int)gridDim.x ? ord_key(lmax[(int64_t)min(q, nq - 1) * gridDim.x + l]) : 0u;
      }
  }
  if (u < n_units) fetch(0, u);
  if (kI8Stages == 3 && u < n_units) fetch(1, u + stride);
  if (MODE == TS_APPEND) {
    if (tau_wave) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
#if MQ_I8_TAU_POP
        // the kTsRank-th largest key (with multiplicity): each lane keeps its own top
        // kPop keys (compare-exchange insertion), then rounds of a wave max whose lowest
        // holder pops its head - ~450 VALU instead of 32 rounds of kPer ballots (~4k
        // instructions while the workgroup's other waves wait at the barrier).  Same T.
        // With kcert > 0 the pops run on to the kcert-th largest (Tk) and the kPop-th (the
        // floor) as well.  Each lane keeps only its best kDepth keys: a lane holding more
        // of the top kPop drops some, so a popped rank can only come out LOWER than the
        // true one - a lower tau (more survivors), never an unsound certificate.
        constexpr int kPop = 32, kDepth = 8;  // kPop >= kTsRank, kScreenMaxK
        unsigned top[kDepth];
#pragma unroll
        for (int i = 0; i < kDepth; ++i) top[i] = 0u;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          if (64 * j < (int)gridDim.x) {  // (uniform) lists past the grid hold key 0
            unsigned x = key[q][j];
#pragma unroll
            for (int i = 0; i < kDepth; ++i) {
              const unsigned hi = max(top[i], x);
              x = min(top[i], x);
              top[i] = hi;
            }
          }
        }
        unsigned T = 0, Tk = 0, Tf = 0;
        const int pops = kcert > 0 ? kPop : kTsRank;
        for (int r = 0; r < pops; ++r) {
          const unsigned m = wave_max_u32(top[0]);
          if (r == kTsRank - 1) T = m;
          if (r == kcert - 1) Tk = m;
          if (r == kPop - 1) Tf = m;
          const unsigned long long holders = __ballot(top[0] == m);
          if (r + 1 < pops && lane == (int)__builtin_ctzll(holders)) {
#pragma unroll
            for (int i = 0; i + 1 < kDepth; ++i) top[i] = top[i + 1];
            top[kDepth - 1] = 0u;
          }
        }
        if (kcert > 0 && stats) {
          // tau <= Tk - 2E: the kcert best sampled rows (one per top list) score >= Tk on
          // the screen, so exact >= Tk - E each, hence e_k >= Tk - E > tau + E - the
          // finish's certificate holds whenever every survivor is kept (the k-th best
          // sample of a clustered query is a cluster-mate, its 8th list maximum too
          // close to e_k: measured gaps ~0.01 against E ~0.013, tools/i8_cert_probe.py).  E as
          // screen_bound(VERIFY_BF16_Q32) computes it (1% and 1e-6 slack for the
          // different summation order of ||q||)
          float ss = 0.f;
#pragma unroll
          for (int e = 0; e < E; ++e) ss += qv[q][e] * qv[q][e];
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
          const float qn = sqrtf(ss);
          const float dmax = st_d * 1.001f, cmax = st_c * 1.001f;
          const float g = 2.f * (float)DIM * 5.9604645e-8f;
          const float Eb = (qn * dmax + g * qn * (cmax + dmax) + g * qn * cmax) * 1.001f + 1e-7f;
          const float tk = Tk == 0u ? -INFINITY : key_ord(Tk);
          const float tc = tk - 2.02f * Eb - 1e-6f;
          const float t8 = T == 0u ? -INFINITY : key_ord(T);
          // ... floored at the kPop-th largest maximum (>= 32 sampled rows: ~512 survivors
          // expected), so a k-th best sample far below the true k-th best (k large against
          // the query's cluster) cannot flood the survivor lists; then the certificate is
          // no longer guaranteed, only likely.  (The 16th failed 7 of 100 clustered k = 5
          // queries by < 0.001: their 16th sample was still a cluster-mate,
          // tools/i8_cert_probe.py)
          const float tf = Tf == 0u ? -INFINITY : key_ord(Tf);
          const float t = fminf(t8, fmaxf(tc, tf));
          T = (MQ_I8_CERT_DBG & 2) ? T : t == -INFINITY ? 0u : ord_key(t);
        }
#else
        unsigned T = 0;
        for (int b = 31; b >= 0; --b) {
          const unsigned cand = T | (1u << b);
          int c = 0;
#pragma unroll
          for (int j = 0; j < kPer; ++j) c += __popcll(__ballot(key[q][j] >= cand));
          if (c >= kTsRank) T = cand;
        }
#endif
        const float t = T == 0u ? -INFINITY : key_ord(T);
        if (lane == 0) {
          th_sh[q] = t;
          if (blockIdx.x == 0 && q < nq) tau[q] = t;
        }
      }
    }
    if (threadIdx.x < NQ) seg_n[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q) th[q] = th_sh[q];
  }
  if constexpr (kI8Stages == 2) {
    // two register stages: the next unit's loads are in flight while one is multiplied
    while (u < n_units) {
      const int64_t u1 = u + stride;
      fetch(1, u1);
      consume(0, u);
      if (u1 >= n_units) break;
      const int64_t u2 = u1 + stride;
      fetch(0, u2);
      consume(1, u1);
      u = u2;
    }
  } else {
    // three: the next two units' loads are in flight while one is multiplied (stage
    // (i mod 3) holds unit u + i stride; fetch clamps past-the-end units to the last one)
    constexpr int s2 = kI8Stages - 1;  // (2; the branch is only taken with three stages)
    while (u < n_units) {
      fetch(s2, u + 2 * stride);
      consume(0, u);
      if (u + stride >= n_units) break;
      fetch(0, u + 3 * stride);
      consume(1, u + stride);
      if (u + 2 * stride >= n_units) break;
      fetch(1, u + 4 * stride);
      consume(s2, u + 2 * stride);
      u += 3 * stride;
    }
  }
  if (MODE == TS_APPEND) {  // the segment counts
    __syncthreads();
    if (threadIdx.x < nq) count[threadIdx.x * gridDim.x + blockIdx.x] = seg_n[threadIdx.x];
  }
  if (MODE == TS_MAX) {  // workgroup maxima: one list per workgroup (a shorter tau pass)
    __shared__ float wmax[4][NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float m = mx[q];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
      if (lane == 0) wmax[threadIdx.x >> 6][q] = m;
    }
    __syncthreads();
    if (threadIdx.x < NQ && (int)threadIdx.x < nq) {
      const int q = threadIdx.x;
      lmax[(int64_t)q * gridDim.x + blockIdx.x] =
          fmaxf(fmaxf(wmax[0][q], wmax[1][q]), fmaxf(wmax[2][q], wmax[3][q]));
    }
  }
}

template <int E4>
void i8_shadow_e4(const float* rows, int64_t n, unsigned* r8, float* scale, float* err, unsigned* stats,
                  hipStream_t s) {
  const unsigned grid = (unsigned)std::min<int64_t>((n + 3) / 4, 8192);
  if (grid == 0) return;
  hipLaunchKernelGGL((i8_shadow_kernel<E4>), dim3(grid), dim3(256), 0, s, rows, n, r8, scale, err, stats);
}

void launch_i8_shadow(const float* rows, int64_t n, int dim, unsigned* r8, float* scale, float* err,
                      unsigned* stats, hipStream_t s) {
  switch (dim / 256) {
    case 1: i8_shadow_e4<1>(rows, n, r8, scale, err, stats, s); break;
    case 2: i8_shadow_e4<2>(rows, n, r8, scale, err, stats, s); break;
    case 3: i8_shadow_e4<3>(rows, n, r8, scale, err, stats, s); break;
    default: i8_shadow_e4<4>(rows, n, r8, scale, err, stats, s); break;
  }
}

int i8_lists(int num_cus) { return std::min(kI8WgPerCu * num_cus, kI8MaxLists); }

template <int E4, int NQ>
void launch_i8_nq(const ThreshI8Args& a, hipStream_t s, Timeline* tl) {
  const int G = i8_lists(a.num_cus);
  const int64_t n_units = (a.n + kI8Rows - 1) / kI8Rows;
  tl->mark(s, 0);
  hipLaunchKernelGGL((i8_thresh_kernel<E4, NQ, TS_MAX>), dim3(G), dim3(256), 0, s, a.q, a.nq, a.r8, a.scale,
                     a.n, n_units, kTsPeriod, a.tau, a.lmax, a.count, a.cs, a.ci, a.zero, a.stats, 0, a.mask);
  hipLaunchKernelGGL((i8_thresh_kernel<E4, NQ, TS_APPEND>), dim3(G), dim3(256), 0, s, a.q, a.nq, a.r8,
                     a.scale, a.n, n_units, 1, a.tau, a.lmax, a.count, a.cs, a.ci, nullptr, a.stats, a.k, a.mask);
}

// K9q segments -> compact (one block per query, thread t owns segment t)
__global__ __launch_bounds__(kI8MaxLists) void i8_compact_kernel(const float* __restrict__ cs,
                                                                const int* __restrict__ ci,
                                                                const int* __restrict__ count, int lists,
                                                                float* __restrict__ out_cs,
                                                                int* __restrict__ out_ci,
                                                                int* __restrict__ out_count) {
  __shared__ int off[kI8MaxLists];
  __shared__ int ovf;
  const int q = blockIdx.x, t = threadIdx.x;
  const int c = t < lists ? count[q * lists + t] : 0;
  if (t == 0) ovf = 0;
  off[t] = min(c, kI8Seg);
  __syncthreads();
  if (c > kI8Seg) ovf = 1;
  for (int d = 1; d < kI8MaxLists; d <<= 1) {  // inclusive scan (Hillis-Steele)
    const int v = t >= d ? off[t - d] : 0;
    __syncthreads();
    off[t] += v;
    __syncthreads();
  }
  const int end = off[t], beg = end - min(c, kI8Seg);
  for (int j = beg; j < end && j < kTsCap; ++j) {
    out_cs[(int64_t)q * kTsCap + j] = cs[((int64_t)q * lists + t) * kI8Seg + j - beg];
    out_ci[(int64_t)q * kTsCap + j] = ci[((int64_t)q * lists + t) * kI8Seg + j - beg];
  }
  if (t == kI8MaxLists - 1) out_count[q] = ovf ? kTsCap + 1 : end;
}

void launch_i8_compact(const float* cs, const int* ci, const int* count, int lists, int nq, float* out_cs,
                       int* out_ci, int* out_count, hipStream_t s) {
  hipLaunchKernelGGL(i8_compact_kernel, dim3(nq), dim3(kI8MaxLists), 0, s, cs, ci, count, lists, out_cs, out_ci,
                     out_count);
}

void launch_select(const float* cs, const int* ci, const int* count, const float* tau, int nq, int kc,
                   float* out_s, int64_t* out_i, hipStream_t s) {
  hipLaunchKernelGGL(bf16_select_kernel, dim3(nq), dim3(256), 0, s, cs, ci, count, tau, kc, out_s, out_i,
                     nullptr, nullptr);
}

// one query per launch (the single-query latency path; NQ > 1 costs registers: 256 VGPRs
// at NQ = 4, dim 768)
void launch_thresh_i8(const ThreshI8Args& a, hipStream_t s, Timeline* tl) {
  switch (a.dim / 256) {
    case 1: launch_i8_nq<1, 1>(a, s, tl); break;
    case 2: launch_i8_nq<2, 1>(a, s, tl); break;
    case 3: launch_i8_nq<3, 1>(a, s, tl); break;
    default: launch_i8_nq<4, 1>(a, s, tl); break;
  }
}

}  // namespace mq
