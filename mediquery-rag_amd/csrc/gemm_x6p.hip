// gemm_x6p.hip - K2p: the split-f32 (x6) encoder GEMM with its weights split once, at
// load time, into the fragment-blocked W3 image (gemm_x6p.hpp), replacing the x6 tiles of
// gemm_f32.hpp that re-split BOTH operands on every K-slice in every workgroup.
//
// out[M,N] = epi(A[M,K] . W[N,K]^T + bias (+ resid)), A fp32, W as W3 (3 bf16 planes).
//
//  * one 512-thread workgroup per CU (8 waves, two per SIMD), persistent over tiles;
//    block tile BM x BN = (WAVES_M 32 TM) x (WAVES_N 32 TN), wave tile TM x TN 32x32 MFMAs;
//  * K advances in 16-deep stages through an NBUF-slot LDS ring filled by LDS-DMA
//    (global_load_lds_dwordx4, no VGPR round trip, no staging VALU): NBUF - 1 stages in
//    flight while one is multiplied, a counted vmcnt and one s_barrier per stage;
//  * W3 stage: BN / 32 x 3 fragments of 1 KB, each one DMA wave-instruction, read back by
//    one ds_read_b128 per lane in lane order (conflict-free by construction);
//  * A stage: BM rows x 16 fp32 (64 B per row), 16 rows per DMA wave-instruction; the four
//    16-B chunks of row R sit at slot c ^ ((R >> 2) & 3) (the XOR goes on the DMA SOURCE
//    address: the DMA destination is lane-linear), which makes the A-fragment
//    ds_read_b128 (lane half h: chunks 2h, 2h + 1 of row r) conflict-free;
//  * A fragments are split into their three bf16 planes in registers right after the
//    read (split3: round-to-nearest per plane, residuals exact) - VALU that issues in the
//    MFMA shadow - and each 32x32 output tile takes the six products a2b0, a1b1, a0b2,
//    a1b0, a0b1, a0b0 per 16-deep step in the order of gemm_f32.hpp's x6 tiles: the same
//    operands in the same order, so the results are bit-identical to those tiles;
//  * tiles are walked in GM-row bands (GM row tiles x all column tiles, column-major
//    inside a band), each XCD taking consecutive tiles: at M = 8192 an XCD's 32 CUs share
//    4 A row panels and 8 W3 column panels in its L2.
#include <algorithm>

#include "gemm_epi.hpp"
#include "gemm_x6p.hpp"

namespace mq {
namespace {

typedef __attribute__((address_space(3))) void x6p_lds_t;

// One LDS-DMA wave-instruction: 16 B from base + voff (per lane) to LDS[lds_dst + 16 lane].
// Inline asm (as thresh.hip's ring): a compiler-visible LDS-DMA is tracked as a pending
// LDS write and every later ds_read of the array would wait vmcnt(0), draining the ring.
__device__ __forceinline__ void x6p_glds(const void* base, unsigned voff, unsigned lds_dst) {
  // the base is workgroup-uniform; say so (the uniformity analysis loses it through some
  // of the tile walks' index arithmetic, and the asm needs an SGPR pair)
  const uint64_t b64 = (uint64_t)(uintptr_t)base;
  base = (const void*)(uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(b64 >> 32)) << 32) |
                                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)b64));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

// Exact 3-way bf16 split of 4 floats (gemm_f32.hpp's split3, same arithmetic) with the
// packing conversion as a compiler-visible fptrunc (v_cvt_pk_bf16_f32, round to nearest
// even) instead of inline asm, so that sched_group_barrier counts it as VALU.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt_pk_bf16(float lo, float hi) {
  float2_t v;
  v.x = lo;
  v.y = hi;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ void split3v(floatx4 x, uint2 (&pl)[3]) {
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const unsigned a = cvt_pk_bf16(x.x, x.y), b = cvt_pk_bf16(x.z, x.w);
    pl[p] = make_uint2(a, b);
    if (p < 2) {  // residual is exact in fp32
      x.x -= bf16_lo(a);
      x.y -= bf16_hi(a);
      x.z -= bf16_lo(b);
      x.w -= bf16_hi(b);
    }
  }
}

// MQ_X6P_DBG (measurement builds only; wrong results): tile codes 8-15 of
// mq_debug_gemm_x6p run tiles 1 / 0 with parts of the stage removed - 1 no DMA, 2 no
// split, 8 no fragment reads, 16 no A DMA, 32 no W3 DMA, 64 prologue DMAs only, 128 no
// barrier, 256 no W3 fragment reads, 512 no A fragment reads - to price each part (the epilogue cannot be dropped: the
// MFMAs would be dead code).
#if defined(MQ_X6P_DBG) && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_X6P_DBG computes wrong results: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
#endif

template <int WAVES_M_, int WAVES_N_, int TM_, int TN_, int NBUF_, int KS_ = 1, int DMAW_ = 8, bool SCHED_ = false,
          int DBG_ = 0, int DSTEP_ = 1, int BR0_ = 0, int PS_ = 4, bool LDR_ = false>
struct X6pTile {
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, TM = TM_, TN = TN_, NBUF = NBUF_;
  static constexpr int KS = KS_;    // 16-deep k-steps per LDS stage (one barrier per stage)
  // DMAW: waves that issue the stage's DMAs (8: all; 4: waves 0-3, so that on every SIMD
  // one of its two waves never stops its MFMA stream to issue DMAs).  SCHED: the k-step
  // is laid out slot by slot (one MFMA per slot, sched_barrier between slots) with the
  // next k-step's fragment reads, this wave's DMAs and the next A fragment's split spread
  // over the slots, so that the split VALU issues in the MFMA shadow (left alone the
  // compiler sinks the split to the next k-step, in front of its MFMAs).
  static constexpr int DMAW = DMAW_;
  static constexpr bool SCHED = SCHED_;
  // SCHED slot plan: DMA t of the stage behind the MFMA of slot t * DSTEP (k-step 0), the
  // next B fragment reads two per slot from slot BR0 (skipping DMA slots), the split
  // pieces from slot PS on
  static constexpr int DSTEP = DSTEP_, BR0 = BR0_, PS = PS_;
  static constexpr int DBG = DBG_;  // measurement builds only (MQ_X6P_DBG)
  // LDR: WAVES_M x WAVES_N = 4 compute waves (one per SIMD) plus 4 loader waves that only
  // issue the stage DMAs (an LDS-DMA holds the issuing wave for ~60-185 cycles; a loader
  // wave pays that beside its SIMD's compute wave, whose MFMA stream it never interrupts)
  static constexpr bool LDR = LDR_;
  static constexpr int NW = WAVES_M * WAVES_N, THREADS = (LDR ? 2 * NW : NW) * 64;
  static constexpr int WM = TM * 32, WN = TN * 32, BM = WAVES_M * WM, BN = WAVES_N * WN;
  static constexpr int A_SUB = BM * 64;  // one k-step of A: 16 fp32 per row
  static constexpr int B_SUB = BN * 96;  // one k-step of W3: 16 k x 3 planes x 2 B per row
  static constexpr int STAGE = KS * (A_SUB + B_SUB);
  static constexpr int NA = BM / 16, NB = BN / 32 * 3;  // DMA wave-instructions per k-step
  static constexpr int NI = KS * (NA + NB);                    // ... per stage
  static constexpr int CNT_LO = NI / DMAW, REM = NI % DMAW, CNT_HI = CNT_LO + (REM ? 1 : 0);
  static_assert(DMAW == 8 || DMAW == 4, "DMA waves");
  static_assert(!LDR || DMAW == 4, "loader mode: the 4 loader waves issue every DMA");
  // stage issue distance: a stage's slot is free once its last k-step's fragments are in
  // registers - at KS = 1 that happens one iteration early (the fragments run one k-step
  // ahead), so the ring can run one stage further ahead
  static constexpr int AHEAD = KS == 1 ? NBUF : NBUF - 1;
#ifndef MQ_X6P_GM  // tuning default: 8 row tiles per band (half the W3 column blocks per XCD
#define MQ_X6P_GM 4  // round) measured the same at every headline shape (tools/gpu_ab_x6p.sh)
#endif
  static constexpr int GM = MQ_X6P_GM;  // row tiles per band of the tile walk
  static_assert(LDR ? NW == 4 : NW == 8, "8-wave workgroups");
  static_assert(!SCHED || (CNT_HI - 1) * DSTEP < TM * TN * 6, "DMAs per k-step slots");
  static_assert(AHEAD >= 2 && NBUF * STAGE <= 160 * 1024, "LDS ring");
};

template <class T, int EPI>
__global__ __launch_bounds__(T::THREADS, 1) void gemm_x6p_kernel(const float* __restrict__ A, int lda,
                                                             const unsigned char* __restrict__ W3,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ resid, int ldr,
                                                             float* __restrict__ out, int ldo, int M, int N,
                                                             int K, int rx) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[T::NBUF * T::STAGE];
  const unsigned lds0 = (unsigned)(uintptr_t)(x6p_lds_t*)lds;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cw = T::LDR ? wave % T::NW : wave;  // compute wave index
  const int wm = cw / T::WAVES_N, wn = cw % T::WAVES_N;
  const int tiles_m = (M + T::BM - 1) / T::BM, tiles_n = (N + T::BN - 1) / T::BN;
  const int total = tiles_m * tiles_n;
  const int G = gridDim.x, per_xcd = G >> 3;
  const int xslot = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  // rx > 0: the tile grid is cut into 8 regions, rx column blocks x 8 / rx row blocks, and
  // the workgroups that share blockIdx.x % 8 (an XCD under round-robin dispatch; a speed
  // assumption, never a correctness one) walk one region - its W3 column panels stay in
  // that XCD's L2 for the whole launch instead of being re-read every round
  int m_lo = 0, rm = tiles_m, n_lo = 0, rn = tiles_n, loc = xslot, wstep = G, rtiles = total;
  if (rx > 0) {
    const Region rg = region_of(rx, blockIdx.x & 7, tiles_m, tiles_n);
    m_lo = rg.m_lo;
    rm = rg.rm;
    n_lo = rg.n_lo;
    rn = rg.rn;
    loc = blockIdx.x >> 3;
    wstep = per_xcd;
    rtiles = rm * rn;
  }
  const int n_tiles = loc < rtiles ? (rtiles - loc + wstep - 1) / wstep : 0;
  if (n_tiles == 0) return;
  const int nk = K >> 4;                 // 16-deep k-steps per tile
  const int nst = nk / T::KS;            // stages per tile (the launcher checks K % (16 KS) == 0)
  const int S = n_tiles * nst;           // stages of this workgroup
  const int nbw = (N + 31) >> 5;
  const int band_tiles = T::GM * rn;
  auto coords = [&](int i, int& m0, int& n0) {  // bands of GM row tiles, column-major inside
    const int t = i * wstep + loc;
    const int band = t / band_tiles;
    const int gm = min(T::GM, rm - band * T::GM);
    const int w = t - band * band_tiles;
    const int tc = w / gm;
    m0 = (m_lo + band * T::GM + (w - tc * gm)) * T::BM;
    n0 = (n_lo + tc) * T::BN;
  };

  // ---- DMA issue of stage `is_j` into a ring slot (past the last stage: the last again,
  // never multiplied).  Instruction `ins` of a stage: k-step ins / (NA + NB), then A rows
  // 16 ins' .. + 15 (ins' < NA) or W3 fragment ins' - NA = 3 (column block) + plane.
  int is_j = 0, is_i = 0, is_kt = 0, is_m0, is_n0;
  coords(0, is_m0, is_n0);
  // A chunk this lane moves: row 16 ins + (lane >> 2), slot lane & 3 -> chunk slot ^ ((row >> 2) & 3)
  const unsigned a_chunk = (unsigned)(((lane & 3) ^ ((lane >> 4) & 3)) * 16);
  // DMA t (< CNT_HI) of this wave for the stage at is_j into slot `buf`
  auto issue_one = [&](int buf, int t) __attribute__((always_inline)) {
    if constexpr (T::DBG & 1) return;
    if constexpr (T::DBG & 64) {  // prologue DMAs only: the loop multiplies stale stages
      if (is_j >= T::AHEAD) return;
    }
    const int dw = T::LDR ? wave - T::NW : wave;  // DMA wave index
    if (dw < 0 || dw >= T::DMAW || (T::REM && t == T::CNT_HI - 1 && dw >= T::REM)) return;
    const unsigned dst = lds0 + (unsigned)(buf * T::STAGE);
    const int ins = dw + t * T::DMAW;
    const int ks = ins / (T::NA + T::NB), in = ins - ks * (T::NA + T::NB);
    const int kt = is_kt + ks;
    if (in < T::NA) {
      if constexpr (T::DBG & 16) return;
      const float* abase = A + (int64_t)is_m0 * lda + kt * 16;
      const unsigned voff = (unsigned)min(16 * in + (lane >> 2), M - 1 - is_m0) * (unsigned)lda * 4u + a_chunk;
      x6p_glds(abase, voff, dst + ks * T::A_SUB + in * 1024);
    } else {
      if constexpr (T::DBG & 32) return;
      const int b = in - T::NA, nbl = b / 3, p = b - nbl * 3;
      const int nbg = min((is_n0 >> 5) + nbl, nbw - 1);
      const unsigned char* wbase = W3 + ((size_t)(nbg * nk + kt) * 3 + p) * 1024;
      x6p_glds(wbase, (unsigned)lane * 16u, dst + T::KS * T::A_SUB + ks * T::B_SUB + b * 1024);
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (is_j + 1 < S) {
      ++is_j;
      is_kt += T::KS;
      if (is_kt == nk) {
        is_kt = 0;
        ++is_i;
        coords(is_i, is_m0, is_n0);
      }
    }
  };
  auto issue = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < T::CNT_HI; ++t) issue_one(buf, t);
    advance();
  };

  // ---- fragments of one k-step (A split into its planes after the read) and its MFMAs:
  // the six products per 32x32 tile
  const int r = lane & 31, h = lane >> 5, sw = (r >> 2) & 3;
  const unsigned a_lo = (unsigned)((((2 * h) ^ sw) * 16)), a_hi = (unsigned)((((2 * h + 1) ^ sw) * 16));
  struct Frags {
    floatx4 raw[T::TM][2];  // A fragment as read (fp32 k = 8h .. 8h + 7)
    bf16x8 a[T::TM][3], b[T::TN][3];
  };
  // fragments of k-step `ks` of the stage in slot `buf`
  auto read_frags = [&](int buf, int ks, Frags& f) __attribute__((always_inline)) {
    if constexpr (T::DBG & 8) return;
    const unsigned char* st = lds + buf * T::STAGE;
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm) {
      const unsigned char* ar = st + ks * T::A_SUB + (wm * T::WM + tm * 32 + r) * 64;
      f.raw[tm][0] = *reinterpret_cast<const floatx4*>(ar + a_lo);
      f.raw[tm][1] = *reinterpret_cast<const floatx4*>(ar + a_hi);
    }
    const unsigned char* bs = st + T::KS * T::A_SUB + ks * T::B_SUB + lane * 16;
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        f.b[tn][p] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(bs + ((wn * T::TN + tn) * 3 + p) * 1024));
  };
  auto split_frags = [&](Frags& f) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm) {
      if constexpr (T::DBG & 2) {
        f.a[tm][0] = __builtin_bit_cast(bf16x8, f.raw[tm][0]);
        f.a[tm][1] = __builtin_bit_cast(bf16x8, f.raw[tm][1]);
        f.a[tm][2] = f.a[tm][0];
        continue;
      }
      uint2 pl[3], ph[3];
      split3v(f.raw[tm][0], pl);
      split3v(f.raw[tm][1], ph);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        uintx4 v;
        v.x = pl[p].x;
        v.y = pl[p].y;
        v.z = ph[p].x;
        v.w = ph[p].y;
        f.a[tm][p] = __builtin_bit_cast(bf16x8, v);
      }
    }
  };
  floatx16 acc[T::TM][T::TN];
  // MFMAs of one k-step; hook(g) after the six products of 32x32 tile g (SPREAD)
  auto mma = [&](const Frags& f, auto&& hook) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn) {
        // smallest terms first (gemm_f32.hpp's x6 order)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][2], f.b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][1], f.b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][0], f.b[tn][2], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][1], f.b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][0], f.b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][0], f.b[tn][0], acc[tm][tn], 0, 0, 0);
        hook(tm * T::TN + tn);
      }
  };
  // ---- explicit slot schedule of one k-step (SCHED): MFMA i of the k-step in slot i;
  // before slot 0 the next k-step's A reads; behind the MFMA of slot i: two of the next
  // B fragment reads (first slots), DMA i of the stage (k-step 0), and from slot PS on
  // the split of the next A fragment in pieces of <= 5 VALU (plane p of an x,y or z,w
  // pair: one v_cvt_pk_bf16_f32, then the two exact residual subtractions)
  auto mma_one = [&](const Frags& f, int i) __attribute__((always_inline)) {
    const int g = i / 6, tm = g / T::TN, tn = g % T::TN, term = i % 6;
    // smallest terms first (gemm_f32.hpp's x6 order): a2b0 a1b1 a0b2 a1b0 a0b1 a0b0
    const int pa = term == 0 ? 2 : term == 1 || term == 3 ? 1 : 0;
    const int pb = term == 0 || term >= 3 ? (term == 4 ? 1 : 0) : term == 1 ? 1 : 2;
    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[tm][pa], f.b[tn][pb], acc[tm][tn], 0, 0, 0);
  };
  auto read_a = [&](int buf, int ks, Frags& f) __attribute__((always_inline)) {
    if constexpr ((T::DBG & 8) || (T::DBG & 512)) {  // no A reads: opaque stale values
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm) asm volatile("" : "+v"(f.raw[tm][0]), "+v"(f.raw[tm][1]));
      return;
    }
    const unsigned char* st = lds + buf * T::STAGE;
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm) {
      const unsigned char* ar = st + ks * T::A_SUB + (wm * T::WM + tm * 32 + r) * 64;
      f.raw[tm][0] = *reinterpret_cast<const floatx4*>(ar + a_lo);
      f.raw[tm][1] = *reinterpret_cast<const floatx4*>(ar + a_hi);
    }
  };
  auto read_b = [&](int buf, int ks, Frags& f, int q) __attribute__((always_inline)) {  // fragment q = 3 tn + p
    if constexpr ((T::DBG & 8) || (T::DBG & 256)) {  // no B reads: opaque stale values
      asm volatile("" : "+v"(f.b[q / 3][q % 3]));
      return;
    }
    const unsigned char* bs = lds + buf * T::STAGE + T::KS * T::A_SUB + ks * T::B_SUB + lane * 16;
    f.b[q / 3][q % 3] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(bs + ((wn * T::TN) * 3 + q) * 1024));
  };
  unsigned pk[T::TM][2][3][2];
  auto piece = [&](Frags& f, int q) __attribute__((always_inline)) {  // q < 12 TM
    const int tm = q / 12, half = (q / 6) % 2, p = (q % 6) / 2, part = q % 2;
    floatx4& x = f.raw[tm][half];
    unsigned u;
    if (part == 0) {
      u = cvt_pk_bf16(x.x, x.y);
      if (p < 2) {
        x.x -= bf16_lo(u);
        x.y -= bf16_hi(u);
      }
    } else {
      u = cvt_pk_bf16(x.z, x.w);
      if (p < 2) {
        x.z -= bf16_lo(u);
        x.w -= bf16_hi(u);
      }
    }
    // keep the piece in its slot (machine sinking would move it past the DMA branches,
    // towards the use in the next k-step)
    asm volatile("" : "+v"(u), "+v"(x));
    pk[tm][half][p][part] = u;
  };
  auto assemble = [&](Frags& f) __attribute__((always_inline)) {
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        uintx4 v;
        v.x = pk[tm][0][p][0];
        v.y = pk[tm][0][p][1];
        v.z = pk[tm][1][p][0];
        v.w = pk[tm][1][p][1];
        f.a[tm][p] = __builtin_bit_cast(bf16x8, v);
        asm volatile("" : "+v"(f.a[tm][p]));  // the split stays in this k-step
      }
  };
  int c_i = 0, c_st = 0;
  auto tile_end = [&]() __attribute__((always_inline)) {
    if (++c_st == nst) {
      c_st = 0;
      int m0, n0;
      coords(c_i, m0, n0);
      if constexpr (!(T::DBG & 4))
        store_wave_tile<EPI, T::TM, T::TN>(acc, m0 + wm * T::WM, n0 + wn * T::WN, M, N, bias, resid, ldr, out, ldo,
                                           lane);
      zero_acc<T>(acc);
      ++c_i;
    }
  };
  // own DMAs landed up to all but the last `stages` stages issued, then everyone's (and
  // every wave is past its reads of the slot the next issue refills)
  auto wait_stages = [&](auto stages) __attribute__((always_inline)) {
    constexpr int n = decltype(stages)::value;
    const int dwi = T::LDR ? wave - T::NW : wave;
    if constexpr (T::DBG & 128) {  // no barrier (races: timing only)
      if (T::REM && dwi >= 0 && dwi < T::REM)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(T::CNT_HI * n) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(T::CNT_LO * n) : "memory");
      return;
    }
    if (T::REM && dwi >= 0 && dwi < T::REM)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::CNT_HI * n) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::CNT_LO * n) : "memory");
    // lgkmcnt(0) as the builtin, visible to the compiler's wait-count pass: it then knows
    // the fragment reads of the previous k-step have landed (as inline asm it does not,
    // and waits lgkmcnt(0) in front of the first MFMA - for this k-step's own reads too)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
  };
  zero_acc<T>(acc);

  // Stage j's k-steps multiply from registers while the next k-step's fragments (k-step
  // 0 of stage j + 1 after the last) are read and split; stage j + 1 has landed before
  // stage j starts, and stage j + AHEAD is issued into the slot freed last.
  if constexpr (T::LDR) {
    if (wave >= T::NW) {  // loader waves: the ring, one barrier per stage as the compute waves
#pragma unroll
      for (int d = 0; d < T::AHEAD; ++d) issue(d);
      wait_stages(IC<T::AHEAD - 1>{});  // stage 0 landed
      for (int j = 0; j < S; ++j) {
        wait_stages(IC<T::AHEAD - 2>{});  // stage j + 1 landed
        issue((j + T::AHEAD) % T::NBUF);  // stage j + AHEAD
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-read DMAs
      return;
    }
  } else {
#pragma unroll
    for (int d = 0; d < T::AHEAD; ++d) issue(d);
  }
  wait_stages(IC<T::AHEAD - 1>{});  // stage 0 landed
  Frags f0 = {}, f1 = {};
  read_frags(0, 0, f0);
  split_frags(f0);
  // iteration j with `fa` holding its first k-step's fragments
  auto step = [&](int j, Frags& fa, Frags& fb) __attribute__((always_inline)) {
    wait_stages(IC<T::AHEAD - 2>{});  // stage j + 1 landed
    const int buf = (j + T::AHEAD) % T::NBUF;  // stage j + AHEAD goes here
    if constexpr (!T::SCHED && !T::LDR) issue(buf);
    static_for<T::KS>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      Frags& cur = ks % 2 == 0 ? fa : fb;
      Frags& nxt = ks % 2 == 0 ? fb : fa;
      if constexpr (T::SCHED) {
        constexpr int NM = T::TM * T::TN * 6, NBR = 3 * T::TN, PS = T::PS, NP = 12 * T::TM;
        constexpr int PER = (NP + (NM - PS) - 1) / (NM - PS);
        const int rbuf = ks + 1 < T::KS ? j % T::NBUF : (j + 1) % T::NBUF;
        constexpr int rks = ks + 1 < T::KS ? ks + 1 : 0;
        read_a(rbuf, rks, nxt);
        __builtin_amdgcn_sched_barrier(0);
        static_for<NM>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          mma_one(cur, i);
          constexpr bool dma_slot = !T::LDR && ks == 0 && i % T::DSTEP == 0 && i / T::DSTEP < T::CNT_HI;
          // B read pair index of slot i: slots from BR0 on that carry no DMA
          constexpr int bslot = [] {
            int n = 0;
            for (int k = T::BR0; k < i; ++k)
              if (!(!T::LDR && ks == 0 && k % T::DSTEP == 0 && k / T::DSTEP < T::CNT_HI) || T::DSTEP == 1) ++n;
            return n;
          }();
          if constexpr (i >= T::BR0 && (!dma_slot || T::DSTEP == 1)) {
            if constexpr (2 * bslot < NBR) read_b(rbuf, rks, nxt, 2 * bslot);
            if constexpr (2 * bslot + 1 < NBR) read_b(rbuf, rks, nxt, 2 * bslot + 1);
          }
          if constexpr (dma_slot) issue_one(buf, i / T::DSTEP);
          if constexpr (i >= PS) {
            static_for<PER>([&](auto pc) {
              constexpr int q = (i - PS) * PER + decltype(pc)::value;
              if constexpr (q < NP) piece(nxt, q);
            });
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        assemble(nxt);
      } else {
        if constexpr (ks + 1 < T::KS)
          read_frags(j % T::NBUF, ks + 1, nxt);
        else
          read_frags((j + 1) % T::NBUF, 0, nxt);
        mma(cur, [](int) {});
        split_frags(nxt);
      }
    });
    if constexpr (T::SCHED && !T::LDR) advance();
    tile_end();
  };
  if constexpr (T::KS % 2 == 0) {
    for (int j = 0; j < S; ++j) step(j, f0, f1);
  } else {
    for (int j = 0; j < S; j += 2) {
      step(j, f0, f1);
      if (j + 1 >= S) break;
      step(j + 1, f1, f0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-read DMAs
}

// W [N][K] fp32 -> W3: one thread per (row n < Np, 8-wide k chunk); rows past N are zero.
__global__ __launch_bounds__(256) void split_w3_kernel(const float* __restrict__ W, int N, int K,
                                                       uintx4* __restrict__ w3) {
  const int k8n = K >> 3, np = (N + 31) & ~31;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)np * k8n) return;
  const int n = (int)(idx / k8n), k8 = (int)(idx - (int64_t)n * k8n);
  floatx4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
  if (n < N) {
    lo = *reinterpret_cast<const floatx4*>(W + (int64_t)n * K + 8 * k8);
    hi = *reinterpret_cast<const floatx4*>(W + (int64_t)n * K + 8 * k8 + 4);
  }
  uint2 pl[3], ph[3];
  split3(lo, pl);
  split3(hi, ph);
  const int kb = k8 >> 1, hh = k8 & 1, nb = n >> 5, rr = n & 31;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    uintx4 v;
    v.x = pl[p].x;
    v.y = pl[p].y;
    v.z = ph[p].x;
    v.w = ph[p].y;
    w3[((int64_t)(nb * (K >> 4) + kb) * 3 + p) * 64 + hh * 32 + rr] = v;
  }
}

// Product tiles (mq_debug_gemm_x6p tile codes 0-3).  Measured at M = 8192 (BERT-base
// batched shapes, tools/gemm_x6p_bench.py): the loader-wave 128 x 192 tile runs at 0.42-0.50
// of the 417 TF fp32-equivalent peak, the 8-wave slot-scheduled ones at 0.44-0.50, the
// first cut (8 waves, DMAs in a burst after the barrier, scheduler's own order) 0.34-0.45.
using X6p0 = X6pTile<2, 2, 2, 3, 4, 1, 4, true, 0, 1, 0, 6, true>;  // 128 x 192, 4 compute + 4 loader waves
using X6p1 = X6pTile<4, 1, 2, 3, 4, 1, 4, true, 0, 1, 0, 6, true>;  // 256 x 96, same
using X6p2 = X6pTile<4, 2, 1, 3, 4, 1, 4, true, 0, 2, 1, 6>;        // 128 x 192, 8 waves, DMAs from 0-3
using X6p3 = X6pTile<4, 2, 2, 3, 4, 1, 8, true, 0, 6, 1, 8>;        // 256 x 192, 8 waves
// measurement variants (tile codes 4-6; 7 is a product tile)
using X6p4 = X6pTile<2, 2, 2, 3, 3, 2, 4, true, 0, 1, 0, 6, true>;  // tile 0 with 32-deep stages, 3 slots
using X6p5 = X6pTile<2, 2, 2, 3, 4, 1, 4, true, 0, 1, 0, 4, true>;  // tile 0, split from slot 4
using X6p6 = X6pTile<2, 2, 2, 3, 5, 1, 4, true, 0, 1, 0, 6, true>;  // tile 0 with 5 slots
using X6p7 = X6pTile<2, 2, 1, 3, 4, 1, 4, true, 0, 1, 0, 6, true>;  // 64 x 192, loaders (product: out-proj)

template <class T, int EPI>
void launch_t(const X6pArgs& g, int num_cus, hipStream_t s) {
  if (g.K % (16 * T::KS) != 0) {  // stage depth must divide K: the 16-deep default tile
    launch_t<X6pTile<4, 2, 1, 3, 4>, EPI>(g, num_cus, s);
    return;
  }
  const int tiles = ((g.M + T::BM - 1) / T::BM) * ((g.N + T::BN - 1) / T::BN);
  const int grid = (std::min(tiles, num_cus) + 7) / 8 * 8;  // one workgroup per CU, a multiple of 8
  const int tiles_m = (g.M + T::BM - 1) / T::BM, tiles_n = (g.N + T::BN - 1) / T::BN;
  int rx = g.rx;
  if (rx < 0) rx = region_pick_rx(tiles_m, tiles_n, (double)T::BM * g.K * 4, (double)T::BN * g.K * 6, grid);
  if (rx > 0 && (8 % rx != 0 || rx > tiles_n || 8 / rx > tiles_m || grid < 8)) rx = 0;  // (a region per XCD)
  hipLaunchKernelGGL((gemm_x6p_kernel<T, EPI>), dim3(grid), dim3(T::THREADS), 0, s, g.A, g.lda,
                     static_cast<const unsigned char*>(g.W3), g.bias, g.resid, g.ldr, g.out, g.ldo, g.M, g.N, g.K, rx);
}

template <int EPI>
void launch_tile(const X6pArgs& g, int tile, int num_cus, hipStream_t s) {
#ifdef MQ_X6P_DBG
  if (tile >= 8) {  // measurement builds: tiles 1 / 0 minus parts (X6pTile DBG bits)
    switch (tile) {
      case 8: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 64, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 9: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 66, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 10: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 8, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 11: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 74, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 12: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 2, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 13: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 256, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      case 14: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 512, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
      default: launch_t<X6pTile<2, 2, 2, 3, 4, 1, 4, true, 128, 1, 0, 6, true>, EPI>(g, num_cus, s); return;
    }
  }
#endif
  switch (tile) {
    case 1: launch_t<X6p1, EPI>(g, num_cus, s); return;
    case 2: launch_t<X6p2, EPI>(g, num_cus, s); return;
    case 3: launch_t<X6p3, EPI>(g, num_cus, s); return;
    case 4: launch_t<X6p4, EPI>(g, num_cus, s); return;
    case 5: launch_t<X6p5, EPI>(g, num_cus, s); return;
    case 6: launch_t<X6p6, EPI>(g, num_cus, s); return;
    case 7: launch_t<X6p7, EPI>(g, num_cus, s); return;
    default: launch_t<X6p0, EPI>(g, num_cus, s); return;
  }
}

}  // namespace

void launch_split_w3(const float* W, int N, int K, void* w3, hipStream_t s) {
  const int64_t n = (int64_t)((N + 31) & ~31) * (K >> 3);
  hipLaunchKernelGGL(split_w3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, N, K,
                     static_cast<uintx4*>(w3));
}

int x6p_pick_tile(int M, int N, int num_cus) {
  // tiles 0 (128 x 192) and 1 (256 x 96) cover the same area at the same measured rate:
  // fewer rounds wins, 128 x 192 on a tie (M = 8192 at N = 768 / 1536 / 2304 / 3072 runs
  // whole rounds of 256 tiles on it)
  auto rounds = [&](int bm, int bn) {
    const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    return (tiles + num_cus - 1) / num_cus;
  };
  return rounds(256, 96) < rounds(128, 192) ? 1 : 0;
}

void launch_gemm_x6p(const X6pArgs& g, int epi, int tile, int num_cus, hipStream_t s) {
  if (tile < 0) {
    tile = x6p_pick_tile(g.M, g.N, num_cus);
    // a short, narrow GEMM (out-proj: N = K = 768) that 128 x 192 covers in one round of
    // one tile per CU runs 64 x 192 tiles, two per CU: the ring carries into the second
    // tile, the first's epilogue overlaps its loads (57.2 vs 59.3 us at M = 8192; slower
    // on the deeper and wider shapes, tools/gemm_x6p_bench.py)
    const int64_t t0 = (int64_t)((g.M + 127) / 128) * ((g.N + 191) / 192);
    if (g.K <= 768 && g.N <= 768 && t0 <= num_cus && t0 * 2 > num_cus) tile = 7;
  }
  switch (epi) {
    case EPI_GELU_ERF: launch_tile<EPI_GELU_ERF>(g, tile, num_cus, s); return;
    case EPI_GELU_TANH: launch_tile<EPI_GELU_TANH>(g, tile, num_cus, s); return;
    case EPI_RESID: launch_tile<EPI_RESID>(g, tile, num_cus, s); return;
    default: launch_tile<EPI_BIAS>(g, tile, num_cus, s); return;
  }
}

}  // namespace mq

extern "C" {

// Test / measurement hooks (include/mq.h).
int64_t mq_debug_w3_bytes(int N, int K) { return N > 0 && K > 0 && K % 16 == 0 ? (int64_t)mq::w3_bytes(N, K) : -1; }

int mq_debug_split_w3(const float* W, int N, int K, void* w3, void* stream) {
  using namespace mq;
  clear_error();
  MQ_CHECK_ARG(W && w3, "NULL buffer");
  MQ_CHECK_ARG(N > 0 && K > 0 && K % 16 == 0, "bad shape N=%d K=%d", N, K);
  launch_split_w3(W, N, K, w3, (hipStream_t)stream);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_debug_gemm_x6p(const float* A, const void* W3, const float* bias, const float* resid, float* out, int M,
                      int N, int K, int epi, int tile, void* stream) {
  using namespace mq;
  clear_error();
  MQ_CHECK_ARG(A && W3 && bias && out && (epi != EPI_RESID || resid), "NULL buffer");
  MQ_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 32 == 0, "bad shape M=%d N=%d K=%d", M, N, K);
  // tile codes >= 100: tile code % 100 with the region split rx = code / 100 - 1 (0 = the
  // plain walk); below 100 the automatic pick
  const int rx = tile >= 100 ? tile / 100 - 1 : -1;
  if (tile >= 100) tile %= 100;
  MQ_CHECK_ARG(epi >= 0 && epi <= 3 && tile >= -1 && tile <= 15 && rx <= 8, "bad epi/tile");
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  X6pArgs g{A, K, W3, bias, resid, N, out, N, M, N, K};
  g.rx = rx;
  launch_gemm_x6p(g, epi, tile, cus, (hipStream_t)stream);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

}  // extern "C"
