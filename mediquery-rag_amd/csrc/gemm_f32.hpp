// gemm_f32.hpp - fp32 MFMA tile core for gfx950.
//
// Computes D[i][j] = sum_k A[i][k] * B[j][k] for a BM x BN block tile, both operands
// K-contiguous ("NT": activations/queries [M][K], weights/corpus rows [N][K]), fp32 in
// HBM.  Two arithmetic variants share the tile walk:
//
//  * exact f32 (X6 = false): v_mfma_f32_32x32x2_f32, a k-ordered fmaf chain (gfx950 has
//    no xf32).  K is staged in 32-wide slices through a double-buffered LDS image
//    [rows][36] floats (144-B rows: conflict-free ds_write_b128 / ds_read_b128,
//    slot = 9*row + 4*h + q mod 16).  MFMA step (q, s), lane half h carries
//    k = 16h + 4q + s for BOTH operands, so a lane reads 16 contiguous floats per slice.
//  * split f32 (X6 = true): every fp32 operand is split EXACTLY into three bf16 pieces
//    x = x0 + x1 + x2 (8 + 8 + 8 significant bits, round-to-nearest at each step) while
//    it is staged, and each product uses the six bf16 MFMAs (v_mfma_f32_32x32x16_bf16)
//    x0y0, x0y1, x1y0, x0y2, x1y1, x2y0 with fp32 accumulation: every bf16 x bf16
//    product is exact in fp32 and the dropped terms x1y2 + x2y1 + x2y2 are < 3 * 2^-24
//    relative, i.e. fp32-class results at 16/6 = 2.67x the f32 MFMA rate.  K is staged
//    in 16-wide slices; an LDS row holds the three planes [3][16] bf16 + 16 B pad
//    (112-B rows: slot = 7*row + 2*plane + h mod 16, conflict-free); lane half h carries
//    k = 8h + j.
//
//  * 256 or 512 threads = 4 or 8 waves laid out WAVES_M x WAVES_N; each wave owns
//    TM x TN MFMA tiles of 32x32 (f32x16 accumulators, 16 regs/lane each).
//  * Global loads run two slices ahead in two named register stages (walk_tiles).
#pragma once

#include "common.hpp"

namespace mq {

constexpr int kBK = 32;              // K granularity every caller must respect
constexpr int kLdsStride = kBK + 4;  // floats per staged row of the exact-f32 image (144 B)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

template <int WAVES_M_, int WAVES_N_, int TM_, int TN_, bool X6_ = false, int PF_ = 2,
          bool BF16_ = false, int BK_ = 0, bool NTB_ = false>
struct F32Tile {
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, TM = TM_, TN = TN_;
  static constexpr bool X6 = X6_;
  // NTB: B-operand loads are non-temporal (the single-query split-K GEMMs of the layers past
  // the encoder's resident_layers: their weights stream once and should not evict the
  // resident layers' weights from MALL)
  static constexpr bool NTB = NTB_;
  static constexpr int PF = PF_;  // register prefetch depth in slices (walk_tiles D)
  // BF16: both operands are bf16 in memory, addressed as float-typed rows of half the
  // width (two bf16 per 4-byte slot): the staging is byte-identical to the f32 path and
  // a 32-slot slice carries 64 k-values; only the MFMA (32x32x16 bf16) differs.
  static constexpr bool BF16 = BF16_;
  static_assert(!(X6 && BF16), "one arithmetic mode");
  static constexpr int WM = TM * 32, WN = TN * 32;  // wave tile
  static constexpr int BM = WAVES_M * WM, BN = WAVES_N * WN;
  static constexpr int THREADS = WAVES_M * WAVES_N * kWave;
  static constexpr int ROWS = BM + BN;
  // K per staged slice: 32 (exact f32 / bf16 default), 16 (split f32; or an exact-f32 tile
  // whose B panel is too tall for two 32-deep stages, e.g. the full-row 32 x 768 tile)
  static constexpr int BK = BK_ ? BK_ : (X6 ? 16 : 32);
  static_assert(BK == 32 || (BK == 16 && !BF16), "slice depth 32, or 16 for the f32 forms");
  static constexpr int F4_PER_ROW = BK / 4;               // float4 per row per slice
  // LDS row stride in 4-B words: 144-B rows at BK 32, 80-B rows at BK 16 (16 rows of one
  // ds_read_b128 group still land in distinct 16-B bank groups), 112-B split-plane rows
  static constexpr int ROW_FLOATS = X6 ? 28 : BK + 4;
  static constexpr int TOTAL_F4 = ROWS * F4_PER_ROW;                  // float4 per slice
  static constexpr int LOADS = (TOTAL_F4 + THREADS - 1) / THREADS;      // per thread
  static constexpr bool PARTIAL = TOTAL_F4 % THREADS != 0;              // last slot ragged
  static constexpr int STAGE_FLOATS = ROWS * ROW_FLOATS;
  static_assert(THREADS == 256 || THREADS == 512, "4- or 8-wave workgroups");
  // workgroups per CU the kernel is built for: 2 x 4 waves, or 1 x 8 waves (LDS)
  static constexpr int WG_PER_CU = THREADS == 256 ? 2 : 1;
  static_assert(BM % 32 == 0 && BN % 32 == 0, "block tile must be a multiple of 32");
  // A rows fill whole load slots (compile-time A / B split) unless the A panel is smaller
  // than one slot (the full-row 32 x H tile: 128 A float4 for 512 threads), then per thread
  static constexpr bool A_SLOTS = (BM * F4_PER_ROW) % THREADS == 0;
};

// Exact 3-way bf16 split of 4 floats: returns plane p as 4 packed bf16 (2 dwords).
__device__ __forceinline__ unsigned pk_bf16(float lo, float hi) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ float bf16_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf16_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

__device__ __forceinline__ void split3(floatx4 x, uint2 (&pl)[3]) {
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const unsigned a = pk_bf16(x.x, x.y), b = pk_bf16(x.z, x.w);
    pl[p] = make_uint2(a, b);
    if (p < 2) {  // residual is exact in fp32
      x.x -= bf16_lo(a);
      x.y -= bf16_hi(a);
      x.z -= bf16_lo(b);
      x.w -= bf16_hi(b);
    }
  }
}

// compile-time loop: f(IC<0>{}) .. f(IC<N-1>{})
template <int V>
struct IC {
  static constexpr int value = V;
};

template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}

// One K-slice of both operands, held in registers between the global load and the
// LDS write (T14 "issue early / write late").  Rows past M / N are clamped onto the
// last valid row instead of being zeroed: an MFMA output element depends only on its
// own A row and B row, so the garbage lands only in output rows / columns the
// epilogue never stores.  The per-slice path is LOADS x global_load_dwordx4.
template <class T>
struct Stager {
  floatx4 r[T::LOADS];

  __device__ __forceinline__ void load(const float* __restrict__ A, int64_t lda, int M, int m0,
                                       const float* __restrict__ B, int64_t ldb, int64_t N,
                                       int64_t n0, int k0, int tid) {
    if constexpr (T::A_SLOTS) {
      // Buffer loads off two per-tile resources (scalar: the panel origins A + m0 lda and
      // B + n0 ldb, so a corpus slab past 4 GB still takes 32-bit offsets), the slice's
      // k0 in soffset, and a 32-bit per-slot offset (row clamped, 16-B chunk): 2 VALU per
      // load instead of the 64-bit address arithmetic of a flat load (~60 VALU per slice).
      const __amdgpu_buffer_rsrc_t ra =
          __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)m0 * lda), (short)0, 0x7fffffff, 0x00020000);
      const __amdgpu_buffer_rsrc_t rb =
          __builtin_amdgcn_make_buffer_rsrc((void*)(B + n0 * ldb), (short)0, 0x7fffffff, 0x00020000);
      const int alim = M - 1 - m0;                      // last valid row of the A panel
      const int blim = (int)min(N - 1 - n0, (int64_t)T::BN - 1);
      const int a4 = (int)lda * 4, b4 = (int)ldb * 4;
#pragma unroll
      for (int i = 0; i < T::LOADS; ++i) {
        const int f = tid + i * T::THREADS;
        if (T::PARTIAL && i == T::LOADS - 1 && f >= T::TOTAL_F4) break;
        const int row = f / T::F4_PER_ROW, ch = f % T::F4_PER_ROW;
        if (i < T::BM * T::F4_PER_ROW / T::THREADS)
          r[i] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 ra, min(row, alim) * a4 + ch * 16, k0 * 4, 0));
        else
          r[i] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rb, min(row - T::BM, blim) * b4 + ch * 16, k0 * 4, T::NTB ? 2 : 0));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < T::LOADS; ++i) {
      const int f = tid + i * T::THREADS;
      if (T::PARTIAL && i == T::LOADS - 1 && f >= T::TOTAL_F4) break;
      const int row = f / T::F4_PER_ROW, ch = f % T::F4_PER_ROW;
      const float* p;
      const bool a_row = T::A_SLOTS ? i < T::BM * T::F4_PER_ROW / T::THREADS  // compile-time: A rows first
                                    : f < T::BM * T::F4_PER_ROW;
      if (a_row) {
        p = A + (int64_t)min(m0 + row, M - 1) * lda;
      } else {
        p = B + min(n0 + (int64_t)(row - T::BM), N - 1) * ldb;
      }
      r[i] = *reinterpret_cast<const floatx4*>(p + k0 + ch * 4);
    }
  }

  __device__ __forceinline__ void store(float* stage, int tid) const {
#pragma unroll
    for (int i = 0; i < T::LOADS; ++i) {
      const int f = tid + i * T::THREADS;
      if (T::PARTIAL && i == T::LOADS - 1 && f >= T::TOTAL_F4) break;
      const int row = f / T::F4_PER_ROW, ch = f % T::F4_PER_ROW;
      if constexpr (T::X6) {
        uint2 pl[3];
        split3(r[i], pl);
        char* base = reinterpret_cast<char*>(stage + row * T::ROW_FLOATS) + ch * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(base + p * 32) = pl[p];
      } else {
        *reinterpret_cast<floatx4*>(stage + row * T::ROW_FLOATS + ch * 4) = r[i];
      }
    }
  }
};

// MFMAs of one staged K-slice for wave (wm, wn).
template <class T>
__device__ __forceinline__ void mma_slice(const float* stage, floatx16 (&acc)[T::TM][T::TN],
                                          int wm, int wn, int lane) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (T::BF16) {
    // lane half h: k = 32h .. 32h+31 of the 64-wide slice; step q takes k = 32h + 8q + j
    const float* as = stage + (wm * T::WM + r) * T::ROW_FLOATS + h * 16;
    const float* bs = stage + (T::BM + wn * T::WN + r) * T::ROW_FLOATS + h * 16;
    // two fragment sets, reads of step q+1 pinned ahead of the MFMAs of step q (as in the
    // f32 path below; a bf16 step is only TM*TN short MFMAs, so an exposed LDS round trip
    // per step costs proportionally more here)
    bf16x8 a[2][T::TM], b[2][T::TN];
    auto frag = [&](int q, bf16x8(&fa)[T::TM], bf16x8(&fb)[T::TN]) {
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
        fa[tm] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const floatx4*>(as + tm * 32 * T::ROW_FLOATS + q * 4));
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn)
        fb[tn] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const floatx4*>(bs + tn * 32 * T::ROW_FLOATS + q * 4));
    };
    frag(0, a[0], b[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = q & 1;
      if (q + 1 < 4) frag(q + 1, a[c ^ 1], b[c ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c][tm], b[c][tn], acc[tm][tn], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }
  if constexpr (T::X6) {
    // lane half h: k = 8h .. 8h+7 of this 16-wide slice, one ds_read_b128 per plane
    const char* as = reinterpret_cast<const char*>(stage + (wm * T::WM + r) * T::ROW_FLOATS) + h * 16;
    const char* bs = reinterpret_cast<const char*>(stage + (T::BM + wn * T::WN + r) * T::ROW_FLOATS) + h * 16;
    bf16x8 a[T::TM][3], b[T::TN][3];
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        a[tm][p] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(as + tm * 32 * T::ROW_FLOATS * 4 + p * 32));
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        b[tn][p] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uintx4*>(bs + tn * 32 * T::ROW_FLOATS * 4 + p * 32));
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn) {
        // smallest terms first
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][2], b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][1], b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][2], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][1], b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][0], acc[tm][tn], 0, 0, 0);
      }
    return;
  }
  // lane half h carries k = h BK/2 + 4 q + s (q < BK / 8)
  constexpr int QN = T::BK / 8;
  const float* as = stage + (wm * T::WM + r) * T::ROW_FLOATS + h * (T::BK / 2);
  const float* bs = stage + (T::BM + wn * T::WN + r) * T::ROW_FLOATS + h * (T::BK / 2);
  // Two fragment sets: the ds_reads of step q+1 go out under the MFMAs of step q.  Left
  // to itself the scheduler reads two steps at once into ONE register set, so the reads
  // of steps 2-3 wait (WAR) for the last MFMA of step 1 and the pipe idles for an LDS
  // round trip mid-slice.  MFMA order per accumulator is unchanged (bit-identical sums).
  floatx4 a[2][T::TM], b[2][T::TN];
  auto frag = [&](int q, floatx4(&fa)[T::TM], floatx4(&fb)[T::TN]) {
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
      fa[tm] = *reinterpret_cast<const floatx4*>(as + tm * 32 * T::ROW_FLOATS + q * 4);
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
      fb[tn] = *reinterpret_cast<const floatx4*>(bs + tn * 32 * T::ROW_FLOATS + q * 4);
  };
  // Each step is its own scheduling block (the scheduler would otherwise pick reads of
  // any step to interleave, or sink the reads to the end of the MFMA run): reads of q+1,
  // then the MFMAs of q, each pinned by a sched_barrier.
  frag(0, a[0], b[0]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < QN; ++q) {
    const int c = q & 1;
    if (q + 1 < QN) frag(q + 1, a[c ^ 1], b[c ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
          acc[tm][tn] =
              __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][tm][s], b[c][tn][s], acc[tm][tn], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <class T>
__device__ __forceinline__ void zero_acc(floatx16 (&acc)[T::TM][T::TN]) {
#pragma unroll
  for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;
}

// Row (within the wave tile) of accumulator register e for this lane; the column is
// tn * 32 + (lane & 31).  C/D map of the 32x32 MFMA family on gfx950.
__device__ __forceinline__ int acc_row(int tm, int e, int lane) {
  return tm * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5): consecutive logical tiles
// land on the same XCD (blocks b and b+8 share one), for L2 reuse of shared panels.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Division by a launch-invariant divisor 1 <= d < 2^31 for dividends 0 <= n < 2^31 by a
// magic multiplier (Granlund-Montgomery): q = (mulhi(n, m) + n) >> s, s = ceil(log2 d).
// The tile walks divide slice and tile counters every K-slice; hipcc's signed 32-bit
// division is ~25 scalar instructions (abs / mul_hi / sign fix-ups) - this is three.
// (Checked exhaustively for d < 3000, n < 2000 and on random d, n < 2^31.)
struct FastDiv {
  unsigned d, m, s;
  __device__ __forceinline__ explicit FastDiv(int d_) : d((unsigned)d_) {
    s = d > 1 ? 32 - __builtin_clz(d - 1) : 0;
    m = (unsigned)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  }
  __device__ __forceinline__ int div(int n) const {
    return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> s);
  }
  __device__ __forceinline__ int mod(int n) const { return n - div(n) * (int)d; }
};

// Operands of a tile walk: A [M][lda], B [N][ldb], both K-contiguous, K % 32 == 0.
struct TileOperands {
  const float* A;
  int64_t lda;
  int M;
  const float* B;
  int64_t ldb;
  int64_t N;
  int K;
};

// Stream every K-slice of this workgroup's tiles through a double-buffered LDS image
// with global loads running D slices ahead in D named register stages (compile-time
// stage indices: no runtime register indexing).  Iteration j: request slice j+D into
// the stage slice j vacated, multiply slice j, then write slice j+1 (requested D-1
// iterations earlier) to the free LDS buffer; one barrier.  The prefetch runs straight
// across tile boundaries.  coords(i, &m0, &n0) gives the origin of the i-th tile;
// epi(i, acc, released_stage) runs after the last slice of tile i, with
// `released_stage` an LDS buffer no wave reads before the next barrier (an epilogue
// that uses it must end with a barrier).
template <class T, int D = T::PF, class Coords, class Epi>
__device__ __forceinline__ void walk_tiles(float* lds, int n_tiles, const TileOperands& op,
                                           Coords coords, Epi epi) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int nk = op.K / T::BK;
  const int S = n_tiles * nk;
  if (S == 0) return;
  const FastDiv nkd(nk);
  auto fetch = [&](Stager<T>& st, int j) {
    const int i = nkd.div(j), kt = j - i * nk;
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    st.load(op.A, op.lda, op.M, m0, op.B, op.ldb, op.N, n0, kt * T::BK, tid);
  };
  // The slice body is branch-free: the prefetch past the last slice re-reads slice S-1
  // and the store after the last slice fills the idle buffer.  A conditional fetch or
  // store makes the compiler's wait-count merge at the join fall back to vmcnt(0) at the
  // top of every slice, i.e. it waits for the loads it has just issued (measured: ~30%
  // of MFMA cycles idle).  Accumulators are zeroed at tile ends, not by a per-slice
  // select that would wait for the MFMA pipe to drain.
  floatx16 acc[T::TM][T::TN];
  Stager<T> st[D];
  static_for<D>([&](auto dc) {
    constexpr int d = decltype(dc)::value;
    fetch(st[d], d < S ? d : S - 1);
  });
  st[0].store(lds, tid);
  zero_acc<T>(acc);
  __syncthreads();
  for (int j0 = 0; j0 < S; j0 += D) {
    bool done = false;
    static_for<D>([&](auto dc) {
      constexpr int d = decltype(dc)::value;
      const int j = j0 + d;
      if (done || j >= S) {
        done = true;
        return;
      }
      fetch(st[d], min(j + D, S - 1));  // slice j's stage is free (stored last iteration)
      // pin the loads at the top of the slice: sunk below the MFMAs, their destinations
      // get coalesced with the fragment registers and the next slice's ds_reads wait on
      // them (WAW)
      __builtin_amdgcn_sched_barrier(0);
      float* cur = lds + (j & 1) * T::STAGE_FLOATS;
      __builtin_amdgcn_s_setprio(1);
      mma_slice<T>(cur, acc, wm, wn, lane);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      st[(d + 1) % D].store(lds + ((j + 1) & 1) * T::STAGE_FLOATS, tid);
      __syncthreads();
      if (nkd.mod(j + 1) == 0) {
        epi(nkd.div(j), acc, cur);
        zero_acc<T>(acc);
      }
    });
  }
}

}  // namespace mq

namespace mq {

// walk_tiles with hooks around the operand staging (D >= 2), for GEMMs that transform an
// operand between its global load and its LDS write (LayerNorm on load, encoder.hip):
//   hk.issue(s, IC<d>)      before the loads of slice s (unclamped; s >= S: the re-read
//                           past the end) into register stage d
//   hk.prepare(s)           at the store phase of the iteration that fetched slice s, before
//                           that iteration's barrier (per-tile state into LDS: read by
//                           xform from the next iteration on)
//   hk.stage_in(s)          at the top of the iteration that stores slice s (before its
//                           MFMAs: per-slice state read from LDS under them)
//   hk.xform(st, s, IC<d>)  on stage d's registers just before they are written to LDS
// Otherwise the slice schedule is walk_tiles' (same loads, MFMAs, barriers).
template <class T, int D = T::PF, class Coords, class Epi, class Hooks>
__device__ __forceinline__ void walk_tiles_hooked(float* lds, int n_tiles, const TileOperands& op,
                                                  Coords coords, Epi epi, Hooks& hk) {
  static_assert(D >= 2, "the hooks need the slice's loads one iteration before its store");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int nk = op.K / T::BK;
  const int S = n_tiles * nk;
  if (S == 0) return;
  const FastDiv nkd(nk);
  auto fetch = [&](Stager<T>& st, int j) {
    const int i = nkd.div(j), kt = j - i * nk;
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    // tile origins are workgroup-uniform: keep them (and the buffer descriptors built from
    // them) scalar whatever the hooks' per-thread code does to the uniformity analysis
    m0 = __builtin_amdgcn_readfirstlane(m0);
    n0 = (int64_t)__builtin_amdgcn_readfirstlane((int)n0);
    st.load(op.A, op.lda, op.M, m0, op.B, op.ldb, op.N, n0, kt * T::BK, tid);
  };
  floatx16 acc[T::TM][T::TN];
  Stager<T> st[D];
  static_for<D>([&](auto dc) {
    constexpr int d = decltype(dc)::value;
    hk.issue(d, dc);
    fetch(st[d], d < S ? d : S - 1);
  });
  static_for<D>([&](auto dc) { hk.prepare(decltype(dc)::value); });
  __syncthreads();
  hk.stage_in(0);
  hk.xform(st[0], 0, IC<0>{});
  st[0].store(lds, tid);
  zero_acc<T>(acc);
  __syncthreads();
  for (int j0 = 0; j0 < S; j0 += D) {
    bool done = false;
    static_for<D>([&](auto dc) {
      constexpr int d = decltype(dc)::value;
      const int j = j0 + d;
      if (done || j >= S) {
        done = true;
        return;
      }
      hk.issue(j + D, dc);
      fetch(st[d], min(j + D, S - 1));
      hk.stage_in(j + 1);
      __builtin_amdgcn_sched_barrier(0);
      float* cur = lds + (j & 1) * T::STAGE_FLOATS;
      __builtin_amdgcn_s_setprio(1);
      mma_slice<T>(cur, acc, wm, wn, lane);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      hk.prepare(j + D);
      hk.xform(st[(d + 1) % D], j + 1, IC<(d + 1) % D>{});
      st[(d + 1) % D].store(lds + ((j + 1) & 1) * T::STAGE_FLOATS, tid);
      __syncthreads();
      if (nkd.mod(j + 1) == 0) {
        epi(nkd.div(j), acc, cur);
        zero_acc<T>(acc);
      }
    });
  }
}

}  // namespace mq
