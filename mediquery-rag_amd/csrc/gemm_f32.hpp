// gemm_f32.hpp - exact-fp32 MFMA tile core for gfx950 (v_mfma_f32_32x32x2_f32).
//
// Computes D[i][j] = sum_k A[i][k] * B[j][k] for a BM x BN block tile, both operands
// K-contiguous ("NT": activations/queries [M][K], weights/corpus rows [N][K]).
//
//  * 256 threads = 4 waves laid out WAVES_M x WAVES_N; each wave owns TM x TN MFMA
//    tiles of 32x32 (f32x16 accumulators, 16 regs/lane each).
//  * K is staged in BK = 32 slices through a double-buffered LDS image
//    [rows][BK + 4] floats: rows of 144 B keep the staging ds_write_b128 and the
//    fragment ds_read_b128 bank-conflict free (slot = 9*row + 4*h + q mod 16).
//  * K order inside a slice is permuted so that one lane's 16 k-values are contiguous:
//    MFMA step (q, s), lane half h (= lane >> 5) carries k = 16h + 4q + s for BOTH
//    operands, so each lane fetches its fragment with 4 ds_read_b128 per slice
//    instead of 16 ds_read_b32.  A dot product is order-free up to fp32 rounding, and
//    the f32 MFMA is an exact fmaf chain (no TF32 / xf32 on gfx950).
//  * Next-slice global loads are issued into registers before the MFMAs of the current
//    slice and written to the other LDS buffer after them: one barrier per slice.
#pragma once

#include "common.hpp"

namespace mq {

constexpr int kBK = 32;
constexpr int kLdsStride = kBK + 4;  // floats per staged row (144 B)

template <int WAVES_M_, int WAVES_N_, int TM_, int TN_>
struct F32Tile {
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, TM = TM_, TN = TN_;
  static constexpr int WM = TM * 32, WN = TN * 32;  // wave tile
  static constexpr int BM = WAVES_M * WM, BN = WAVES_N * WN;
  static constexpr int THREADS = WAVES_M * WAVES_N * kWave;
  static constexpr int ROWS = BM + BN;
  static constexpr int LOADS = ROWS * (kBK / 4) / THREADS;  // float4 per thread per slice
  static constexpr int STAGE_FLOATS = ROWS * kLdsStride;
  static_assert(THREADS == 256, "tile core assumes 256-thread workgroups");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "block tile must be a multiple of 32");
  static_assert(ROWS * (kBK / 4) % THREADS == 0, "staging must divide evenly");
};

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
#pragma unroll
    for (int i = 0; i < T::LOADS; ++i) {
      const int f = tid + i * T::THREADS;
      const int row = f >> 3, ch = f & 7;
      const float* p;
      if (i < T::BM / 32) {  // compile-time after unrolling: rows [32i, 32i+32) are A rows
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
      const int row = f >> 3, ch = f & 7;
      *reinterpret_cast<floatx4*>(stage + row * kLdsStride + ch * 4) = r[i];
    }
  }
};

// MFMAs of one staged K-slice for wave (wm, wn).
template <class T>
__device__ __forceinline__ void mma_slice(const float* stage, floatx16 (&acc)[T::TM][T::TN],
                                          int wm, int wn, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const float* as = stage + (wm * T::WM + r) * kLdsStride + h * 16;
  const float* bs = stage + (T::BM + wn * T::WN + r) * kLdsStride + h * 16;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    floatx4 a[T::TM], b[T::TN];
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
      a[tm] = *reinterpret_cast<const floatx4*>(as + tm * 32 * kLdsStride + q * 4);
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
      b[tn] = *reinterpret_cast<const floatx4*>(bs + tn * 32 * kLdsStride + q * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
          acc[tm][tn] =
              __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][s], b[tn][s], acc[tm][tn], 0, 0, 0);
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
// with global loads running TWO slices ahead (two named register stages, so no runtime
// register indexing): slice j+2 is requested while slice j is multiplied, and slice
// j+1 - requested one whole slice earlier - is written to the free buffer after the
// MFMAs.  The prefetch runs straight across tile boundaries.  coords(i, &m0, &n0)
// gives the origin of the i-th tile; epi(i, acc, released_stage) runs after the last
// slice of tile i, with `released_stage` an LDS buffer no wave reads until the next
// barrier the epilogue itself must end with if it uses it.
template <class T, class Coords, class Epi>
__device__ __forceinline__ void walk_tiles(float* lds, int n_tiles, const TileOperands& op,
                                           Coords coords, Epi epi) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int nk = op.K / kBK;
  const int S = n_tiles * nk;
  if (S == 0) return;
  auto fetch = [&](Stager<T>& st, int j) {
    const int i = j / nk, kt = j - (j / nk) * nk;
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    st.load(op.A, op.lda, op.M, m0, op.B, op.ldb, op.N, n0, kt * kBK, tid);
  };
  floatx16 acc[T::TM][T::TN];
  Stager<T> ra, rb;
  fetch(ra, 0);
  if (S > 1) fetch(rb, 1);
  ra.store(lds, tid);
  __syncthreads();
  float* buf0 = lds;
  float* buf1 = lds + T::STAGE_FLOATS;
  for (int j = 0; j < S; j += 2) {
    // even half: slice j in buf0, slice j+1 in flight in rb
    if (j % nk == 0) zero_acc<T>(acc);
    if (j + 2 < S) fetch(ra, j + 2);
    mma_slice<T>(buf0, acc, wm, wn, lane);
    if (j + 1 < S) rb.store(buf1, tid);
    __syncthreads();
    if ((j + 1) % nk == 0) epi(j / nk, acc, buf0);
    if (j + 1 >= S) break;
    // odd half: slice j+1 in buf1, slice j+2 in flight in ra
    if ((j + 1) % nk == 0) zero_acc<T>(acc);
    if (j + 3 < S) fetch(rb, j + 3);
    mma_slice<T>(buf1, acc, wm, wn, lane);
    if (j + 2 < S) ra.store(buf0, tid);
    __syncthreads();
    if ((j + 2) % nk == 0) epi((j + 1) / nk, acc, buf1);
  }
}

}  // namespace mq
