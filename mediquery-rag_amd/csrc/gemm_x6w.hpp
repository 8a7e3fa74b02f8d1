// gemm_x6w.hpp - wide split-f32 GEMM core for gfx950: 8-wave workgroups, operands in
// the tiled pre-split layout P3T, fed global -> LDS by LDS-DMA (global_load_lds_dwordx4).
//
// Same arithmetic as the X6 path of gemm_f32.hpp (three exact bf16 planes per operand,
// six v_mfma_f32_32x32x16_bf16 per 32x32x16 block, smallest terms first, fp32
// accumulate, k-chunks in order), so results are bit-identical to it.  What changes is
// the feed, built for the MFMA rate of bf16 (cdna_hip_programming.md §5, "Pipelining
// across barriers" and the projection-GEMM notes):
//  * P3T: X [R][K] is stored as 1-KiB pieces, piece (rb, c, p) = rows 32rb..32rb+31,
//    k-chunk c (16 wide), plane p, laid out [h][32 rows][8 bf16] (h = which 8 k of the
//    chunk).  One piece is exactly the LDS image of one MFMA operand fragment block, and
//    one wave instruction of global_load_lds_dwordx4 copies it (lane l: bytes 16l..16l+15)
//    - fully coalesced reads, lane-linear LDS writes, conflict-free ds_read_b128 (lanes
//    0-15 read 256 contiguous bytes).  Rows are padded to a multiple of 32.
//  * 8 waves (two per SIMD), a BM x BN block tile, CH k-chunks per stage, two stages.
//    Per stage: issue the next stage's DMA, wait (counted vmcnt) for this stage's own
//    DMA, raw barrier, fragments + MFMAs, raw barrier.  No __syncthreads (its fence
//    would drain the in-flight DMA), no VGPR staging, no VALU split.
//  * Persistent workgroups (one per CU) walk tiles; blocks b and b+8 share an XCD.
#pragma once

#include "gemm_f32.hpp"

namespace mq {

// ----------------------------------------------------------------- P3T layout -----
// Floats of a P3T matrix with `rows` rows (padded to 32) and K columns.
__host__ __device__ inline int64_t p3t_floats(int64_t rows, int K) {
  return (rows + 31) / 32 * 32 * (int64_t)K * 3 / 2;
}

// Float offset of piece (rb, c, p) of a P3T matrix with K columns.
__device__ __forceinline__ int64_t p3t_piece(int64_t rb, int c, int p, int K) {
  return ((rb * (K >> 4) + c) * 3 + p) * 256;
}

// src [rows][K] fp32 (row stride lds) -> P3T; one thread per (row block, chunk, row),
// row fastest: consecutive threads write consecutive 16-B slots.  Pad rows repeat the
// last row (finite values; their products only reach output rows nobody stores).
template <int Unused = 0>
__global__ __launch_bounds__(256) void split_p3t_kernel(const float* __restrict__ src, int64_t lds,
                                                        int64_t rows, int K, float* __restrict__ dst) {
  const int64_t chunks = K >> 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t rbs = (rows + 31) / 32;
  if (i >= rbs * chunks * 32) return;
  const int r32 = (int)(i & 31);
  const int64_t t = i >> 5, c = t % chunks, rb = t / chunks;
  const int64_t r = min(rb * 32 + r32, rows - 1);
  const floatx4* s = reinterpret_cast<const floatx4*>(src + r * lds + c * 16);
  uint2 pl[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q) split3(s[q], pl[q]);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    float* piece = dst + p3t_piece(rb, (int)c, p, K);
    *reinterpret_cast<uintx4*>(piece + r32 * 4) = uintx4{pl[0][p].x, pl[0][p].y, pl[1][p].x, pl[1][p].y};
    *reinterpret_cast<uintx4*>(piece + 128 + r32 * 4) =
        uintx4{pl[2][p].x, pl[2][p].y, pl[3][p].x, pl[3][p].y};
  }
}

inline void launch_split_p3t(const float* src, int64_t lds, int64_t rows, int K, float* dst,
                             hipStream_t s) {
  const int64_t n = (rows + 31) / 32 * (K >> 4) * 32;
  if (rows > 0)
    hipLaunchKernelGGL(split_p3t_kernel<0>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src,
                       lds, rows, K, dst);
}

// Store 4 consecutive values (columns col..col+3, col % 4 == 0) of row `row` into a
// P3T matrix with K columns: 8 B per plane.
__device__ __forceinline__ void p3t_store4(float* __restrict__ dst, int64_t row, int col, int K,
                                           floatx4 v) {
  uint2 pl[3];
  split3(v, pl);
  const int64_t rb = row >> 5;
  const int c = col >> 4, h = (col >> 3) & 1;
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<uint2*>(dst + p3t_piece(rb, c, p, K) + h * 128 + (row & 31) * 4 + ((col & 7) >> 1)) = pl[p];
}

// Store 16 consecutive values (columns col..col+15, col % 16 == 0) of one row: 6 x 16 B.
__device__ __forceinline__ void p3t_store16(float* __restrict__ dst, int64_t row, int col, int K,
                                            const floatx4 (&v)[4]) {
  uint2 pl[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q) split3(v[q], pl[q]);
  const int64_t rb = row >> 5;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    float* piece = dst + p3t_piece(rb, col >> 4, p, K) + (row & 31) * 4;
    *reinterpret_cast<uintx4*>(piece) = uintx4{pl[0][p].x, pl[0][p].y, pl[1][p].x, pl[1][p].y};
    *reinterpret_cast<uintx4*>(piece + 128) = uintx4{pl[2][p].x, pl[2][p].y, pl[3][p].x, pl[3][p].y};
  }
}

// ------------------------------------------------------------------ tile core -----
template <int WAVES_M_, int WAVES_N_, int TM_, int TN_, int CH_>
struct WTile {
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, TM = TM_, TN = TN_, CH = CH_;
  static constexpr int WAVES = WAVES_M * WAVES_N;
  static constexpr int THREADS = WAVES * kWave;
  static constexpr int WM = TM * 32, WN = TN * 32;
  static constexpr int BM = WAVES_M * WM, BN = WAVES_N * WN;
  static constexpr int RBA = BM / 32, RBB = BN / 32, RB = RBA + RBB;  // 32-row blocks
  static constexpr int BK = 16 * CH;
  static constexpr int NP = CH * 3 * RB;                  // 1-KiB pieces per stage
  static constexpr int NG = (NP + WAVES - 1) / WAVES;      // DMA instructions per wave per stage
  static constexpr int STAGE_FLOATS = NP * 256;
  static_assert(2 * STAGE_FLOATS * 4 <= 160 * 1024, "two stages must fit the LDS");
  static_assert(NG < 32, "vmcnt immediate");
};

// LDS byte address of a __shared__ pointer (the DMA's M0 operand).
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)p));
}

// One 1-KiB LDS-DMA piece: lane l copies 16 B from `src` to lds_base + 16 l.  Inline asm
// so hipcc does not treat it as an LDS store aliasing the fragment reads (the builtin
// makes it wait vmcnt(0) before every ds_read); completion is counted by hand.  M0 is
// saved and restored inside the statement.
__device__ __forceinline__ void dma16(const float* src, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_base)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier that leaves LDS-DMA in flight (retires this wave's LDS reads first).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Operands of a wide walk: A3 / B3 are P3T with M / N rows and K columns.
struct WideOperands {
  const float* A3;
  int M;
  const float* B3;
  int N;
  int K;
};

// Request stage data for k-chunks [c0, c0 + CH) of the tile at (m0, n0) into `stage`.
// Piece q = (c * 3 + p) * RB + block; blocks < RBA are A row blocks.  Waves take pieces
// wave, wave + WAVES, ...; a wave with a spare slot repeats the last piece (same bytes to
// the same place), so every wave issues exactly NG instructions.
template <class T>
__device__ __forceinline__ void dma_stage(float* stage, const WideOperands& op, int m0, int n0,
                                          int c0, int wave, int lane) {
  const int64_t rbA_last = (op.M - 1) >> 5, rbB_last = (op.N - 1) >> 5;
#pragma unroll
  for (int i = 0; i < T::NG; ++i) {
    const int q = min(wave + i * T::WAVES, T::NP - 1);
    const int c = q / (3 * T::RB), rem = q - c * (3 * T::RB);
    const int p = rem / T::RB, blk = rem - p * T::RB;
    const float* src;
    if (blk < T::RBA)
      src = op.A3 + p3t_piece(min((int64_t)(m0 >> 5) + blk, rbA_last), c0 + c, p, op.K);
    else
      src = op.B3 + p3t_piece(min((int64_t)(n0 >> 5) + blk - T::RBA, rbB_last), c0 + c, p, op.K);
    dma16(src + lane * 4, __builtin_amdgcn_readfirstlane(lds_addr(stage + q * 256)));
  }
}

// The MFMAs of one stage for wave (wm, wn): per chunk, fragments of every plane, then
// the six products per block, smallest first (same order as gemm_f32.hpp's X6 path).
template <class T>
__device__ __forceinline__ void mma_stage(const float* stage, floatx16 (&acc)[T::TM][T::TN], int wm,
                                          int wn, int lane) {
  const int off = (lane >> 5) * 128 + (lane & 31) * 4;  // [h][row][8 bf16] inside a piece
#pragma unroll
  for (int c = 0; c < T::CH; ++c) {
    bf16x8 a[T::TM][3], b[T::TN][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
        a[tm][p] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uintx4*>(stage + ((c * 3 + p) * T::RB + wm * T::TM + tm) * 256 + off));
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn)
        b[tn][p] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uintx4*>(
                        stage + ((c * 3 + p) * T::RB + T::RBA + wn * T::TN + tn) * 256 + off));
    }
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn) {
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][2], b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][1], b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][2], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][1], b[tn][0], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][1], acc[tm][tn], 0, 0, 0);
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm][0], b[tn][0], acc[tm][tn], 0, 0, 0);
      }
  }
}

template <class T>
__device__ __forceinline__ void zero_acc_w(floatx16 (&acc)[T::TM][T::TN]) {
#pragma unroll
  for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;
}

// Walk the stages of this workgroup's tiles (two LDS stages, DMA one stage ahead).
// coords(i, m0, n0) gives tile i's origin; epi(i, acc, stage) runs after its last stage
// with every wave past a barrier that follows the last fragment reads of `stage`, so the
// epilogue may use `stage` as scratch (the walk barriers again before refilling it).
// Every stage runs the same instruction stream: the DMA past the last stage re-reads
// stage S-1's data into the idle buffer.
template <class T, class Coords, class Epi>
__device__ __forceinline__ void walk_tiles_wide(float* lds, int n_tiles, const WideOperands& op,
                                                Coords coords, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int nk = op.K / T::BK;
  const int S = n_tiles * nk;
  if (S == 0) return;
  auto fetch = [&](int j) {
    const int i = j / nk, kt = j - i * nk;
    int m0;
    int n0;
    coords(i, m0, n0);
    dma_stage<T>(lds + (j & 1) * T::STAGE_FLOATS, op, m0, n0, kt * T::CH, wave, lane);
  };
  floatx16 acc[T::TM][T::TN];
  zero_acc_w<T>(acc);
  fetch(0);
  for (int j = 0; j < S; ++j) {
    fetch(min(j + 1, S - 1));   // into the other buffer, free since the last barrier
    wait_vmcnt<T::NG>();        // this wave's DMA for stage j has landed ...
    lds_barrier();              // ... and every other wave's
    float* cur = lds + (j & 1) * T::STAGE_FLOATS;
    __builtin_amdgcn_s_setprio(1);
    mma_stage<T>(cur, acc, wm, wn, lane);
    __builtin_amdgcn_s_setprio(0);
    lds_barrier();              // every wave is done reading `cur`
    if ((j + 1) % nk == 0) {
      epi(j / nk, acc, cur);
      zero_acc_w<T>(acc);
      lds_barrier();            // the epilogue's scratch use of `cur` is over
    }
  }
  wait_vmcnt<0>();  // the trailing DMA must land before the workgroup retires its LDS
}

}  // namespace mq
