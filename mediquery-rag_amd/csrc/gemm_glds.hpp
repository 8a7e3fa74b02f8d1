// gemm_glds.hpp - exact-fp32 MFMA tile core fed by LDS-DMA (global_load_lds), gfx950.
//
// Same arithmetic as gemm_f32.hpp (v_mfma_f32_32x32x2_f32, lane half h carries k =
// 16h..16h+15 of each 32-wide K-slice), different feed:
//  * K-slices go global -> LDS directly with `global_load_lds_dwordx4` (no staging
//    VGPRs, no ds_write): one wave instruction fills 1 KiB = 8 rows x 128 B.
//  * LDS rows are NOT padded (the DMA destination is lane-linear); bank conflicts are
//    removed by an XOR swizzle of the 16-B chunk index, applied on the per-lane SOURCE
//    address and on the ds_read address (cdna_hip_programming.md §5.4 rule 21):
//        LDS chunk = logical chunk ^ ((row >> 1) & 7)
//    For ds_read_b128 lane groups (16 distinct rows mod 16, one logical chunk) the 16
//    (row parity, swizzled chunk) pairs are distinct -> conflict-free.
//  * NS-stage LDS ring, slices fetched NS-1 ahead; one raw s_barrier per slice behind a
//    counted `s_waitcnt vmcnt` (never __syncthreads, whose fence would drain the DMA).
#pragma once

#include "common.hpp"
#include "gemm_f32.hpp"  // TileOperands, acc_row, zero_acc, kBK

namespace mq {

template <int WAVES_M_, int WAVES_N_, int TM_, int TN_, int NS_>
struct GTile {
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, TM = TM_, TN = TN_, NS = NS_;
  static constexpr int WM = TM * 32, WN = TN * 32;
  static constexpr int BM = WAVES_M * WM, BN = WAVES_N * WN;
  static constexpr int WAVES = WAVES_M * WAVES_N;
  static constexpr int THREADS = WAVES * kWave;
  static constexpr int ROWS = BM + BN;
  static constexpr int STAGE_FLOATS = ROWS * kBK;  // 128-B rows, no padding
  static constexpr int GLDS = ROWS / 8 / WAVES;    // DMA instructions per wave per slice
  static constexpr int LDS_FLOATS = NS * STAGE_FLOATS;
  static constexpr int BLOCKS_PER_CU = (160 * 1024) / (LDS_FLOATS * 4) >= 2 && WAVES == 4 ? 2 : 1;
  static_assert(ROWS % (8 * WAVES) == 0, "each wave must fill whole 8-row DMA pieces");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "block tile must be a multiple of 32");
  static_assert(NS >= 2 && LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ int chunk_swz(int row) { return (row >> 1) & 7; }

// LDS byte address of a __shared__ pointer (the DMA's M0 operand).
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)p));
}

// One 1-KiB LDS-DMA piece: every lane copies 16 B from `src` to lds_base + 16 * lane.
// Issued through inline asm so hipcc does not treat it as an LDS store that may alias
// the ring's ds_reads (the builtin form makes it wait vmcnt(0) before every fragment
// read); completion is counted by hand (wait_vmcnt) before the barrier that publishes
// the stage.  M0 is saved/restored inside the statement (cdna_hip_programming.md §5.7).
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

// Request K-slice [k0, k0+32) of the tile at (m0, n0) into `stage`.
template <class T>
__device__ __forceinline__ void dma_slice(float* stage, const TileOperands& op, int m0, int64_t n0,
                                          int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < T::GLDS; ++i) {
    const int r0 = (wave * T::GLDS + i) * 8;  // wave-uniform first row of this 1-KiB piece
    const int row = r0 + (lane >> 3);
    const int c = (lane & 7) ^ chunk_swz(row);  // logical chunk this lane's 16 B belong to
    const float* p = r0 < T::BM ? op.A + (int64_t)min(m0 + row, op.M - 1) * op.lda
                                : op.B + min(n0 + (int64_t)(row - T::BM), op.N - 1) * op.ldb;
    dma16(p + k0 + c * 4, __builtin_amdgcn_readfirstlane(lds_addr(stage + r0 * kBK)));
  }
}

// MFMAs of one staged slice (swizzled image) for wave (wm, wn).
template <class T>
__device__ __forceinline__ void mma_slice_swz(const float* stage, floatx16 (&acc)[T::TM][T::TN],
                                              int wm, int wn, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int key = chunk_swz(r);  // rows r + 32t share it
  const float* as = stage + (wm * T::WM + r) * kBK;
  const float* bs = stage + (T::BM + wn * T::WN + r) * kBK;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int off = (((4 * h + q) ^ key) * 4);
    floatx4 a[T::TM], b[T::TN];
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm) a[tm] = *reinterpret_cast<const floatx4*>(as + tm * 32 * kBK + off);
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn) b[tn] = *reinterpret_cast<const floatx4*>(bs + tn * 32 * kBK + off);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][s], b[tn][s], acc[tm][tn], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Raw workgroup barrier that does not drain in-flight LDS-DMA (no vmcnt(0) fence);
// LDS reads issued before it are retired first.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Walk every K-slice of this workgroup's tiles through the NS-stage ring.
// coords(i, m0, n0): origin of the i-th tile.  epi(i, acc, stage): after the last
// slice of tile i; `stage` (STAGE_FLOATS) is free for the epilogue, which must end
// with lds_barrier() if it writes it.
template <class T, class Coords, class Epi>
__device__ __forceinline__ void walk_tiles_dma(float* lds, int n_tiles, const TileOperands& op,
                                               Coords coords, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int nk = op.K / kBK;
  const int S = n_tiles * nk;
  if (S == 0) return;
  auto fetch = [&](int j) {
    const int i = j / nk, kt = j - i * nk;
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    dma_slice<T>(lds + (j % T::NS) * T::STAGE_FLOATS, op, m0, n0, kt * kBK, wave, lane);
  };
#pragma unroll
  for (int p = 0; p < T::NS - 1; ++p)
    if (p < S) fetch(p);
  floatx16 acc[T::TM][T::TN];
  for (int j = 0; j < S; ++j) {
    // my DMA for slice j is done once at most the NS-2 younger slices are in flight
    if (j + T::NS - 2 < S)
      wait_vmcnt<T::GLDS*(T::NS - 2)>();
    else
      wait_vmcnt<0>();
    lds_barrier();  // every wave's slice j landed; every wave is done with slice j-1
    if (j + T::NS - 1 < S) fetch(j + T::NS - 1);  // refills the stage of slice j-1
    if (j % nk == 0) zero_acc<T>(acc);
    float* st = lds + (j % T::NS) * T::STAGE_FLOATS;
    mma_slice_swz<T>(st, acc, wm, wn, lane);
    if ((j + 1) % nk == 0) epi(j / nk, acc, st);
  }
}

}  // namespace mq
