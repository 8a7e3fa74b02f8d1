// index.hip - HBM-resident flat index: K8 add/normalise, K9 fused score + top-k,
// K10 candidate merge, and the mq_index_* / mq_topk_merge_* C ABI (include/mq.h).
//
// Replaces the k-NN half of Chroma's similarity_search (reference
// src/agents/nodes.py:93 on the store of src/medical_engine.py:52): exact cosine
// ranking over L2-normalised rows, (score desc, row asc).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>

#include <unistd.h>

#include "common.hpp"
#include "gemm_f32.hpp"
#include "thresh.hpp"
#include "topk.hpp"

namespace mq {

// ============================================================ K8: add rows =====
// One wave per row: sum of squares in registers, wave reduction, scaled store.
// Row / max(||row||, 1e-12) - the F.normalize / Ollama normalisation semantics.
__global__ __launch_bounds__(256) void add_rows_kernel(const float* __restrict__ src,
                                                       float* __restrict__ dst, int64_t n,
                                                       int dim) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const floatx4* s = reinterpret_cast<const floatx4*>(src + row * dim);
  floatx4* d = reinterpret_cast<floatx4*>(dst + row * dim);
  const int nv = dim >> 2;
  float ss = 0.f;
  for (int i = lane; i < nv; i += 64) {
    floatx4 v = s[i];
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
  const float inv = 1.0f / fmaxf(sqrtf(ss), 1e-12f);
  for (int i = lane; i < nv; i += 64) {
    floatx4 v = s[i];
    d[i] = v * inv;
  }
}

// Row gather for select/compaction: one wave per output row, a plain copy (stored rows
// are already unit-norm, so no re-normalisation).
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ src,
                                                          const int64_t* __restrict__ sel, int64_t n,
                                                          int dim, float* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const floatx4* s = reinterpret_cast<const floatx4*>(src + sel[r] * dim);
  floatx4* d = reinterpret_cast<floatx4*>(dst + r * dim);
  for (int i = lane; i < (dim >> 2); i += 64) d[i] = s[i];
}

// ============================================ row masks (filtered search) ======
// A metadata condition over one column: codes[r] (-1 = key absent in row r) index a
// per-distinct-value truth table lut (its last entry: absent); 64 rows per wave, one
// ballot, lanes 0 / 32 write the two words.  mode: MQ_MASK_SET / AND / OR into bits.
// (lut == NULL: the table is the bits of lw, n_lut <= 256 - passed by value, no
// host-to-device copy for it)
struct LutWords {
  unsigned long long w[4];
};
__global__ __launch_bounds__(256) void mask_eval_kernel(const int* __restrict__ codes, int64_t n,
                                                        const unsigned char* __restrict__ lut, LutWords lw,
                                                        int n_lut, unsigned* __restrict__ bits, int mode) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool v = false;
  if (r < n) {
    const int c = codes[r];
    const int i = (c >= 0 && c < n_lut - 1) ? c : n_lut - 1;
    const unsigned long long w = i < 64 ? lw.w[0] : i < 128 ? lw.w[1] : i < 192 ? lw.w[2] : lw.w[3];
    v = lut ? lut[i] != 0 : ((w >> (i & 63)) & 1ull) != 0;
  }
  const unsigned long long b = __ballot(v);
  const int lane = threadIdx.x & 63;
  if ((lane & 31) == 0 && r < n) {
    const unsigned w = (unsigned)(lane ? b >> 32 : b);
    unsigned* d = bits + (r >> 5);
    *d = mode == MQ_MASK_AND ? (*d & w) : mode == MQ_MASK_OR ? (*d | w) : w;
  }
}

// dst (op)= src; src == NULL: op MQ_MASK_SET fills ones, MQ_MASK_AND leaves dst;
// MQ_MASK_CLEAR zeroes dst
__global__ __launch_bounds__(256) void mask_combine_kernel(unsigned* __restrict__ dst,
                                                           const unsigned* __restrict__ src,
                                                           int64_t n_words, int mode) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= n_words) return;
  const unsigned x = src ? src[w] : ~0u;
  dst[w] = mode == MQ_MASK_AND ? (dst[w] & x) : mode == MQ_MASK_OR ? (dst[w] | x) : mode == MQ_MASK_CLEAR ? 0u : x;
}

// sorted compaction of the set bits of rows [0, n): pass 1 = per-block counts (256 words
// per block), pass 2 = one block scans them (exclusive, in place; total in blk[nb]),
// pass 3 = each block writes its rows in order
__device__ __forceinline__ unsigned mask_word(const unsigned* bits, int64_t w, int64_t n) {
  if (w * 32 >= n) return 0u;
  const unsigned x = bits[w];
  const int64_t rem = n - w * 32;
  return rem >= 32 ? x : (x & ((1u << rem) - 1u));
}
__device__ __forceinline__ int block_excl_scan256(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) base += i < wave ? sh[i] : 0;
  *total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return base + incl - v;
}
__global__ __launch_bounds__(256) void mask_count_kernel(const unsigned* __restrict__ bits, int64_t n,
                                                         int* __restrict__ blk) {
  __shared__ int sh[4];
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int total;
  block_excl_scan256(__popc(mask_word(bits, w, n)), sh, &total);
  if (threadIdx.x == 0) blk[blockIdx.x] = total;
}
__global__ __launch_bounds__(256) void mask_scan_kernel(int* __restrict__ blk, int nb) {
  __shared__ int sh[4];
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int i = b0 + threadIdx.x;
    const int v = i < nb ? blk[i] : 0;
    int total;
    const int ex = block_excl_scan256(v, sh, &total);
    if (i < nb) blk[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) blk[nb] = carry;
}
__global__ __launch_bounds__(256) void mask_compact_kernel(const unsigned* __restrict__ bits, int64_t n,
                                                           const int* __restrict__ blk,
                                                           int64_t* __restrict__ rows) {
  __shared__ int sh[4];
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned x = mask_word(bits, w, n);
  int total;
  int at = blk[blockIdx.x] + block_excl_scan256(__popc(x), sh, &total);
  while (x) {
    const int b = __builtin_ctz(x);
    rows[at++] = w * 32 + b;
    x &= x - 1u;
  }
}
// result ids of the gathered sub-index -> store rows
__global__ __launch_bounds__(256) void remap_ids_kernel(int64_t* __restrict__ ids, int64_t count,
                                                        const int64_t* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < count && ids[i] >= 0) ids[i] = rows[ids[i]];
}

// ================================================ K9: fused score + top-k ======
// Search tile geometries: (WAVES_M, WAVES_N, TM, TN).
using SearchWide = F32Tile<2, 2, 2, 2>;    // 128 queries x 128 rows per block
#ifndef MQ_X6_PF
#define MQ_X6_PF 2
#endif
using SearchWideX6 = F32Tile<2, 2, 2, 2, true, MQ_X6_PF>;  // same, split-f32 arithmetic
#ifndef MQ_BF_PF
#define MQ_BF_PF 2
#endif
using SearchWideBF = F32Tile<2, 2, 2, 2, false, MQ_BF_PF, true>;  // bf16 coarse scan
using SearchNarrowBF = F32Tile<1, 4, 1, 1, false, 2, true>;  // bf16 coarse, small batches
using SearchNarrow = F32Tile<1, 4, 1, 1>;  // 32 queries x 128 rows per block (small batches)

template <class T>
struct SearchSmem {
  // The finished wave tile is scanned in TN passes of 32 columns; each pass parks the
  // wave's [WM][32] scores in the LDS stage buffer the last K-slice just released
  // (row stride 36 floats = 144 B: conflict-free ds_read_b128 row scans).
  // (exact-f32 stages hold 32-column passes; the smaller split-f32 stages 16-column ones)
  static constexpr int PASS_COLS = T::X6 ? 16 : 32;
  static constexpr int SCORE_STRIDE = PASS_COLS + 4;
  static constexpr int SCORE_FLOATS = T::WM * SCORE_STRIDE;  // per wave per pass
  static constexpr int LPQ = kWave / T::WM;                   // lanes scanning one query row
  static constexpr int COLS = PASS_COLS / LPQ;                // columns per lane per pass
  static_assert(4 * SCORE_FLOATS <= T::STAGE_FLOATS, "score tile must fit a stage buffer");
  static_assert(2 * T::STAGE_FLOATS * 4 <= 80 * 1024, "two workgroups per CU");
};

// Grid: nqt query tiles x G row groups (G % 8 == 0).  Block (qt, g) scans row tiles
// g, g+G, g+2G, ... for queries [qt*BM, qt*BM + BM) and leaves, per lane, the best
// kl (<= KC) of what it saw in cand[list][query][0..kl) with
// list = (g*WAVES_N + wn)*LPQ + part.
// Scores never leave the chip: each finished tile goes accumulator -> LDS (the stage
// buffer the last slice released) -> one lane per (query, part) scans its row against
// its register top-KC list; only beating the list tail costs an insertion.
// Scan geometry shared by the host plan and the device-count fallback (which picks it
// in-kernel from the failure count): nqt query tiles of BM, G row groups (a multiple of
// 8, <= the row tiles) so that about per_cu x CUs workgroups run.
struct ScanGeom {
  int nqt, G;
};
__host__ __device__ inline ScanGeom scan_geom(int64_t nq, int BM, int BN, int per_cu, int num_cus,
                                              int64_t n_rows) {
  ScanGeom g;
  g.nqt = (int)((nq + BM - 1) / BM);
  const int64_t ntiles = (n_rows + BN - 1) / BN;
  int64_t G = (int64_t)per_cu * num_cus / g.nqt;
  G = G < 1 ? 1 : G;
  G = G > ntiles ? ntiles : G;
  g.G = (int)((G + 7) / 8 * 8);
  return g;
}

template <class T, int KC>
__device__ __forceinline__ void flat_search_block(float* lds, const float* __restrict__ Q, int nq,
                                                  const float* __restrict__ C, int64_t n_rows,
                                                  int dim, int G, int nqt, int kl,
                                                  float* __restrict__ cand_s,
                                                  int* __restrict__ cand_i, int b) {
  using S = SearchSmem<T>;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;

  // blocks b and b+8 share an XCD: give the nqt query tiles of one row group to one
  // XCD so the second read of each row tile is an L2 hit.
  const int xcd = b & 7, slot = b >> 3;
  const int qt = slot % nqt, g = (slot / nqt) * 8 + xcd;
  const int m0 = qt * T::BM;
  const int64_t ntiles = (n_rows + T::BN - 1) / T::BN;
  const int q_local = lane % T::WM, part = lane / T::WM;

  TopList<KC> top;
  top.init();

  const int n_tiles = g < ntiles ? (int)((ntiles - g + G - 1) / G) : 0;
  auto coords = [&](int i, int& mm0, int64_t& n0) __attribute__((always_inline)) {
    mm0 = m0;
    n0 = (g + (int64_t)i * G) * T::BN;
  };
  // accumulator -> released stage buffer [WM][32] per wave per pass -> row scans
  // (always_inline: an outlined epilogue would take `top` and `acc` by address and
  // put both in scratch)
  auto epi = [&](int i, floatx16(&acc)[T::TM][T::TN], float* stage) __attribute__((always_inline)) {
    float* score = stage + wave * S::SCORE_FLOATS;
    const int64_t col0 = (g + (int64_t)i * G) * T::BN + wn * T::WN;
#pragma unroll
    for (int pass = 0; pass < T::TN * 32 / S::PASS_COLS; ++pass) {
      const int tn2 = pass * S::PASS_COLS / 32, sub = pass % (32 / S::PASS_COLS);
      if ((lane & 31) / S::PASS_COLS == sub) {
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            score[acc_row(tm, e, lane) * S::SCORE_STRIDE + (lane & 31) % S::PASS_COLS] = acc[tm][tn2][e];
      }
      __syncthreads();
      const float* row = score + q_local * S::SCORE_STRIDE + part * S::COLS;
      const int64_t c0 = col0 + pass * S::PASS_COLS + part * S::COLS;
#pragma unroll
      for (int c4 = 0; c4 < S::COLS; c4 += 4) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(row + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t col = c0 + c4 + e;
          if (col < n_rows && top.beats_tail(v[e], (int)col)) top.insert(v[e], (int)col);
        }
      }
      __syncthreads();
    }
  };
  walk_tiles<T>(lds, n_tiles, TileOperands{Q, dim, nq, C, dim, n_rows, dim}, coords, epi);

  const int list = (g * T::WAVES_N + wn) * S::LPQ + part;
  const int qg = m0 + wm * T::WM + q_local;
  if (qg < nq) {
    const int64_t base = ((int64_t)list * nq + qg) * kl;
#pragma unroll
    for (int i = 0; i < KC; ++i)
      if (i < kl) {
        cand_s[base + i] = top.s[i];
        cand_i[base + i] = top.id[i];
      }
  }
}

template <class T, int KC>
__global__ __launch_bounds__(256, KC <= 16 ? 2 : 1) void flat_search_kernel(
    const float* __restrict__ Q, int nq, const float* __restrict__ C, int64_t n_rows, int dim,
    int G, int nqt, int kl, float* __restrict__ cand_s, int* __restrict__ cand_i) {
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  flat_search_block<T, KC>(lds, Q, nq, C, n_rows, dim, G, nqt, kl, cand_s, cand_i, blockIdx.x);
}

// ============================================ K9s: streaming scan, few queries ==
// For a handful of queries the MFMA tiles above are mostly padding (32 query rows per
// tile) while the row stream is what bounds the scan, so small batches use a plain
// streaming dot-product kernel instead: 16 lanes per row (each 16-B load instruction
// of a wave covers four 256-B row segments), queries in LDS, two rows in flight per
// lane group, fp32 FMA, a 16-lane butterfly per (row, query), and lane j of the group
// keeps query j's register top list; the block merges its 16 groups' lists at the end.
// List = block: cand[block][query][0..kl).
// BF: the rows are the bf16 shadow (half the bytes; a 16-B load carries 8 elements, each
// widened exactly to fp32 and multiplied with the fp32 query) - the certified screen's
// single-query scan.
// MASKED (filtered search): row r is scored only when bit r % 32 of mask word r / 32 is
// set - the exact scan over the allowed rows with no gather of them.
constexpr int kStreamMaxNV = 16;  // 16-B loads per lane per row: dim <= 1024

template <int NQ, int KC, int NV, bool BF = false, bool MASKED = false>
__global__ __launch_bounds__(256) void stream_search_kernel(const float* __restrict__ Q, int nq,
                                                            const float* __restrict__ C,
                                                            int64_t n_rows, int dim, int kl,
                                                            float* __restrict__ cand_s,
                                                            int* __restrict__ cand_i,
                                                            const unsigned* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float qs[];  // [NQ][dim], zero padded
  const int tid = threadIdx.x, gl = tid & 15;
  for (int i = tid; i < NQ * dim; i += 256) {
    const int j = i / dim;
    qs[i] = j < nq ? Q[(int64_t)j * dim + (i - j * dim)] : 0.f;
  }
  __syncthreads();
  constexpr int EPV = BF ? 8 : 4;  // elements per 16-B load
  // NV < max: compiled for dim = 16 EPV NV
  const int nv = NV == kStreamMaxNV ? dim / (16 * EPV) : NV;
  const int row_words = BF ? dim / 2 : dim;  // row stride in 4-byte words
  const int64_t group = (int64_t)blockIdx.x * 16 + (tid >> 4);
  const int64_t n_groups = (int64_t)gridDim.x * 16;
  TopList<KC> top;
  top.init();
  const bool owner = gl < nq && gl < NQ;  // lane gl keeps query gl's list
  const float* qbase = qs + gl * EPV;

  auto score_rows = [&](const floatx4 (&v)[2][NV], int64_t r0, int nr, const unsigned (&mw)[2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float mine = 0.f;
      // one query at a time: 12 ds_read_b128 of its slice, 48 FMA, 16-lane butterfly
      constexpr int kUnrollQ = NQ <= 2 ? NQ : 1;
#pragma unroll kUnrollQ
      for (int j = 0; j < NQ; ++j) {
        const float* qj = qbase + j * dim;
        if constexpr (NQ > 2) asm volatile("" : "+v"(qj));
        float acc = 0.f;
#pragma unroll
        for (int it = 0; it < NV; ++it) {
          if (it < nv) {
            if constexpr (BF) {
              const floatx4 q0 = *reinterpret_cast<const floatx4*>(qj + it * 128);
              const floatx4 q1 = *reinterpret_cast<const floatx4*>(qj + it * 128 + 4);
              const unsigned w0 = __float_as_uint(v[u][it].x), w1 = __float_as_uint(v[u][it].y);
              const unsigned w2 = __float_as_uint(v[u][it].z), w3 = __float_as_uint(v[u][it].w);
              acc = fmaf(bf16_lo(w0), q0.x, fmaf(bf16_hi(w0), q0.y,
                    fmaf(bf16_lo(w1), q0.z, fmaf(bf16_hi(w1), q0.w, acc))));
              acc = fmaf(bf16_lo(w2), q1.x, fmaf(bf16_hi(w2), q1.y,
                    fmaf(bf16_lo(w3), q1.z, fmaf(bf16_hi(w3), q1.w, acc))));
            } else {
              const floatx4 qv = *reinterpret_cast<const floatx4*>(qj + it * 64);
              acc = fmaf(v[u][it].x, qv.x, fmaf(v[u][it].y, qv.y,
                    fmaf(v[u][it].z, qv.z, fmaf(v[u][it].w, qv.w, acc))));
            }
          }
        }
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
        mine = gl == j ? acc : mine;
      }
      const int64_t r = r0 + u * n_groups;
      const bool here = !MASKED || ((mw[u] >> (r & 31)) & 1u);
      if (u < nr && owner && here && top.beats_tail(mine, (int)r)) top.insert(mine, (int)r);
    }
  };

  for (int64_t r0 = group; r0 < n_rows; r0 += 2 * n_groups) {
    const int nr = r0 + n_groups < n_rows ? 2 : 1;
    floatx4 v[2][NV];
    unsigned mw[2] = {~0u, ~0u};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t r = u < nr ? r0 + u * n_groups : r0;
      const floatx4* rp = reinterpret_cast<const floatx4*>(C + r * row_words) + gl;
#pragma unroll
      for (int it = 0; it < NV; ++it)
        if (it < nv) v[u][it] = __builtin_nontemporal_load(rp + it * 16);
      if constexpr (MASKED) mw[u] = mask[r >> 5];
    }
    score_rows(v, r0, nr, mw);
  }
  // Block-level merge of the 16 lane groups' lists: one list per (block, query), so K10
  // merges 16x fewer lists (for a single query its 8192-list merge was 78 us).  Lists go
  // through LDS (the query image is dead by now); wave j % 4 merges query j: lane l folds
  // candidates l, l+64, ... into a register list, then kl wave arg-best rounds emit the
  // block's sorted list.  The K10 overflow check stays sound: a group list that dropped
  // a top-k member holds kl entries better than the k-th result, so the block list does.
  __syncthreads();
  float* lst_s = qs;                                       // [16][NQ][KC]
  int* lst_i = reinterpret_cast<int*>(qs + 16 * NQ * KC);  // [16][NQ][KC]
  if (owner) {
    const int g = tid >> 4;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      lst_s[(g * NQ + gl) * KC + i] = top.s[i];
      lst_i[(g * NQ + gl) * KC + i] = top.id[i];
    }
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  for (int j = wave; j < min(nq, NQ); j += 4) {
    TopList<KC> t;
    t.init();
    for (int c = lane; c < 16 * kl; c += 64) {
      const int g = c / kl, i = c - g * kl;
      const float x = lst_s[(g * NQ + j) * KC + i];
      const int xi = lst_i[(g * NQ + j) * KC + i];
      if (xi >= 0 && t.beats_tail(x, xi)) t.insert(x, xi);
    }
    const int64_t base = ((int64_t)blockIdx.x * nq + j) * kl;
    for (int r = 0; r < kl; ++r) {
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
      if (lane == 0) {
        cand_s[base + r] = bs;
        cand_i[base + r] = bi;
      }
      if (lane == bt && bi >= 0) t.pop_front();
    }
  }
}

// ================================================= bf16 coarse path (config 5) ==
// fp32 -> bf16 (round to nearest even), two elements per thread.
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src,
                                                      unsigned* __restrict__ dst, int64_t n_pairs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_pairs) return;
  const float2 v = reinterpret_cast<const float2*>(src)[i];
  dst[i] = pk_bf16(v.x, v.y);
}

// bf16 shadow of stored rows (same layout as to_bf16_kernel) plus the rounding
// statistics the certified screens need: max over rows of ||c - bf16(c)|| into stats[0]
// and of ||c|| into stats[1] (non-negative floats order like their bit patterns, so an
// unsigned atomicMax is a float max).  One wave per row.
__global__ __launch_bounds__(256) void bf16_shadow_kernel(const float* __restrict__ src,
                                                          unsigned* __restrict__ dst, int64_t n,
                                                          int dim, unsigned* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const floatx4* s = reinterpret_cast<const floatx4*>(src + row * dim);
  uint2* d = reinterpret_cast<uint2*>(dst + row * (dim / 2));
  float sd = 0.f, sc = 0.f;
  for (int i = lane; i < (dim >> 2); i += 64) {
    const floatx4 v = s[i];
    const unsigned a = pk_bf16(v.x, v.y), b = pk_bf16(v.z, v.w);
    d[i] = make_uint2(a, b);
    const float e0 = v.x - bf16_lo(a), e1 = v.y - bf16_hi(a);  // exact residuals
    const float e2 = v.z - bf16_lo(b), e3 = v.w - bf16_hi(b);
    sd += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
    sc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sd += __shfl_xor(sd, off);
    sc += __shfl_xor(sc, off);
  }
  if (lane == 0) {
    atomicMax(stats, __float_as_uint(sqrtf(sd)));
    atomicMax(stats + 1, __float_as_uint(sqrtf(sc)));
  }
}

// Results of a re-run subset back into the caller's [nq, k] outputs: row j -> idx[j].
__global__ __launch_bounds__(256) void scatter_results_kernel(const float* __restrict__ ss,
                                                              const int64_t* __restrict__ si,
                                                              const int64_t* __restrict__ idx,
                                                              int64_t n, int k, float* __restrict__ os,
                                                              int64_t* __restrict__ oi) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * k) return;
  const int64_t j = t / k, c = t - j * k;
  os[idx[j] * k + c] = ss[t];
  oi[idx[j] * k + c] = si[t];
}

// Certificate of the screened exact search (MQ_DTYPE_F32_SCREEN).  A screen scan kept
// the kc best rows of each query by its approximate score s, so a row r outside them
// has s_r <= s_kc; if every s is within E of the exact dot e, and e_k (the fp32 re-rank
// of the candidates, k-th best) is within its own rounding bound, then
// s_kc + E_total < e_k proves no outside row can enter the exact top-k.  E per mode:
//  VERIFY_X6 (split-f32 MFMA scan): dropped split terms < 3 2^-24 |q||c| per product,
//    fp32 accumulation over <= 64 x 6 MFMA steps: <= 2.5e-5 ||q|| for unit rows and
//    dim <= 1024; re-rank <= 18 roundings; E_total = 2 x 4e-5 ||q||.
//  VERIFY_BF16_Q16 (bf16 MFMA scan, query rounded to bf16 bq, row to bc):
//    |q.c - bq.bc| <= ||q - bq|| ||c|| + ||bq|| ||c - bc|| (Cauchy-Schwarz), fp32
//    accumulation <= g ||bq|| ||bc|| with g = 2 dim 2^-24, re-rank <= g ||q|| ||c||;
//    ||c|| <= cmax and ||c - bc|| <= dmax are the shadow's measured maxima (stats).
//  VERIFY_BF16_Q32 (bf16 rows streamed against the fp32 query): as above, ||q - bq|| = 0.
// A query that fails is appended to fail[] (count in *n_fail) and re-run one tier down.
// One wave per query.
enum { VERIFY_X6 = 0, VERIFY_BF16_Q16 = 1, VERIFY_BF16_Q32 = 2 };
constexpr int kNoPrune = -1;

// The screen's bound E on |screen score - exact fp32 dot| for query q (per mode, above),
// from wave-reduced ||q||^2, ||q - bq||^2, ||bq||^2 (Q16: bq = q rounded as
// to_bf16_kernel does).  Evaluated by one full wave; every lane returns E.
__device__ __forceinline__ float screen_bound(const float* __restrict__ Q, int dim, int64_t q,
                                              int mode, const unsigned* __restrict__ stats,
                                              int lane) {
  const floatx4* q4 = reinterpret_cast<const floatx4*>(Q + q * dim);
  float ss = 0.f, sd = 0.f, sb = 0.f;
  for (int i = lane; i < (dim >> 2); i += 64) {
    const floatx4 v = q4[i];
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    if (mode == VERIFY_BF16_Q16) {  // the same rounding as to_bf16_kernel
      const unsigned a = pk_bf16(v.x, v.y), b = pk_bf16(v.z, v.w);
      const float b0 = bf16_lo(a), b1 = bf16_hi(a), b2 = bf16_lo(b), b3 = bf16_hi(b);
      const float e0 = v.x - b0, e1 = v.y - b1, e2 = v.z - b2, e3 = v.w - b3;
      sd += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
      sb += b0 * b0 + b1 * b1 + b2 * b2 + b3 * b3;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    ss += __shfl_xor(ss, off);
    sd += __shfl_xor(sd, off);
    sb += __shfl_xor(sb, off);
  }
  const float qn = sqrtf(ss);
  if (mode == VERIFY_X6) return 8e-5f * qn;
  // 1.001: slack for the fp32 evaluation of the norms and of this bound
  const float dmax = __uint_as_float(stats[0]) * 1.001f, cmax = __uint_as_float(stats[1]) * 1.001f;
  const float g = 2.f * (float)dim * 5.9604645e-8f;
  const float dq = mode == VERIFY_BF16_Q16 ? sqrtf(sd) : 0.f;
  const float bqn = mode == VERIFY_BF16_Q16 ? sqrtf(sb) : qn;
  return (dq * cmax + bqn * dmax + g * bqn * (cmax + dmax) + g * qn * cmax) * 1.001f + 1e-7f;
}

// compact (optional, the asynchronous batch path): the failed query's vector is also
// copied to row `slot` of compact, the block the device re-run scans.
__global__ __launch_bounds__(256) void screen_verify_kernel(const float* __restrict__ Q, int dim,
                                                            const float* __restrict__ cs, int kc,
                                                            const float* __restrict__ es, int k,
                                                            int64_t nq, int mode,
                                                            const unsigned* __restrict__ stats,
                                                            int* __restrict__ n_fail,
                                                            int64_t* __restrict__ fail,
                                                            float* __restrict__ compact) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  const float E = screen_bound(Q, dim, q, mode, stats, lane);
  // cs_kc = -inf: the scan kept fewer than kc rows with tau = -inf, i.e. every row it
  // could see (a filter's allowed rows) is a candidate - the re-rank is the exact answer
  const float ckc = cs[q * kc + kc - 1];
  const bool failed = !(ckc + E < es[q * k + k - 1]) && ckc != -INFINITY;  // wave-uniform
  if (!failed) return;
  int slot = 0;
  if (lane == 0) {
    slot = atomicAdd(n_fail, 1);
    fail[slot] = q;
  }
  if (!compact) return;
  slot = __shfl(slot, 0);
  const floatx4* src = reinterpret_cast<const floatx4*>(Q + q * dim);
  floatx4* dst = reinterpret_cast<floatx4*>(compact + (int64_t)slot * dim);
  for (int i = lane; i < (dim >> 2); i += 64) dst[i] = src[i];
}

// Exact fp32 re-rank of the coarse candidates: one block per query, one wave per
// candidate dot product (768-wide, float4 per lane), then every candidate's rank by
// (score desc, id asc) picks its output slot.
// prune_mode (a VERIFY_* mode, or kNoPrune): with screen scores cs (sorted desc) and the
// screen's bound E, a candidate with cs < cs_k - 2E cannot be in the exact top-k (the k
// best screen scores are exact >= cs_k - E each, it is exact <= cs + E), so only the
// prefix cs >= cs_k - 2E is gathered and dotted (typically a handful of 64).
__global__ __launch_bounds__(256) void rerank_kernel(const float* __restrict__ Q,
                                                     const float* __restrict__ rows, int dim,
                                                     const int64_t* __restrict__ cand, int kc,
                                                     int k, float* __restrict__ out_s,
                                                     int64_t* __restrict__ out_i,
                                                     const float* __restrict__ cs, int prune_mode,
                                                     const unsigned* __restrict__ stats) {
  __shared__ float sc[MQ_MAX_K];
  __shared__ long long sid[MQ_MAX_K];
  __shared__ int n_live;
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const floatx4* q4 = reinterpret_cast<const floatx4*>(Q + q * dim);
  if (tid < kc) {
    sc[tid] = -INFINITY;
    sid[tid] = -1;
  }
  if (wave == 0) {
    int live = kc;
    if (prune_mode != kNoPrune && k < kc) {
      const float E = screen_bound(Q, dim, q, prune_mode, stats, lane);
      const float cut = cs[q * kc + k - 1] - 2.f * E;
      // candidates are sorted by screen score: the live ones are a prefix
      const bool keep = lane < kc && !(cs[q * kc + lane] < cut);
      live = __popcll(__ballot(keep)) + (kc > 64 ? kc - 64 : 0);
      live = max(live, k);
    }
    if (lane == 0) n_live = live;
  }
  __syncthreads();
  const int kl = n_live;
  // eight candidates per wave per round, all their row loads in flight together (the
  // gathered rows come from HBM: the round is latency-bound)
  constexpr int U = 8;
  const int slot = rerank_slot(lane);
  for (int c0 = wave * U; c0 < kl; c0 += 4 * U) {
    long long id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) id[u] = c0 + u < kl ? cand[q * kc + c0 + u] : -1;
    const float dot = rerank_dots8(q4, rows, dim, id, lane);
    long long my_id = id[0];
#pragma unroll
    for (int u = 1; u < U; ++u) my_id = slot == u ? id[u] : my_id;
    if ((lane & 7) == 0 && c0 + slot < kl) {
      sc[c0 + slot] = my_id >= 0 ? dot : -INFINITY;
      sid[c0 + slot] = my_id;
    }
  }
  // every slot starts as padding: the padding candidates (id -1, fewer real candidates than
  // k - a filter admitting few rows, or k > kc) all rank alike and write no slot below
  if (tid < k) {
    out_s[q * k + tid] = -INFINITY;
    out_i[q * k + tid] = -1;
  }
  __syncthreads();
  if (tid < kc && sid[tid] >= 0) {
    int rank = 0;
    for (int u = 0; u < kc; ++u) rank += better(sc[u], sid[u], sc[tid], sid[tid]) ? 1 : 0;
    if (rank < k) {
      out_s[q * k + rank] = sc[tid];
      out_i[q * k + rank] = sid[tid];
    }
  }
}

#ifndef MQ_FIN_DBG  // measurement builds only (wrong results): 1 = no survivor ranking, 2 = no re-rank gathers,
                    // 4 = return at once, 8 = no survivors loaded, 16 = phase times (printf, 100 MHz ticks)
#define MQ_FIN_DBG 0
#endif
#if MQ_FIN_DBG != 0 && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_FIN_DBG computes wrong results: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
#endif
// rank of (x, xi) by (score desc, id asc) among n4 * 4 LDS entries (vs, vi): float4 /
// int4 reads, unrolled so the reads pipeline (an early-exit scalar loop paid the LDS
// latency per entry: ~38 us for 320 survivors)
__device__ __forceinline__ int lds_rank4(const floatx4* vs, const int4* vi, int n4, float x, int xi) {
  int r = 0;
#pragma unroll 4
  for (int j = 0; j < n4; ++j) {
    const floatx4 a = vs[j];
    const int4 b = vi[j];
    r += (a.x > x || (a.x == x && b.x < xi)) + (a.y > x || (a.y == x && b.y < xi)) +
         (a.z > x || (a.z == x && b.z < xi)) + (a.w > x || (a.w == x && b.w < xi));
  }
  return r;
}

// order-preserving float <-> unsigned (key 0 is below every float)
__device__ __forceinline__ unsigned fin_ord(float x) {
  const unsigned b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fin_unord(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

constexpr int kScreenMaxK = 16;  // screened (certified) searches: k <= 16
constexpr int kFinW = 8, kFinT = 64 * kFinW;  // K9q finish: 8 waves, 64 re-rank gathers per round
constexpr int kFinMaxSurv = 1024;  // survivors the finish ranks (more: the query is passed down)
constexpr int kFinLive = 512;      // live candidates it re-ranks (more: passed down)
// K9q finish, one block per query (the single-query int8 screen, fused to save launches
// on the latency path).  The threshold scan kept every row whose screen score s clears
// tau (count[q] of them, at most kTsCap stored).  The screen's error on row r is bounded
// by E_r (the VERIFY_BF16_Q32 form of screen_bound with the row's own int8 error
// ||c_r - scale_r r8_r|| in place of the shadow's maximum; E >= every E_r is the global
// form):
//  * lo_r = s_r - E_r <= exact_r <= s_r + E_r = hi_r; with L_k the k-th largest lo among
//    the survivors, k survivors have exact >= L_k, so a survivor with hi_r < L_k cannot
//    reach the exact top-k: only the live survivors hi_r >= L_k are re-ranked in fp32 (as
//    rerank_kernel: same dot arithmetic), and their top-k by (score desc, id asc) is the
//    answer among the survivors (the per-row bound keeps ~half the live rows of the r5
//    global s >= cs_k - 2E rule on isotropic data: fewer gather rounds);
//  * a row that did not survive has s < tau, exact < tau + E: the answer is certified
//    when tau + E < e_k (the k-th exact score), with every survivor kept and ranked and
//    every live one re-ranked.
// The certificate is against tau itself, not the 64th-best survivor (r4): on a clustered
// corpus the query's cluster-mates crowd the top 64 screen scores within the int8 bound,
// while tau - set by the scan from the sample pass (i8_thresh_kernel: at most the k-th
// best sample - 2E) - sits below e_k - E.
__global__ __launch_bounds__(kFinT) void i8_finish_kernel(const float* __restrict__ Q,
                                                        const float* __restrict__ rows, int dim,
                                                        const float* __restrict__ ts_cs,
                                                        const int* __restrict__ ts_ci,
                                                        const int* __restrict__ count, int lists,
                                                        const float* __restrict__ tau, int k,
                                                        const unsigned* __restrict__ stats,
                                                        const float* __restrict__ err8,
                                                        float* __restrict__ os, int64_t* __restrict__ oi,
                                                        int* __restrict__ n_fail,
                                                        int64_t* __restrict__ fail) {
  // lo / li and sc / sid are padded to a multiple of 4 with (-inf, INT_MAX), never better
  // than a real entry: the rank counts read them as float4 / int4 (lds_rank4)
  __shared__ float ls[kFinMaxSurv];  // hi_r
  __shared__ floatx4 lo4[kFinMaxSurv / 4];
  __shared__ int4 li4[kFinMaxSurv / 4];
  __shared__ floatx4 sc4[kFinLive / 4];
  __shared__ int4 sid4[kFinLive / 4];
  __shared__ int lv[kFinLive];
  __shared__ unsigned long long wk[kFinW * kScreenMaxK];
  float* lo = reinterpret_cast<float*>(lo4);
  int* li = reinterpret_cast<int*>(li4);
  float* sc = reinterpret_cast<float*>(sc4);
  int* sid = reinterpret_cast<int*>(sid4);
  __shared__ float e_sh, qn_sh, ek_sh, lk_sh;
  __shared__ int nlive_sh, ovf_sh;
  __shared__ int wsum[kFinW];
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if MQ_FIN_DBG & 16
  unsigned long long tsx[8];
  tsx[0] = wall_clock64();
#define MQ_FIN_TS(i) tsx[i] = wall_clock64()
#else
#define MQ_FIN_TS(i)
#endif
  if (MQ_FIN_DBG & 4) {
    if (tid == 0) fail[atomicAdd(n_fail, 1)] = q;
    return;
  }
  // the survivors' segments (one per scan workgroup, thresh.hpp kI8Seg): thread t owns
  // segments t and t + kFinT; an exclusive scan of their counts places them
  static_assert(kI8MaxLists <= 2 * kFinT, "two segments per thread");
  int c0 = 0, c1 = 0;
  if (!(MQ_FIN_DBG & 8)) {
    c0 = tid < lists ? count[q * lists + tid] : 0;
    c1 = tid + kFinT < lists ? count[q * lists + tid + kFinT] : 0;
  }
  const bool seg_ovf = c0 > kI8Seg || c1 > kI8Seg;
  c0 = min(c0, kI8Seg);
  c1 = min(c1, kI8Seg);
  int incl = c0 + c1;  // inclusive scan: waves, then the wave totals
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  if (tid == 0) ovf_sh = 0;
  __syncthreads();
  if (seg_ovf) ovf_sh = 1;
  int base = 0;
#pragma unroll
  for (int w = 0; w < kFinW; ++w) base += w < wave ? wsum[w] : 0;
  int total = 0;
#pragma unroll
  for (int w = 0; w < kFinW; ++w) total += wsum[w];
  const int beg = base + incl - c0 - c1;
  __syncthreads();
  const bool ranked = total <= kFinMaxSurv && ovf_sh == 0;  // block-uniform
  const int cnt = ranked ? total : 0;
  if (wave == 0) {  // ||q|| and the global bound
    const floatx4* q4 = reinterpret_cast<const floatx4*>(Q + q * dim);
    float ss = 0.f;
    for (int i = lane; i < (dim >> 2); i += 64) {
      const floatx4 v = q4[i];
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    const float E = screen_bound(Q, dim, q, VERIFY_BF16_Q32, stats, lane);
    if (lane == 0) {
      e_sh = E;
      qn_sh = sqrtf(ss);
      ek_sh = -INFINITY;
      lk_sh = -INFINITY;
      nlive_sh = 0;
    }
  }
  __syncthreads();
  MQ_FIN_TS(1);
  {
    // E_r as screen_bound forms E, with d = ||c_r - scale_r r8_r|| (x 1.001 slack, as the maxima)
    const float qn = qn_sh, cmax = __uint_as_float(stats[1]) * 1.001f;
    const float g = 2.f * (float)dim * 5.9604645e-8f;
    for (int j = 0; ranked && j < c0 + c1; ++j) {
      const int64_t at = (q * lists + (j < c0 ? tid : tid + kFinT)) * kI8Seg + (j < c0 ? j : j - c0);
      const float x = ts_cs[at];
      const int xi = ts_ci[at];
      const float d = err8[xi] * 1.001f;
      const float Er = (qn * d + g * qn * (cmax + d) + g * qn * cmax) * 1.001f + 1e-7f;
      lo[beg + j] = x - Er;
      ls[beg + j] = x + Er;
      li[beg + j] = xi;
    }
    if (tid < ((cnt + 3) & ~3) - cnt) {
      lo[cnt + tid] = -INFINITY;
      li[cnt + tid] = INT_MAX;
    }
  }
  __syncthreads();
  MQ_FIN_TS(2);
  // L_k: the survivor of rank k - 1 by (lo desc, id asc).  Each wave pops its k best
  // (lanes hold survivors tid and tid + kFinT, keys (ord(lo), ~id): larger is better, all
  // distinct), then the 8k wave winners are ranked against each other (the all-pairs rank
  // of every survivor cost ~13 us at 320).  Fewer than k survivors leave -inf (every
  // survivor live, and the certificate fails below)
  if (!(MQ_FIN_DBG & 1)) {
    auto fkey = [&](int i) -> unsigned long long {
      return i < cnt ? ((unsigned long long)fin_ord(lo[i]) << 32) | (unsigned)~li[i] : 0ull;
    };
    unsigned long long a = fkey(tid), b = fkey(tid + kFinT);
    if (b > a) {
      const unsigned long long t = a;
      a = b;
      b = t;
    }
    for (int r = 0; r < k; ++r) {
      const unsigned hi = wave_max_u32((unsigned)(a >> 32));
      const unsigned lw = wave_max_u32((unsigned)(a >> 32) == hi ? (unsigned)a : 0u);
      const unsigned long long m = ((unsigned long long)hi << 32) | lw;
      if (lane == 0) wk[wave * k + r] = m;
      if (a == m && m != 0ull) {
        a = b;
        b = 0ull;
      }
    }
  }
  __syncthreads();
  if (tid < kFinW * k) {
    const unsigned long long x = wk[tid];
    int rank = 0;
#pragma unroll 4
    for (int j = 0; j < kFinW * k; ++j) rank += wk[j] > x ? 1 : 0;
    if (rank == k - 1 && x != 0ull) lk_sh = fin_unord((unsigned)(x >> 32));
  }
  __syncthreads();
  MQ_FIN_TS(3);
  const float lk = lk_sh;
  for (int i = tid; i < cnt; i += kFinT)
    if (!(ls[i] < lk)) {
      const int j = atomicAdd(&nlive_sh, 1);
      if (j < kFinLive) lv[j] = i;
    }
  __syncthreads();
  MQ_FIN_TS(4);
  const int nl = min(nlive_sh, kFinLive);
  if (tid < ((nl + 3) & ~3) - nl) {
    sc[nl + tid] = -INFINITY;
    sid[nl + tid] = INT_MAX;
  }
  const floatx4* q4 = reinterpret_cast<const floatx4*>(Q + q * dim);
  constexpr int U = 8;  // eight candidates per wave per round (rerank_kernel's arithmetic): 64 per round
  const int slot = rerank_slot(lane);
  for (int c0 = wave * U; c0 < nl; c0 += kFinW * U) {
    long long id[U];
#pragma unroll
    for (int u = 0; u < U; ++u) id[u] = c0 + u < nl ? li[lv[c0 + u]] : -1;
    const float dot = (MQ_FIN_DBG & 2) ? 0.f : rerank_dots8(q4, rows, dim, id, lane);
    long long my_id = id[0];
#pragma unroll
    for (int u = 1; u < U; ++u) my_id = slot == u ? id[u] : my_id;
    if ((lane & 7) == 0 && c0 + slot < nl) {
      sc[c0 + slot] = dot;  // (the live ids are real rows)
      sid[c0 + slot] = (int)my_id;
    }
  }
  __syncthreads();
  MQ_FIN_TS(5);
  for (int t = tid; t < nl; t += kFinT) {
    const int rank = lds_rank4(sc4, sid4, (nl + 3) >> 2, sc[t], sid[t]);
    if (rank < k) {
      os[q * k + rank] = sc[t];
      oi[q * k + rank] = sid[t];
      if (rank == k - 1) ek_sh = sc[t];
    }
  }
  if (tid >= nl && tid < k) {  // fewer live rows than k: padding (and no certificate)
    os[q * k + tid] = -INFINITY;
    oi[q * k + tid] = -1;
  }
  __syncthreads();
  MQ_FIN_TS(6);
  if (tid == 0) {
    // fewer than k live rows: exact only when tau = -inf (every row the scan saw survived:
    // a filter admitting fewer than k rows) - the padded answer is then the whole set
    const bool cert = ranked && nlive_sh <= kFinLive &&
                      (nl >= k ? tau[q] + e_sh < ek_sh : tau[q] == -INFINITY);
    if (!cert) fail[atomicAdd(n_fail, 1)] = q;
#if MQ_FIN_DBG & 16
    printf("FIN cnt %d nl %d dt %llu %llu %llu %llu %llu %llu\n", cnt, nl, tsx[1] - tsx[0], tsx[2] - tsx[1],
           tsx[3] - tsx[2], tsx[4] - tsx[3], tsx[5] - tsx[4], tsx[6] - tsx[5]);
#endif
  }
#undef MQ_FIN_TS
}

// ======================================================= K10: merge lists ======
// One block per query.  Each list is sorted, so a thread walks its share of the lists
// (lists tid, tid+256, ...) reading heads in batches of 8 independent loads, and only
// a head that beats its register top-KC tail pulls further entries of that list.
// Then every wave pops its 64 lanes' best k_out (shuffle arg-best, no block barrier),
// and the 4*k_out wave winners are ranked against each other in LDS to place them.
// Overflow checks (results stay exact; the caller re-runs on a set bit):
//  bit 0 (list_kc < k_out, the scan kept only list_kc entries per list): a list whose
//        last kept entry beats the final k_out-th result may have dropped a member of
//        the top-k -> re-scan with full-length lists.  Unfilled lists hold padding.
//  bit 1 (KC < k_out, 16-entry thread lists for large k): same test on each thread's
//        register list -> re-run only this merge with KC = 64.
template <int KC, typename IdIn>
__device__ __forceinline__ void merge_threadlists(const float* __restrict__ cs,
                                                  const IdIn* __restrict__ ci, int n_lists,
                                                  int64_t nq, int k_in, int k_out,
                                                  float* __restrict__ out_s,
                                                  int64_t* __restrict__ out_i, int list_kc,
                                                  int* __restrict__ overflow, int64_t q) {
  constexpr int U = 8;
  __shared__ float ws[4 * MQ_MAX_K];
  __shared__ long long wi[4 * MQ_MAX_K];
  __shared__ float kth_s;
  __shared__ long long kth_i;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // local lists hold int ids; shard-merge ids are int64 -> use a 64-bit twin list
  float ls[KC];
  long long li[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    ls[i] = -INFINITY;
    li[i] = -1;
  }
  auto push = [&](float x, long long xi) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const bool sw = better(x, xi, ls[i], li[i]);
      const float ts = ls[i];
      const long long ti = li[i];
      ls[i] = sw ? x : ts;
      li[i] = sw ? xi : ti;
      x = sw ? ts : x;
      xi = sw ? ti : xi;
    }
  };
  for (int l0 = tid; l0 < n_lists; l0 += 256 * U) {
    float hs[U];
    long long hi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int lst = l0 + 256 * u;
      hs[u] = -INFINITY;
      hi[u] = -1;
      if (lst < n_lists) {
        const int64_t off = ((int64_t)lst * nq + q) * k_in;
        hs[u] = cs[off];
        hi[u] = (long long)ci[off];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (hi[u] < 0 || !better(hs[u], hi[u], ls[KC - 1], li[KC - 1])) continue;
      push(hs[u], hi[u]);
      const int64_t off = ((int64_t)(l0 + 256 * u) * nq + q) * k_in;
      // rest of the sorted list while it still beats the tail, 8 entries per round of
      // independent loads (one dependent load per entry was ~2/3 of the k_out = 64 merge)
      for (int kk0 = 1; kk0 < k_in; kk0 += U) {
        float xs[U];
        long long xis[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const bool in = kk0 + j < k_in;
          xs[j] = in ? cs[off + kk0 + j] : -INFINITY;
          xis[j] = in ? (long long)ci[off + kk0 + j] : -1;
        }
        bool stop = false;
#pragma unroll
        for (int j = 0; j < U; ++j) {
          stop = stop || xis[j] < 0 || !better(xs[j], xis[j], ls[KC - 1], li[KC - 1]);
          if (!stop) push(xs[j], xis[j]);
        }
        if (stop) break;
      }
    }
  }
  // thread-list overflow (KC < k_out): remember this thread's KC-th entry
  const float tail_s = ls[KC - 1];
  const long long tail_i = li[KC - 1];
  // per-wave arg-best rounds: wave winners in order into ws/wi[wave * k_out + r]
  for (int r = 0; r < k_out; ++r) {
    float bs = ls[0];
    long long bi = li[0];
    int bt = lane;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off);
      const long long oi = __shfl_xor(bi, off);
      const int ot = __shfl_xor(bt, off);
      if (better(os, oi, bs, bi)) {
        bs = os;
        bi = oi;
        bt = ot;
      }
    }
    if (lane == 0) {
      ws[wave * k_out + r] = bs;
      wi[wave * k_out + r] = bi;
    }
    if (lane == bt && bi >= 0) {  // pop this lane's head
#pragma unroll
      for (int i = 0; i + 1 < KC; ++i) {
        ls[i] = ls[i + 1];
        li[i] = li[i + 1];
      }
      ls[KC - 1] = -INFINITY;
      li[KC - 1] = -1;
    }
  }
  if (tid == 0) {
    kth_s = -INFINITY;
    kth_i = -1;
  }
  __syncthreads();
  // rank the 4*k_out wave winners; valid ids are distinct, so valid ranks are too
  const int nc = 4 * k_out;
  for (int c = tid; c < nc; c += 256) {
    const float x = ws[c];
    const long long xi = wi[c];
    if (xi < 0) continue;
    int rank = 0;
    for (int u = 0; u < nc; ++u) rank += (wi[u] >= 0 && better(ws[u], wi[u], x, xi)) ? 1 : 0;
    if (rank < k_out) {
      out_s[q * k_out + rank] = x;
      out_i[q * k_out + rank] = xi;
      if (rank == k_out - 1) {
        kth_s = x;
        kth_i = xi;
      }
    }
  }
  // padding past the valid results
  int nvalid = 0;
  for (int u = 0; u < nc; ++u) nvalid += wi[u] >= 0 ? 1 : 0;
  for (int r = nvalid + tid; r < k_out; r += 256) {
    out_s[q * k_out + r] = -INFINITY;
    out_i[q * k_out + r] = -1;
  }
  if (KC < k_out) {
    // a thread holding KC entries that all beat the k_out-th result may have dropped
    // more: bit 1 asks the caller to re-run the merge with 64-entry thread lists
    __syncthreads();
    if (overflow && tail_i >= 0 && better(tail_s, tail_i, kth_s, kth_i)) atomicOr(overflow, 2);
  }
  if (overflow && list_kc < k_out) {
    __syncthreads();
    // entries a full list dropped are worse than its last kept one: only a last entry
    // strictly better than the k_out-th result (or any full list, when fewer than k_out
    // results exist) can hide a member of the top-k
    for (int lst = tid; lst < n_lists; lst += 256) {
      const int64_t off = ((int64_t)lst * nq + q) * k_in + (list_kc - 1);
      const long long xi = (long long)ci[off];
      if (xi >= 0 && better(cs[off], xi, kth_s, kth_i)) atomicOr(overflow, 1);
    }
  }
}

template <int KC, typename IdIn>
__global__ __launch_bounds__(256) void merge_kernel(const float* __restrict__ cs,
                                                    const IdIn* __restrict__ ci, int n_lists,
                                                    int64_t nq, int k_in, int k_out,
                                                    float* __restrict__ out_s,
                                                    int64_t* __restrict__ out_i, int list_kc,
                                                    int* __restrict__ overflow) {
  merge_threadlists<KC, IdIn>(cs, ci, n_lists, nq, k_in, k_out, out_s, out_i, list_kc, overflow,
                              blockIdx.x);
}

// K10 (threshold form, the default): one block per query.  T = the largest score such
// that at least k_out list HEADS score >= T (a 32-step bitwise search on order-
// preserving keys, heads held in registers); any entry scoring below T has k_out
// strictly better heads, so the top-k_out are among the entries >= T.  Those survivors
// (each sorted list walked while >= T; typically ~k_out of them) are gathered in LDS and
// ranked exactly by (score desc, id asc).  Same results and overflow bit 0 as the
// thread-list merge, which it falls back to (block-uniform) when n_lists > 4096 or more
// than kSelCap entries tie at or above T.
constexpr int kSelCap = 2048;
constexpr int kSelHeads = 16;  // heads per thread: n_lists <= 4096

__device__ __forceinline__ unsigned score_key(float x) {  // order-preserving, > 0
  const unsigned b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

template <int KC, typename IdIn>
__device__ __forceinline__ void merge_select_block(const float* __restrict__ cs,
                                                   const IdIn* __restrict__ ci, int n_lists,
                                                   int64_t nq, int k_in, int k_out,
                                                   float* __restrict__ out_s,
                                                   int64_t* __restrict__ out_i, int list_kc,
                                                   int* __restrict__ overflow, int64_t q) {
  constexpr int U = 8;
  __shared__ float ss[kSelCap];
  __shared__ long long si[kSelCap];
  __shared__ int part[4];
  __shared__ int n_s;
  __shared__ float kth_s;
  __shared__ long long kth_i;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (n_lists > 256 * kSelHeads) {
    merge_threadlists<KC, IdIn>(cs, ci, n_lists, nq, k_in, k_out, out_s, out_i, list_kc, overflow, q);
    return;
  }
  unsigned key[kSelHeads];
#pragma unroll
  for (int j = 0; j < kSelHeads; ++j) {
    const int lst = tid + 256 * j;
    key[j] = 0;  // absent list / padding entry
    if (lst < n_lists) {
      const int64_t off = ((int64_t)lst * nq + q) * k_in;
      if ((long long)ci[off] >= 0) key[j] = score_key(cs[off]);
    }
  }
  // Per wave: Tw = the largest key with at least k_out of the WAVE's heads >= Tw (bitwise
  // search, ballot counts, no block barrier); T = max over the 4 waves still has k_out
  // heads >= T (all in one wave), so it is a valid threshold, for 62 fewer barriers.
  // Survivors are usually a few times the block-wide k_out-th head's, but nothing bounds
  // them: when no single wave holds k_out valid heads (many empty lists) T = 0 and every
  // valid entry is admitted; past kSelCap the block falls back to the thread-list merge
  // below, so results stay exact either way.
  const int jn = min(kSelHeads, (n_lists + 255) / 256);  // head slots in use
  unsigned T = 0;
  for (int b = 31; b >= 0; --b) {
    const unsigned cand = T | (1u << b);
    int c = 0;
#pragma unroll
    for (int j = 0; j < kSelHeads; ++j)
      if (j < jn) c += __popcll(__ballot(key[j] >= cand));  // jn is block-uniform
    if (c >= k_out) T = cand;
  }
  if (lane == 0) part[wave] = (int)T;
  __syncthreads();
  T = max(max((unsigned)part[0], (unsigned)part[1]), max((unsigned)part[2], (unsigned)part[3]));
  const unsigned adm = T > 1u ? T : 1u;  // fewer than k_out valid heads: every valid entry
  if (tid == 0) {
    n_s = 0;
    kth_s = -INFINITY;
    kth_i = -1;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSelHeads; ++j) {
    if (key[j] < adm) continue;
    const int64_t off = ((int64_t)(tid + 256 * j) * nq + q) * k_in;
    for (int kk0 = 0; kk0 < k_in; kk0 += U) {
      float xs[U];
      long long xis[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = kk0 + u < k_in;
        xs[u] = in ? cs[off + kk0 + u] : -INFINITY;
        xis[u] = in ? (long long)ci[off + kk0 + u] : -1;
      }
      bool stop = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        stop = stop || xis[u] < 0 || score_key(xs[u]) < adm;
        if (!stop) {
          const int pos = atomicAdd(&n_s, 1);
          if (pos < kSelCap) {
            ss[pos] = xs[u];
            si[pos] = xis[u];
          }
        }
      }
      if (stop) break;
    }
  }
  __syncthreads();
  const int ns = n_s;
  if (ns > kSelCap) {  // massive ties at the threshold: the thread-list merge handles them
    merge_threadlists<KC, IdIn>(cs, ci, n_lists, nq, k_in, k_out, out_s, out_i, list_kc, overflow, q);
    return;
  }
  // rank the survivors; valid ids are distinct, so the ranks are too
  for (int c = tid; c < ns; c += 256) {
    const float x = ss[c];
    const long long xi = si[c];
    int rank = 0;
    for (int u = 0; u < ns; ++u) rank += better(ss[u], si[u], x, xi) ? 1 : 0;
    if (rank < k_out) {
      out_s[q * k_out + rank] = x;
      out_i[q * k_out + rank] = xi;
      if (rank == k_out - 1) {
        kth_s = x;
        kth_i = xi;
      }
    }
  }
  for (int r = ns + tid; r < k_out; r += 256) {  // padding past the valid results
    out_s[q * k_out + r] = -INFINITY;
    out_i[q * k_out + r] = -1;
  }
  if (overflow && list_kc < k_out) {
    __syncthreads();
    // as in merge_threadlists: a full list whose last kept entry beats the k_out-th
    // result (or any full list, when fewer than k_out results exist) may hide a member
    for (int lst = tid; lst < n_lists; lst += 256) {
      const int64_t off = ((int64_t)lst * nq + q) * k_in + (list_kc - 1);
      const long long xi = (long long)ci[off];
      if (xi >= 0 && better(cs[off], xi, kth_s, kth_i)) atomicOr(overflow, 1);
    }
  }
}

template <int KC, typename IdIn>
__global__ __launch_bounds__(256) void merge_select_kernel(const float* __restrict__ cs,
                                                           const IdIn* __restrict__ ci, int n_lists,
                                                           int64_t nq, int k_in, int k_out,
                                                           float* __restrict__ out_s,
                                                           int64_t* __restrict__ out_i, int list_kc,
                                                           int* __restrict__ overflow) {
  merge_select_block<KC, IdIn>(cs, ci, n_lists, nq, k_in, k_out, out_s, out_i, list_kc, overflow,
                               blockIdx.x);
}

// ---------------------------------------------- asynchronous screen fallback ------
// The batched certified screen (TIER_BF16) does not read its failure count back to the
// host.  screen_verify_kernel copies each uncertified query into a compact block as it
// lists it, and two kernels are enqueued behind it every time, both returning at once
// when *n_fail == 0: fallback_search_kernel re-runs ALL nf failed queries in one pass over
// the slab on the exact-f32 MFMA tile (the direct scan's K9 body) - the query count is
// read on the device, so the tile shape and the grid are picked in-kernel from nf (the
// narrow 32-query tile for nf <= 64, the wide 128-query tile above, exactly as
// plan_search would for a batch of nf) over a grid launched for the worst case, whose
// surplus workgroups return at once - and fallback_merge_kernel merges each failed
// query's lists (K10) and writes its row in place into the caller's outputs.  Cost: one
// direct exact scan of nf queries (r3's VALU fallback made one slab pass per 4 queries).
constexpr int kFbNarrowMax = 64;  // nf <= this: narrow tile (plan_search's `wide = nq > 64`)

template <int KC>
__global__ __launch_bounds__(256, KC <= 16 ? 2 : 1) void fallback_search_kernel(
    const float* __restrict__ Qc, const int* __restrict__ n_fail, const float* __restrict__ C,
    int64_t n_rows, int dim, int num_cus, int kl, float* __restrict__ cand_s,
    int* __restrict__ cand_i) {
  constexpr int kLds = 2 * (SearchWide::STAGE_FLOATS > SearchNarrow::STAGE_FLOATS ? SearchWide::STAGE_FLOATS
                                                                                     : SearchNarrow::STAGE_FLOATS);
  __shared__ __attribute__((aligned(16))) float lds[kLds];
  const int nf = __builtin_amdgcn_readfirstlane(*n_fail);
  if (nf == 0) return;
  constexpr int per_cu = KC <= 16 ? 2 : 1;
  if (nf > kFbNarrowMax) {
    const ScanGeom g = scan_geom(nf, SearchWide::BM, SearchWide::BN, per_cu, num_cus, n_rows);
    if ((int)blockIdx.x >= g.G * g.nqt) return;  // workgroup-uniform
    flat_search_block<SearchWide, KC>(lds, Qc, nf, C, n_rows, dim, g.G, g.nqt, kl, cand_s, cand_i, blockIdx.x);
  } else {
    const ScanGeom g = scan_geom(nf, SearchNarrow::BM, SearchNarrow::BN, per_cu, num_cus, n_rows);
    if ((int)blockIdx.x >= g.G * g.nqt) return;
    flat_search_block<SearchNarrow, KC>(lds, Qc, nf, C, n_rows, dim, g.G, g.nqt, kl, cand_s, cand_i, blockIdx.x);
  }
}

// One block per possible failure slot j (grid = the batch size): blocks j >= *n_fail
// return; block j merges the lists of compact query j (= fail[j]) into the outputs' row
// fail[j].  Block 0 adds the count to the index's cumulative fallback counter.
template <int KC, int SCAN_KC>
__global__ __launch_bounds__(256) void fallback_merge_kernel(const float* __restrict__ cs,
                                                             const int* __restrict__ ci, int num_cus,
                                                             int64_t n_rows, int k, int kl,
                                                             const int* __restrict__ n_fail,
                                                             const int64_t* __restrict__ fail,
                                                             float* __restrict__ os,
                                                             int64_t* __restrict__ oi,
                                                             unsigned long long* __restrict__ total) {
  const int nf = __builtin_amdgcn_readfirstlane(*n_fail);
  const int64_t j = blockIdx.x;
  if (j == 0 && threadIdx.x == 0 && nf > 0) atomicAdd(total, (unsigned long long)nf);
  if (j >= nf) return;
  constexpr int per_cu = SCAN_KC <= 16 ? 2 : 1;
  int n_lists;
  if (nf > kFbNarrowMax) {
    const ScanGeom g = scan_geom(nf, SearchWide::BM, SearchWide::BN, per_cu, num_cus, n_rows);
    n_lists = g.G * SearchWide::WAVES_N * SearchSmem<SearchWide>::LPQ;
  } else {
    const ScanGeom g = scan_geom(nf, SearchNarrow::BM, SearchNarrow::BN, per_cu, num_cus, n_rows);
    n_lists = g.G * SearchNarrow::WAVES_N * SearchSmem<SearchNarrow>::LPQ;
  }
  const int64_t shift = (fail[j] - j) * k;  // the block writes row j of (os + shift) = row fail[j]
  merge_select_block<KC, int>(cs, ci, n_lists, nf, kl, k, os + shift, oi + shift, kl, nullptr, j);
}

}  // namespace mq

// ================================================================ host side =====
using namespace mq;

namespace {

// Grow-only device workspace.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return MQ_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, need) != hipSuccess) MQ_FAIL(MQ_ENOMEM, "hipMalloc(%zu bytes) failed", need);
    bytes = need;
    return MQ_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// register list lengths: the fused scan keeps 8 or 16 entries per lane (k > 16 runs
// with 16 + the merge's overflow check, re-running with 64 only when it fires); the
// merge keeps up to 64 per thread
int kc_scan(int k) { return k <= 8 ? 8 : 16; }
int kc_merge(int k) { return k <= 8 ? 8 : (k <= 16 ? 16 : 64); }

}  // namespace

struct mq_index {
  int device = 0;
  int dim = 0;
  int dtype = MQ_DTYPE_F32;
  int64_t n = 0;    // rows stored
  int64_t cap = 0;  // rows reserved
  float* rows = nullptr;  // [cap, dim], every stored row unit-norm
  int num_cus = 256;
  int* host_flag = nullptr;  // pinned: the status word a search reads back (a pageable
                             // 4-byte D2H copy is staged and costs more than the scan tail)
  DevBuf stage, cand_s, cand_i, out_s, out_i;
  DevBuf sel;  // device copy of a mq_index_select row list
  DevBuf rows16;     // bf16 shadow of `rows` for the coarse path ([cap, dim] bf16)
  int64_t n16 = 0;   // rows already mirrored into rows16
  DevBuf stats16;    // shadow rounding maxima: [0] max ||c - bf16(c)||, [1] max ||c|| (float bits)
  DevBuf q16, coarse_s, coarse_i;
  DevBuf fb_cs, fb_ci;  // coarse candidates of the bf16-mode queries re-run on the tiled scan
  DevBuf flag;          // merge overflow flag (k > 16) / screen failure count
  DevBuf tier_fail[4], tier_q[4], tier_s[4], tier_i[4];  // per screen tier: re-run subset
  int64_t rescans = 0;   // searches re-run with 64-entry scan lists
  int64_t remerges = 0;  // merges re-run with 64-entry thread lists
  int64_t screen_fallbacks = 0;  // screened queries re-run on the direct exact scan
  int64_t screen_passdowns = 0;  // bf16-screened queries re-run on the split-f32 screen
  int stream_max_q = 4;  // batches up to this size use the streaming kernel (K9s)
  bool thresh_scan = true;  // batched bf16 screens use the threshold scan (K9t)
  DevBuf ts_lmax, ts_tau, ts_count, ts_cs, ts_ci;  // K9t / K9q: sample maxima, tau, survivors
  DevBuf i8c_cs, i8c_ci, i8c_count;  // K9q survivors compacted (the debug select path)
  DevBuf msel, mblk;     // masked search: the allowed rows (sorted) + per-block counts
  DevBuf mres_s, mres_i;  // masked search: results staged for the host
  PinBuf pin;             // pinned host staging of the host-pointer search calls
  DevBuf rows8, scale8, err8, stats8;  // int8 shadow [cap, dim] + per-row scales, errors ||c - scale r8|| + maxima (as stats16)
  int64_t n8 = 0;                // rows already mirrored into rows8
  int64_t masked_gathers = 0;    // masked searches the int8 screen could not certify (gathered)
  bool i8_screen = true;         // single queries screen on the int8 shadow first (K9q)
  double i8_fail_avg = 0.0;      // running share of single queries the int8 screen failed to certify
  int i8_skip = 0;               // searches left that bypass the int8 tier after a bad run
  int64_t i8_skips = 0;          // single-query searches that sat the int8 tier out
  // asynchronous batched screen (TIER_BF16): the uncertified queries are re-run on the
  // device (fallback_scan / fallback_merge) instead of behind a host read of the failure
  // count; after a batch is seen to have failed, the next kAsyncCooldown batched screens
  // run the synchronous tiered path (split-f32 tier first, cheaper for many failures)
  bool async_screen = true;
  int sync_left = 0;
  DevBuf afb_q, afb_cs, afb_ci, afb_total;  // compact failed queries, their scan lists, cumulative count (u64)
  unsigned long long* afb_host = nullptr;  // pinned copy of the cumulative count
  hipEvent_t afb_event = nullptr;          // recorded after that copy
  unsigned long long afb_seen = 0;         // count already folded into screen_fallbacks
  // bf16 tier self-disable: running share of batched queries the bf16 certificate failed
  // (measured on the synchronous path); above kBfSkipShare the batched screen goes
  // straight to the split-f32 tier for bf_skip searches
  double bf_fail_avg = 0.0;
  int bf_skip = 0;
  int64_t bf_skips = 0;  // searches that bypassed the bf16 tier that way
  Timeline tl;  // stages: 0 = K9 score + top-k, 1 = K10 merge
  int precision = MQ_DTYPE_F32;
  std::mutex mu;
};

namespace {

template <class T, int KC>
void launch_search(const mq_index* ix, const float* q, int nq, int k, int G, int nqt,
                   float* cs, int* ci, hipStream_t s) {
  // bf16 tiles read the bf16 shadow as float-typed rows of half the width
  const float* rows = T::BF16 ? ix->rows16.as<float>() : ix->rows;
  const int dim = T::BF16 ? ix->dim / 2 : ix->dim;
  hipLaunchKernelGGL((flat_search_kernel<T, KC>), dim3(G * nqt), dim3(256), 0, s, q, nq, rows,
                     ix->n, dim, G, nqt, k, cs, ci);
}

template <int KC, typename IdIn>
void launch_merge(const float* cs, const IdIn* ci, int n_lists, int64_t nq, int k_in, int k_out,
                  float* os, int64_t* oi, int list_kc, int* overflow, hipStream_t s) {
  // k_out <= 16 over a batch: register thread lists (25 us at B = 256); larger k_out or
  // a few queries: the threshold merge (k_out = 64: 38 us vs 96 us with 16-entry thread
  // lists + overflow check; one query's 512 stream lists, k_out = 16: 29 vs 48 us)
  if (k_out <= 16 && nq > 32)
    hipLaunchKernelGGL((merge_kernel<KC, IdIn>), dim3((unsigned)nq), dim3(256), 0, s, cs, ci,
                       n_lists, nq, k_in, k_out, os, oi, list_kc, overflow);
  else
    hipLaunchKernelGGL((merge_select_kernel<KC, IdIn>), dim3((unsigned)nq), dim3(256), 0, s, cs, ci,
                       n_lists, nq, k_in, k_out, os, oi, list_kc, overflow);
}

template <typename IdIn>
void merge_dispatch(const float* cs, const IdIn* ci, int n_lists, int64_t nq, int k_in, int k_out,
                    float* os, int64_t* oi, hipStream_t s, int list_kc = 1 << 30,
                    int* overflow = nullptr, int kc = 0) {
  switch (kc ? kc : kc_merge(k_out)) {
    case 8: launch_merge<8>(cs, ci, n_lists, nq, k_in, k_out, os, oi, list_kc, overflow, s); break;
    case 16: launch_merge<16>(cs, ci, n_lists, nq, k_in, k_out, os, oi, list_kc, overflow, s); break;
    default: launch_merge<64>(cs, ci, n_lists, nq, k_in, k_out, os, oi, list_kc, overflow, s); break;
  }
}

struct SearchPlan {
  bool wide;
  int nqt;
  int G;
  int64_t n_lists;
};

SearchPlan plan_search(const mq_index* ix, int64_t nq, int kc) {
  SearchPlan p;
  p.wide = nq > kFbNarrowMax;
  const int BM = p.wide ? SearchWide::BM : SearchNarrow::BM;
  const int BN = p.wide ? SearchWide::BN : SearchNarrow::BN;
  const int wn = p.wide ? SearchWide::WAVES_N : SearchNarrow::WAVES_N;
  const int lpq = p.wide ? SearchSmem<SearchWide>::LPQ : SearchSmem<SearchNarrow>::LPQ;
  // resident 256-thread blocks per CU: 2 with an 8/16-entry register top list, 1 with
  // 64 (VGPR budget); G row groups per query tile, a multiple of 8 (XCD mapping)
  const ScanGeom g = scan_geom(nq, BM, BN, kc <= 16 ? 2 : 1, ix->num_cus, ix->n);
  p.nqt = g.nqt;
  p.G = g.G;
  p.n_lists = (int64_t)p.G * wn * lpq;
  return p;
}

int fill_padding(float* os, int64_t* oi, int64_t count, hipStream_t s) {
  std::vector<float> ps((size_t)count, -INFINITY);
  std::vector<int64_t> pi((size_t)count, -1);
  MQ_HIP(hipMemcpyAsync(os, ps.data(), ps.size() * 4, hipMemcpyHostToDevice, s));
  MQ_HIP(hipMemcpyAsync(oi, pi.data(), pi.size() * 8, hipMemcpyHostToDevice, s));
  MQ_HIP(hipStreamSynchronize(s));
  return MQ_OK;
}

enum ScanKind { SCAN_F32, SCAN_X6, SCAN_BF16, SCAN_STREAM, SCAN_STREAM16 };

template <int NQ, int KC, bool BF>
void launch_stream_nq(const mq_index* ix, const float* q, int nq, int kl, int blocks, float* cs,
                      int* ci, hipStream_t s, const unsigned* mask) {
  // query image, then the block merge's [16][NQ][KC] (score, id) lists in the same LDS
  const size_t lds = std::max((size_t)NQ * ix->dim * sizeof(float), (size_t)16 * NQ * KC * 8);
  auto launch = [&](auto kern) {
    if (lds > 64 * 1024)  // above the default dynamic-LDS limit (64-entry lists, NQ >= 8)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, s, q, nq,
                       BF ? ix->rows16.as<float>() : ix->rows, ix->n, ix->dim, kl, cs, ci, mask);
  };
  if constexpr (!BF) {  // the masked scan reads the fp32 rows
    if (mask) {
      if (ix->dim == 768)
        launch(stream_search_kernel<NQ, KC, 12, false, true>);
      else
        launch(stream_search_kernel<NQ, KC, kStreamMaxNV, false, true>);
      return;
    }
  }
  if (ix->dim == 768)  // the dmeta / BERT-base width, register arrays sized exactly
    launch(stream_search_kernel<NQ, KC, BF ? 6 : 12, BF>);
  else
    launch(stream_search_kernel<NQ, KC, kStreamMaxNV, BF>);
}

template <int KC, bool BF = false>
void launch_stream(const mq_index* ix, const float* q, int nq, int kl, int blocks, float* cs,
                   int* ci, hipStream_t s, const unsigned* mask = nullptr) {
  if (nq <= 1)
    launch_stream_nq<1, KC, BF>(ix, q, nq, kl, blocks, cs, ci, s, mask);
  else if (nq <= 2)
    launch_stream_nq<2, KC, BF>(ix, q, nq, kl, blocks, cs, ci, s, mask);
  else if (nq <= 4)
    launch_stream_nq<4, KC, BF>(ix, q, nq, kl, blocks, cs, ci, s, mask);
  else if (nq <= 8)
    launch_stream_nq<8, KC, BF>(ix, q, nq, kl, blocks, cs, ci, s, mask);
  else
    launch_stream_nq<16, KC, BF>(ix, q, nq, kl, blocks, cs, ci, s, mask);
}

// streaming-kernel grid: up to 2 blocks per CU, at least ~8 rows per lane group
int stream_blocks(const mq_index* ix) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(2 * ix->num_cus, (ix->n + 127) / 128));
}

template <int KC>
void launch_scan(const mq_index* ix, int kind, bool wide, const float* q, int nq, int kl, int G,
                 int nqt, float* cs, int* ci, hipStream_t s) {
  if (kind == SCAN_BF16) {
    if (wide)
      launch_search<SearchWideBF, KC>(ix, q, nq, kl, G, nqt, cs, ci, s);
    else
      launch_search<SearchNarrowBF, KC>(ix, q, nq, kl, G, nqt, cs, ci, s);
    return;
  }
  if constexpr (KC <= 16) {  // (a 64-entry list spills next to the x6 operands)
    if (kind == SCAN_X6 && wide) {
      launch_search<SearchWideX6, KC>(ix, q, nq, kl, G, nqt, cs, ci, s);
      return;
    }
  }
  if (wide)
    launch_search<SearchWide, KC>(ix, q, nq, kl, G, nqt, cs, ci, s);
  else
    launch_search<SearchNarrow, KC>(ix, q, nq, kl, G, nqt, cs, ci, s);
}

// Read a device status word back through the index's pinned host word (synchronises s).
int read_flag(mq_index* ix, const int* dflag, hipStream_t s, int* out) {
  if (!ix->host_flag) MQ_HIP(hipHostMalloc((void**)&ix->host_flag, sizeof(int), hipHostMallocDefault));
  MQ_HIP(hipMemcpyAsync(ix->host_flag, dflag, sizeof(int), hipMemcpyDeviceToHost, s));
  MQ_HIP(hipStreamSynchronize(s));
  *out = *ix->host_flag;
  return MQ_OK;
}

// K9 fused scan + K10 merge -> exact top-k of the whole index for every query.
// k <= 16 runs with lists of 8/16.  For 16 < k <= 64 the scan still keeps 16 per list
// and the merge checks that no list overflowed (see merge_kernel); if one did, the
// batch is re-scanned with 64-entry lists, so results are exact either way.  The
// check costs one 4-byte device->host read, i.e. k > 16 calls are synchronous.
int scan_topk(mq_index* ix, int kind, const float* q, int64_t nq, int k, float* os, int64_t* oi,
              hipStream_t s, const unsigned* mask = nullptr) {  // (mask: SCAN_STREAM only)
  // the bf16 scan keeps 8-entry lists whatever k (measured: 16-entry lists cost it ~40%;
  // k > 8 then runs with the merge's overflow check)
  int kc = kind == SCAN_BF16 ? 8 : kc_scan(k);
  for (;;) {
    const int kl = std::min(kc, k);
    const bool check = kl < k;
    SearchPlan p = plan_search(ix, nq, kc);
    const bool stream = kind == SCAN_STREAM || kind == SCAN_STREAM16;
    if (stream) p.n_lists = stream_blocks(ix);  // one list per block
    const size_t n_cand = (size_t)p.n_lists * nq * kl;
    int rc = ix->cand_s.ensure(n_cand * sizeof(float));
    if (!rc) rc = ix->cand_i.ensure(n_cand * sizeof(int));
    if (!rc && check) rc = ix->flag.ensure(sizeof(int));
    if (rc) return rc;
    float* cs = ix->cand_s.as<float>();
    int* ci = ix->cand_i.as<int>();
    int* flag = check ? ix->flag.as<int>() : nullptr;
    if (flag) MQ_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
    if (ix->tl.used > 4096) ix->tl.drain();
    ix->tl.mark(s, 0);
    if (kind == SCAN_STREAM) {
      const int nb = stream_blocks(ix);
      switch (kc) {
        case 8: launch_stream<8>(ix, q, (int)nq, kl, nb, cs, ci, s, mask); break;
        case 16: launch_stream<16>(ix, q, (int)nq, kl, nb, cs, ci, s, mask); break;
        default: launch_stream<MQ_MAX_K>(ix, q, (int)nq, kl, nb, cs, ci, s, mask); break;
      }
    } else if (kind == SCAN_STREAM16) {
      const int nb = stream_blocks(ix);
      switch (kc) {
        case 8: launch_stream<8, true>(ix, q, (int)nq, kl, nb, cs, ci, s); break;
        case 16: launch_stream<16, true>(ix, q, (int)nq, kl, nb, cs, ci, s); break;
        default: launch_stream<MQ_MAX_K, true>(ix, q, (int)nq, kl, nb, cs, ci, s); break;
      }
    } else switch (kc) {
      case 8: launch_scan<8>(ix, kind, p.wide, q, (int)nq, kl, p.G, p.nqt, cs, ci, s); break;
      case 16: launch_scan<16>(ix, kind, p.wide, q, (int)nq, kl, p.G, p.nqt, cs, ci, s); break;
      default: launch_scan<MQ_MAX_K>(ix, kind, p.wide, q, (int)nq, kl, p.G, p.nqt, cs, ci, s); break;
    }
    MQ_HIP(hipGetLastError());
    ix->tl.mark(s, 1);
    // k > 16: 16-entry thread lists in the merge too (KC = 64 costs ~20x more)
    const int merge_kc = flag ? 16 : kc_merge(k);
    merge_dispatch<int>(cs, ci, (int)p.n_lists, nq, kl, k, os, oi, s, kl, flag, merge_kc);
    ix->tl.close(s);
    MQ_HIP(hipGetLastError());
    if (!flag) return MQ_OK;
    int overflow = 0;
    rc = read_flag(ix, flag, s, &overflow);
    if (rc) return rc;
    if (overflow & 1) {  // a scan list overflowed: re-scan with full-length lists
      ++ix->rescans;
      kc = MQ_MAX_K;
      if (kind == SCAN_X6) kind = SCAN_F32;
      continue;
    }
    if (overflow & 2) {  // only a merge thread list overflowed: re-merge with KC = 64
      ++ix->remerges;
      merge_dispatch<int>(cs, ci, (int)p.n_lists, nq, kl, k, os, oi, s, kl, nullptr, MQ_MAX_K);
      MQ_HIP(hipGetLastError());
    }
    return MQ_OK;
  }
}

// bf16 shadow of the stored rows, mirrored lazily (rows added since the last bf16 search),
// with the rounding maxima the bf16 screens certify against (reset on a rebuild).
int ensure_shadow(mq_index* ix, hipStream_t s) {
  // padded to whole 32-row blocks: the threshold scan (K9t) reads blocks unclamped
  int rc = ix->rows16.ensure((size_t)(ix->cap + kTsRows) * ix->dim * 2);
  if (!rc) rc = ix->stats16.ensure(2 * sizeof(unsigned));
  if (rc) return rc;
  if (ix->n16 < ix->n) {
    if (ix->n16 == 0) MQ_HIP(hipMemsetAsync(ix->stats16.p, 0, 2 * sizeof(unsigned), s));
    const int64_t nr = ix->n - ix->n16;
    hipLaunchKernelGGL(bf16_shadow_kernel, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, s,
                       ix->rows + ix->n16 * ix->dim,
                       ix->rows16.as<unsigned>() + ix->n16 * ix->dim / 2, nr, ix->dim,
                       ix->stats16.as<unsigned>());
    MQ_HIP(hipGetLastError());
    ix->n16 = ix->n;
  }
  return MQ_OK;
}

int queries_to_bf16(mq_index* ix, const float* q, int64_t nq, hipStream_t s) {
  int rc = ix->q16.ensure((size_t)nq * ix->dim * 2);
  if (rc) return rc;
  const int64_t qpairs = nq * ix->dim / 2;
  hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)((qpairs + 255) / 256)), dim3(256), 0, s, q,
                     ix->q16.as<unsigned>(), qpairs);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// K9t: bf16 top-kc candidates of a batch by the threshold scan.  Sample pass (every
// kTsPeriod-th block, per-list maxima) -> tau per query -> full pass appending the rows
// that clear tau -> per-query select of the best kc survivors.  Stage 0 of the timeline
// = the two scans, stage 1 = tau + select.
bool thresh_ok(const mq_index* ix, int64_t nq) {
  const int nch = ix->dim / 64;
  return ix->thresh_scan && nq > 64 && ix->dim % 64 == 0 && (nch == 4 || nch == 8 || nch == 12) &&
         ix->n >= kTsMinRows && ix->n < (1ll << 31);
}

int thresh_topk(mq_index* ix, const float* q16, int64_t nq, int kc, float* os, int64_t* oi,
                hipStream_t s, int tau_rank, int* fail_count, int64_t* fail, const unsigned* mask = nullptr) {
  const size_t n_lists = 2 * (size_t)ix->num_cus;
  int rc = ix->ts_lmax.ensure(n_lists * nq * sizeof(float));
  if (!rc) rc = ix->ts_tau.ensure(nq * sizeof(float));
  if (!rc) rc = ix->ts_count.ensure(nq * sizeof(int));
  if (!rc) rc = ix->ts_cs.ensure((size_t)nq * kTsCap * sizeof(float));
  if (!rc) rc = ix->ts_ci.ensure((size_t)nq * kTsCap * sizeof(int));
  if (rc) return rc;
  ThreshArgs a{q16, (int)nq, ix->rows16.as<unsigned char>(), ix->n, ix->dim, ix->num_cus, kc,
               ix->ts_lmax.as<float>(), ix->ts_tau.as<float>(), ix->ts_count.as<int>(),
               ix->ts_cs.as<float>(), ix->ts_ci.as<int>(), os, oi, tau_rank, fail_count, fail, mask};
  if (ix->tl.used > 4096) ix->tl.drain();
  launch_thresh(a, s, &ix->tl);
  ix->tl.close(s);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// int8 shadow (K9q) of the stored rows, extended lazily like the bf16 one.
int ensure_i8(mq_index* ix, hipStream_t s) {
  int rc = ix->rows8.ensure((size_t)(ix->cap + kI8PadRows) * ix->dim);
  if (!rc) rc = ix->scale8.ensure((size_t)(ix->cap + kI8PadRows) * sizeof(float));
  if (!rc) rc = ix->err8.ensure((size_t)(ix->cap + kI8PadRows) * sizeof(float));
  if (!rc) rc = ix->stats8.ensure(2 * sizeof(unsigned));
  if (rc) return rc;
  if (ix->n8 < ix->n) {
    if (ix->n8 == 0) MQ_HIP(hipMemsetAsync(ix->stats8.p, 0, 2 * sizeof(unsigned), s));
    launch_i8_shadow(ix->rows + ix->n8 * ix->dim, ix->n - ix->n8, ix->dim,
                     ix->rows8.as<unsigned>() + ix->n8 * ix->dim / 4, ix->scale8.as<float>() + ix->n8,
                     ix->err8.as<float>() + ix->n8, ix->stats8.as<unsigned>(), s);
    MQ_HIP(hipGetLastError());
    ix->n8 = ix->n;
  }
  return MQ_OK;
}

// The int8 screen applies to one query over >= kTsMinRows rows of dim 256..1024, unless
// it failed to certify most recent queries (then it sits out i8_skip searches).
bool i8_ok(mq_index* ix, int64_t nq) {
  if (!ix->i8_screen || nq != 1 || ix->dim % 256 != 0 || ix->dim > 1024 || ix->n < kTsMinRows ||
      ix->n >= (1ll << 31))
    return false;
  if (ix->i8_skip > 0) {
    --ix->i8_skip;
    ++ix->i8_skips;
    return false;
  }
  return true;
}

// K9q scans for nq = 1 query, then (os != null) the select of the top-kc candidates;
// `zero` (optional) is set to 0 by the sample pass.  The timeline stays open (stage 1).
int i8_topk(mq_index* ix, const float* q, int64_t nq, int kc, float* os, int64_t* oi, hipStream_t s,
            int* zero = nullptr, int kcert = 0, const unsigned* mask = nullptr) {
  const size_t n_lists = (size_t)i8_lists(ix->num_cus);
  int rc = ensure_i8(ix, s);
  if (!rc) rc = ix->ts_lmax.ensure(n_lists * nq * sizeof(float));
  if (!rc) rc = ix->ts_tau.ensure(nq * sizeof(float));
  if (!rc) rc = ix->ts_count.ensure(nq * n_lists * sizeof(int));
  if (!rc) rc = ix->ts_cs.ensure((size_t)nq * n_lists * kI8Seg * sizeof(float));
  if (!rc) rc = ix->ts_ci.ensure((size_t)nq * n_lists * kI8Seg * sizeof(int));
  if (!rc && os) rc = ix->i8c_count.ensure(nq * sizeof(int));
  if (!rc && os) rc = ix->i8c_cs.ensure((size_t)nq * kTsCap * sizeof(float));
  if (!rc && os) rc = ix->i8c_ci.ensure((size_t)nq * kTsCap * sizeof(int));
  if (rc) return rc;
  ThreshI8Args a{q, (int)nq, ix->rows8.as<unsigned>(), ix->scale8.as<float>(), ix->n, ix->dim, ix->num_cus,
                 ix->ts_lmax.as<float>(), ix->ts_tau.as<float>(), ix->ts_count.as<int>(),
                 ix->ts_cs.as<float>(), ix->ts_ci.as<int>(), zero, ix->stats8.as<unsigned>(), kcert, mask};
  if (ix->tl.used > 4096) ix->tl.drain();
  launch_thresh_i8(a, s, &ix->tl);
  ix->tl.mark(s, 1);
  if (os) {
    launch_i8_compact(ix->ts_cs.as<float>(), ix->ts_ci.as<int>(), ix->ts_count.as<int>(), (int)n_lists, (int)nq,
                      ix->i8c_cs.as<float>(), ix->i8c_ci.as<int>(), ix->i8c_count.as<int>(), s);
    launch_select(ix->i8c_cs.as<float>(), ix->i8c_ci.as<int>(), ix->i8c_count.as<int>(), ix->ts_tau.as<float>(),
                  (int)nq, kc, os, oi, s);
  }
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// screen tiers (see search_screened)
enum ScreenTier { TIER_BF16_STREAM = 0, TIER_BF16 = 1, TIER_X6 = 2, TIER_I8 = 3 };

// the bf16 candidate scan of a batch: K9t when it applies, else the tiled K9 + K10.
// K9t's tau is the tau_rank-th sample list maximum (the screens keep kTsRank: ~128
// survivors, the certificate covers a short list); with `fail` set, queries whose
// survivors overflowed kTsCap or fell short of kc are listed there for a re-run.
int bf16_candidates(mq_index* ix, const float* q16, int64_t nq, int kc, float* os, int64_t* oi,
                    hipStream_t s, int tau_rank = kTsRank, int* fail_count = nullptr,
                    int64_t* fail = nullptr) {
  if (thresh_ok(ix, nq)) return thresh_topk(ix, q16, nq, kc, os, oi, s, tau_rank, fail_count, fail);
  return scan_topk(ix, SCAN_BF16, q16, nq, kc, os, oi, s);
}

// Config 5: bf16 coarse scan for the best `kc` rows per query (kc = max(2k, 50) capped
// at MQ_MAX_K and n), then an exact fp32 re-rank of those candidates to the final top-k.
// No certificate covers this mode, so every query must come out of the threshold scan
// with at least kc survivors: tau sits at the min(kc, 24)-th sample list maximum (at
// least that many survivors by construction; ~24 x 16 = 384 expected at the 1/16 sample,
// so fewer than 64 is a > 4-sigma event - tau at the 64th would keep ~1024 and cost the
// scan ~50%), and a query whose survivors still fall short of kc, or overflow kTsCap
// (heavy duplicates), is re-run on the tiled bf16 scan, which always yields the exact
// bf16 top-kc.  Synchronous when the threshold scan ran.
int search_bf16_rerank(mq_index* ix, const float* q, int64_t nq, int k, float* os, int64_t* oi,
                       hipStream_t s) {
  int rc = ensure_shadow(ix, s);
  if (!rc) rc = queries_to_bf16(ix, q, nq, s);
  if (rc) return rc;
  const int kc = (int)std::min<int64_t>(std::max(2 * k, 50), std::min<int64_t>(MQ_MAX_K, ix->n));
  const bool ts = thresh_ok(ix, nq);
  rc = ix->coarse_s.ensure((size_t)nq * kc * sizeof(float));
  if (!rc) rc = ix->coarse_i.ensure((size_t)nq * kc * sizeof(int64_t));
  if (!rc && ts) rc = ix->flag.ensure(sizeof(int));
  if (!rc && ts) rc = ix->tier_fail[TIER_BF16].ensure((size_t)nq * sizeof(int64_t));
  if (rc) return rc;
  int64_t* fail = ts ? ix->tier_fail[TIER_BF16].as<int64_t>() : nullptr;
  if (ts) MQ_HIP(hipMemsetAsync(ix->flag.p, 0, sizeof(int), s));
  rc = bf16_candidates(ix, ix->q16.as<float>(), nq, kc, ix->coarse_s.as<float>(), ix->coarse_i.as<int64_t>(),
                       s, std::min(kc, 24), ts ? ix->flag.as<int>() : nullptr, fail);
  if (rc) return rc;
  hipLaunchKernelGGL(rerank_kernel, dim3((unsigned)nq), dim3(256), 0, s, q, ix->rows, ix->dim,
                     ix->coarse_i.as<int64_t>(), kc, k, os, oi, nullptr, kNoPrune, nullptr);
  MQ_HIP(hipGetLastError());
  if (!ts) return MQ_OK;
  int n_fail = 0;
  rc = read_flag(ix, ix->flag.as<int>(), s, &n_fail);
  if (rc || n_fail == 0) return rc;
  ++ix->rescans;
  rc = ix->tier_q[TIER_BF16].ensure((size_t)n_fail * ix->dim * sizeof(float));
  if (!rc) rc = ix->tier_s[TIER_BF16].ensure((size_t)n_fail * k * sizeof(float));
  if (!rc) rc = ix->tier_i[TIER_BF16].ensure((size_t)n_fail * k * sizeof(int64_t));
  if (!rc) rc = ix->fb_cs.ensure((size_t)n_fail * kc * sizeof(float));
  if (!rc) rc = ix->fb_ci.ensure((size_t)n_fail * kc * sizeof(int64_t));
  if (rc) return rc;
  float* sq = ix->tier_q[TIER_BF16].as<float>();
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n_fail + 3) / 4)), dim3(256), 0, s, q, fail,
                     (int64_t)n_fail, ix->dim, sq);
  MQ_HIP(hipGetLastError());
  rc = queries_to_bf16(ix, sq, n_fail, s);
  if (!rc) rc = scan_topk(ix, SCAN_BF16, ix->q16.as<float>(), n_fail, kc, ix->fb_cs.as<float>(),
                          ix->fb_ci.as<int64_t>(), s);
  if (rc) return rc;
  hipLaunchKernelGGL(rerank_kernel, dim3((unsigned)n_fail), dim3(256), 0, s, sq, ix->rows, ix->dim,
                     ix->fb_ci.as<int64_t>(), kc, k, ix->tier_s[TIER_BF16].as<float>(),
                     ix->tier_i[TIER_BF16].as<int64_t>(), nullptr, kNoPrune, nullptr);
  const int64_t total = (int64_t)n_fail * k;
  hipLaunchKernelGGL(scatter_results_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     ix->tier_s[TIER_BF16].as<float>(), ix->tier_i[TIER_BF16].as<int64_t>(), fail,
                     (int64_t)n_fail, k, os, oi);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// The direct exact fp32 scan: streaming kernel for a handful of queries, MFMA tiles else.
bool stream_ok(const mq_index* ix) { return ix->dim % 64 == 0 && ix->dim <= 64 * kStreamMaxNV; }

int search_direct(mq_index* ix, const float* q, int64_t nq, int k, float* os, int64_t* oi,
                  hipStream_t s) {
  if (nq <= ix->stream_max_q && stream_ok(ix)) return scan_topk(ix, SCAN_STREAM, q, nq, k, os, oi, s);
  return scan_topk(ix, SCAN_F32, q, nq, k, os, oi, s);
}

// Exact fp32 top-k through certified screens (MQ_DTYPE_F32_SCREEN).  A tier scans with
// cheaper arithmetic for kc > k candidates per query, re-ranks them in fp32
// (rerank_kernel) and certifies each query (screen_verify_kernel); the queries whose
// certificate fails are gathered and re-run one tier down, and their results scattered
// back.  Tiers:
//   TIER_BF16_STREAM  few queries: bf16 shadow streamed against the fp32 query (half the
//                     HBM bytes of the exact stream) -> direct exact stream
//   TIER_BF16         batches: bf16 MFMA scan of the shadow -> split-f32 tier (> 64
//                     failing queries) or the direct exact scan
//   TIER_X6           split-f32 MFMA scan -> direct exact scan
//   TIER_I8           one query: int8 shadow threshold scan (K9q, a quarter of the fp32
//                     bytes) for 64 candidates -> TIER_BF16_STREAM
// Synchronous (reads the failure count).

bool x6_tier_ok(const mq_index* ix, int64_t nq, int k) {
  return nq > 64 && k + 8 <= MQ_MAX_K && ix->dim <= 1024;
}

// The approximate tiers (int8, bf16) keep 64 candidates (16-48 on the bf16 stream) against
// bounds of ~2e-3 .. 1.4e-2 on unit vectors, so the k-th best must clear the kc-th by
// twice that.  Over 1M isotropic 768-d rows the k-th and 64-th best scores are ~0.58 /
// 0.33 / 0.16 sigma (sigma = 0.036) apart at k = 5 / 16 / 32, and ~0.03 sigma at k = 50:
// past k = 16 most certificates would fail and every batch would pay the screen AND the
// re-run, so larger k goes straight to the split-f32 tier (bound 8e-5, kc = k + 8) or the
// direct exact scan.  (kScreenMaxK = 16 is defined with the K9q finish, which sizes its
// wave winners by it.)
constexpr double kBfSkipShare = 0.2;  // bf16 certificate failure share that disables the tier
constexpr int kBfSkipSearches = 64;

int batch_tier(mq_index* ix, int64_t nq, int k) {
  if (k <= kScreenMaxK) {
    if (ix->bf_skip == 0) return TIER_BF16;
    --ix->bf_skip;
    ++ix->bf_skips;
  }
  return x6_tier_ok(ix, nq, k) ? TIER_X6 : -1;
}

constexpr int kAsyncCooldown = 16;

// Fold a completed pinned copy of the device fallback count into screen_fallbacks (no
// wait: an unfinished copy is read at a later call); a new failure starts the cooldown.
void poll_async_fallbacks(mq_index* ix) {
  if (!ix->afb_event || hipEventQuery(ix->afb_event) != hipSuccess) return;
  const unsigned long long tot = *ix->afb_host;
  if (tot > ix->afb_seen) {
    ix->screen_fallbacks += (int64_t)(tot - ix->afb_seen);
    ix->afb_seen = tot;
    ix->sync_left = kAsyncCooldown;
  }
}

// Worst case over every failure count nf = 1..nq of one tile shape's fallback scan:
// workgroups to launch and candidate entries (lists x nf x kl).
template <class T>
void fallback_extent(const mq_index* ix, int64_t nf_lo, int64_t nf_hi, int per_cu, int kl,
                     int64_t* grid, int64_t* cand) {
  for (int64_t nqt = (nf_lo + T::BM - 1) / T::BM; nqt * T::BM < nf_hi + T::BM; ++nqt) {
    const int64_t nf = std::min(nf_hi, nqt * T::BM);  // the most queries with this nqt
    const ScanGeom g = scan_geom(nf, T::BM, T::BN, per_cu, ix->num_cus, ix->n);
    *grid = std::max<int64_t>(*grid, (int64_t)g.G * g.nqt);
    *cand = std::max<int64_t>(*cand, (int64_t)g.G * T::WAVES_N * SearchSmem<T>::LPQ * nf * kl);
  }
}

template <int KC>
void launch_fallback_scans(mq_index* ix, int64_t nq, int k, const int* nf, const int64_t* fail,
                           float* os, int64_t* oi, int64_t grid, hipStream_t s) {
  const float* qc = ix->afb_q.as<float>();
  float* cs = ix->afb_cs.as<float>();
  int* ci = ix->afb_ci.as<int>();
  hipLaunchKernelGGL((fallback_search_kernel<KC>), dim3((unsigned)grid), dim3(256), 0, s, qc, nf, ix->rows,
                     ix->n, ix->dim, ix->num_cus, k, cs, ci);
  auto* tot = ix->afb_total.as<unsigned long long>();
  const dim3 mgrid((unsigned)nq);
  if (k <= 8)
    hipLaunchKernelGGL((fallback_merge_kernel<8, KC>), mgrid, dim3(256), 0, s, cs, ci, ix->num_cus, ix->n, k, k,
                       nf, fail, os, oi, tot);
  else
    hipLaunchKernelGGL((fallback_merge_kernel<16, KC>), mgrid, dim3(256), 0, s, cs, ci, ix->num_cus, ix->n, k,
                       k, nf, fail, os, oi, tot);
}

// Device-side exact re-run of the uncertified queries (count, list and compact query
// block from screen_verify_kernel; k <= 16), results written into os / oi; nothing is
// read back.  fallback_prepare sizes the workspace (before the verify launch, which
// writes the compact block) and says whether the asynchronous path applies: not when the
// worst-case candidate lists plus the compact query block would take more than kFbMaxBytes
// (very large batches stay synchronous).
constexpr size_t kFbMaxBytes = 256ull << 20;

struct FallbackPlan {
  bool ok = false;
  int64_t grid = 0;
};

int fallback_prepare(mq_index* ix, int64_t nq, int k, FallbackPlan* fp) {
  const int per_cu = 2;  // 8- / 16-entry scan lists
  int64_t grid_n = 0, grid_w = 0, cand = 0;
  fallback_extent<SearchNarrow>(ix, 1, std::min<int64_t>(nq, kFbNarrowMax), per_cu, k, &grid_n, &cand);
  if (nq > kFbNarrowMax) fallback_extent<SearchWide>(ix, kFbNarrowMax + 1, nq, per_cu, k, &grid_w, &cand);
  fp->ok = false;
  // the budget counts the compact query block too (nq x dim floats): a batch of
  // millions of queries with small k stays synchronous instead of keeping a second copy
  if ((size_t)cand * (sizeof(float) + sizeof(int)) + (size_t)nq * ix->dim * sizeof(float) > kFbMaxBytes)
    return MQ_OK;
  int rc = ix->afb_q.ensure((size_t)nq * ix->dim * sizeof(float));
  if (!rc) rc = ix->afb_cs.ensure((size_t)cand * sizeof(float));
  if (!rc) rc = ix->afb_ci.ensure((size_t)cand * sizeof(int));
  if (!rc && !ix->afb_total.p) {
    rc = ix->afb_total.ensure(sizeof(unsigned long long));
    if (!rc) MQ_HIP(hipMemset(ix->afb_total.p, 0, sizeof(unsigned long long)));
  }
  if (rc) return rc;
  if (!ix->afb_host) {
    MQ_HIP(hipHostMalloc((void**)&ix->afb_host, sizeof(unsigned long long), hipHostMallocDefault));
    *ix->afb_host = 0;
  }
  if (!ix->afb_event) MQ_HIP(hipEventCreateWithFlags(&ix->afb_event, hipEventDisableTiming));
  fp->ok = true;
  fp->grid = std::max(grid_n, grid_w);
  return MQ_OK;
}

// launch_fallback_scans' list widths are 8 / 16: the async path runs only for k <= kScreenMaxK
static_assert(kScreenMaxK <= 16, "fallback_search_kernel<KC> has KC = 8 or 16");
int launch_async_fallback(mq_index* ix, const FallbackPlan& fp, int64_t nq, int k, float* os, int64_t* oi,
                          const int64_t* fail, hipStream_t s) {
  const int* nf = ix->flag.as<int>();
  if (k <= 8)
    launch_fallback_scans<8>(ix, nq, k, nf, fail, os, oi, fp.grid, s);
  else
    launch_fallback_scans<16>(ix, nq, k, nf, fail, os, oi, fp.grid, s);
  MQ_HIP(hipGetLastError());
  MQ_HIP(hipMemcpyAsync(ix->afb_host, ix->afb_total.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  MQ_HIP(hipEventRecord(ix->afb_event, s));
  return MQ_OK;
}

int search_screened(mq_index* ix, int tier, const float* q, int64_t nq, int k, float* os,
                    int64_t* oi, hipStream_t s) {
  const bool bf = tier == TIER_BF16_STREAM || tier == TIER_BF16;
  // candidates: the bf16 screen's error bound is ~3.5e-3 for unit vectors, so it keeps
  // a wide margin - 64 per query in batches (the k-th and 64-th scores of 1M random-ish
  // rows are ~0.02 apart).  Streamed queries keep the fp32 query (bound ~2e-3): 16 for
  // k <= 5 - exactly the stream kernel's 16-entry lists, so the scan needs no overflow
  // check and its host round trip (single-query latency) - else max(32, k + 16).  The
  // split-f32 screen (bound 8e-5) keeps k + 3 while that fits its 8-entry lists (k <= 5),
  // else k + 8
  const int want = tier == TIER_BF16 || tier == TIER_I8 ? MQ_MAX_K
                   : tier == TIER_BF16_STREAM ? (k + 11 <= 16 ? 16 : std::min(std::max(32, k + 16), MQ_MAX_K))
                   : (k + 3 <= 8 ? 8 : k + 8);
  const int kc = (int)std::min<int64_t>(want, ix->n);
  int rc = bf ? ensure_shadow(ix, s) : MQ_OK;
  if (!rc && tier == TIER_BF16) rc = queries_to_bf16(ix, q, nq, s);
  if (!rc) rc = ix->coarse_s.ensure((size_t)nq * kc * sizeof(float));
  if (!rc) rc = ix->coarse_i.ensure((size_t)nq * kc * sizeof(int64_t));
  if (!rc) rc = ix->flag.ensure(sizeof(int));
  if (!rc) rc = ix->tier_fail[tier].ensure((size_t)nq * sizeof(int64_t));
  if (rc) return rc;
  int64_t* fail = ix->tier_fail[tier].as<int64_t>();
  if (tier == TIER_I8) {
    // scans (the sample pass zeroes the failure count), then select + re-rank + certificate
    // in one launch; the int8 screen's bound has the Q32 form (fp32 query) with the int8
    // shadow's maxima (kc = 64 < n: the int8 tier needs >= kTsMinRows rows)
    rc = i8_topk(ix, q, nq, kc, nullptr, nullptr, s, ix->flag.as<int>(), k);
    if (rc) return rc;
    hipLaunchKernelGGL(i8_finish_kernel, dim3((unsigned)nq), dim3(kFinT), 0, s, q, ix->rows, ix->dim,
                       ix->ts_cs.as<float>(), ix->ts_ci.as<int>(), ix->ts_count.as<int>(),
                       i8_lists(ix->num_cus), ix->ts_tau.as<float>(), k, ix->stats8.as<unsigned>(), ix->err8.as<float>(), os, oi, ix->flag.as<int>(), fail);
    ix->tl.close(s);
    MQ_HIP(hipGetLastError());
  } else {
    const int kind = tier == TIER_X6 ? SCAN_X6 : tier == TIER_BF16 ? SCAN_BF16 : SCAN_STREAM16;
    const float* qs = tier == TIER_BF16 ? ix->q16.as<float>() : q;
    rc = kind == SCAN_BF16 ? bf16_candidates(ix, qs, nq, kc, ix->coarse_s.as<float>(), ix->coarse_i.as<int64_t>(), s)
                           : scan_topk(ix, kind, qs, nq, kc, ix->coarse_s.as<float>(), ix->coarse_i.as<int64_t>(), s);
    if (rc) return rc;
    const int mode = tier == TIER_X6 ? VERIFY_X6 : tier == TIER_BF16 ? VERIFY_BF16_Q16 : VERIFY_BF16_Q32;
    const unsigned* stats = bf ? ix->stats16.as<unsigned>() : nullptr;
    hipLaunchKernelGGL(rerank_kernel, dim3((unsigned)nq), dim3(256), 0, s, q, ix->rows, ix->dim,
                       ix->coarse_i.as<int64_t>(), kc, k, os, oi, ix->coarse_s.as<float>(), mode, stats);
    MQ_HIP(hipGetLastError());
    if (kc >= ix->n) return MQ_OK;  // every row was a candidate: the re-rank is the answer
    FallbackPlan fp;
    if (tier == TIER_BF16) {
      poll_async_fallbacks(ix);
      if (ix->async_screen && ix->sync_left == 0 && k <= kScreenMaxK) {
        rc = fallback_prepare(ix, nq, k, &fp);
        if (rc) return rc;
      }
      if (!fp.ok && ix->sync_left > 0) --ix->sync_left;
    }
    MQ_HIP(hipMemsetAsync(ix->flag.p, 0, sizeof(int), s));
    hipLaunchKernelGGL(screen_verify_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, q,
                       ix->dim, ix->coarse_s.as<float>(), kc, os, k, nq, mode, stats, ix->flag.as<int>(),
                       fail, fp.ok ? ix->afb_q.as<float>() : nullptr);
    MQ_HIP(hipGetLastError());
    if (fp.ok) return launch_async_fallback(ix, fp, nq, k, os, oi, fail, s);
  }
  int n_fail = 0;
  rc = read_flag(ix, ix->flag.as<int>(), s, &n_fail);
  if (rc) return rc;
  if (tier == TIER_I8) {
    // a corpus whose top scores crowd within the int8 bound fails most certificates: after
    // a run of failures the single-query path goes straight to the bf16 stream for a while
    ix->i8_fail_avg = 0.9 * ix->i8_fail_avg + 0.1 * (double)n_fail / (double)nq;
    if (ix->i8_fail_avg > 0.3) {
      ix->i8_skip = 256;
      ix->i8_fail_avg = 0.0;
    }
  } else if (tier == TIER_BF16) {
    // the same for batches: a crowded corpus (near-duplicates, clusters denser than the
    // bf16 bound) sends the batched screen straight to the split-f32 tier for a while
    ix->bf_fail_avg = 0.75 * ix->bf_fail_avg + 0.25 * (double)n_fail / (double)nq;
    if (ix->bf_fail_avg > kBfSkipShare) {
      ix->bf_skip = kBfSkipSearches;
      ix->bf_fail_avg = 0.0;
    }
  }
  if (n_fail == 0) return MQ_OK;
  // re-run the uncertified queries one tier down, into this tier's scratch
  rc = ix->tier_q[tier].ensure((size_t)n_fail * ix->dim * sizeof(float));
  if (!rc) rc = ix->tier_s[tier].ensure((size_t)n_fail * k * sizeof(float));
  if (!rc) rc = ix->tier_i[tier].ensure((size_t)n_fail * k * sizeof(int64_t));
  if (rc) return rc;
  float* sq = ix->tier_q[tier].as<float>();
  float* ss = ix->tier_s[tier].as<float>();
  int64_t* si = ix->tier_i[tier].as<int64_t>();
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n_fail + 3) / 4)), dim3(256), 0, s, q,
                     fail, (int64_t)n_fail, ix->dim, sq);
  MQ_HIP(hipGetLastError());
  if (tier == TIER_BF16 && x6_tier_ok(ix, n_fail, k)) {
    ix->screen_passdowns += n_fail;
    rc = search_screened(ix, TIER_X6, sq, n_fail, k, ss, si, s);
  } else if (tier == TIER_I8) {
    ix->screen_passdowns += n_fail;
    rc = search_screened(ix, TIER_BF16_STREAM, sq, n_fail, k, ss, si, s);
  } else {
    ix->screen_fallbacks += n_fail;
    rc = search_direct(ix, sq, n_fail, k, ss, si, s);
  }
  if (rc) return rc;
  const int64_t total = (int64_t)n_fail * k;
  hipLaunchKernelGGL(scatter_results_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     ss, si, fail, (int64_t)n_fail, k, os, oi);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// Search with queries and outputs already in device memory (asynchronous for k <= 16,
// except the screened mode).
int search_device(mq_index* ix, const float* q, int64_t nq, int k, float* os, int64_t* oi,
                  hipStream_t s) {
  if (ix->n == 0) return fill_padding(os, oi, nq * k, s);
  const bool screen = ix->precision == MQ_DTYPE_F32_SCREEN;
  if (nq <= ix->stream_max_q && stream_ok(ix)) {  // few queries: streaming scans
    const bool approx = screen && k <= kScreenMaxK;
    if (approx && i8_ok(ix, nq)) return search_screened(ix, TIER_I8, q, nq, k, os, oi, s);
    if (approx && ix->dim % 128 == 0) return search_screened(ix, TIER_BF16_STREAM, q, nq, k, os, oi, s);
    return scan_topk(ix, SCAN_STREAM, q, nq, k, os, oi, s);
  }
  if (ix->precision == MQ_DTYPE_BF16 && ix->dim % 64 == 0)
    return search_bf16_rerank(ix, q, nq, k, os, oi, s);
  if (screen && ix->dim % 64 == 0 && ix->dim <= 1024) {
    const int tier = batch_tier(ix, nq, k);
    if (tier >= 0) return search_screened(ix, tier, q, nq, k, os, oi, s);
    return search_direct(ix, q, nq, k, os, oi, s);
  }
  return scan_topk(ix, ix->precision == MQ_DTYPE_F32X6 ? SCAN_X6 : SCAN_F32, q, nq, k, os, oi, s);
}

int reserve_rows(mq_index* ix, int64_t need_rows, hipStream_t s) {
  if (need_rows <= ix->cap) return MQ_OK;
  int64_t new_cap = std::max<int64_t>(need_rows, ix->cap + ix->cap / 2);
  new_cap = std::max<int64_t>(new_cap, 1024);
  float* fresh = nullptr;
  if (hipMalloc((void**)&fresh, (size_t)new_cap * ix->dim * sizeof(float)) != hipSuccess)
    MQ_FAIL(MQ_ENOMEM, "hipMalloc of %lld rows failed", (long long)new_cap);
  if (ix->n > 0) {
    MQ_HIP(hipMemcpyAsync(fresh, ix->rows, (size_t)ix->n * ix->dim * sizeof(float),
                          hipMemcpyDeviceToDevice, s));
    MQ_HIP(hipStreamSynchronize(s));
  }
  if (ix->rows) MQ_HIP(hipFree(ix->rows));
  ix->rows = fresh;
  ix->cap = new_cap;
  ix->n16 = 0;  // the bf16 / int8 shadows are rebuilt at the next screened search
  ix->n8 = 0;
  return MQ_OK;
}

constexpr char kMagic[8] = {'M', 'Q', 'F', 'L', 'A', 'T', '0', '1'};

struct FileHeader {
  char magic[8];
  int32_t dim;
  int32_t dtype;
  int64_t n_rows;
};

}  // namespace

extern "C" {

int mq_index_create(int device, int dim, int64_t capacity, int dtype, mq_index** out) {
  clear_error();
  MQ_CHECK_ARG(out != nullptr, "out is NULL");
  *out = nullptr;
  MQ_CHECK_ARG(dim > 0 && dim % kBK == 0, "dim must be a positive multiple of %d (got %d)", kBK,
               dim);
  MQ_CHECK_ARG(capacity >= 0, "negative capacity");
  MQ_CHECK_ARG(dtype == MQ_DTYPE_F32, "only the f32 index dtype is implemented (got %d)", dtype);
  DeviceGuard dg(device);
  if (!dg.ok) MQ_FAIL(MQ_EHIP, "hipSetDevice(%d) failed", device);
  auto ix = std::make_unique<mq_index>();
  ix->device = device;
  ix->dim = dim;
  ix->dtype = dtype;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      cus > 0)
    ix->num_cus = cus;
  if (capacity > 0) {
    int rc = reserve_rows(ix.get(), capacity, nullptr);
    if (rc) return rc;
  }
  *out = ix.release();
  return MQ_OK;
}

int mq_index_destroy(mq_index* ix) {
  clear_error();
  if (!ix) return MQ_OK;
  {
    DeviceGuard dg(ix->device);
    if (ix->rows) (void)hipFree(ix->rows);
    if (ix->host_flag) (void)hipHostFree(ix->host_flag);
    ix->pin.release();
    ix->stage.release();
    ix->cand_s.release();
    ix->cand_i.release();
    ix->out_s.release();
    ix->out_i.release();
    ix->rows16.release();
    ix->q16.release();
    ix->coarse_s.release();
    ix->coarse_i.release();
    ix->flag.release();
    ix->stats16.release();
    for (DevBuf* b : {&ix->ts_lmax, &ix->ts_tau, &ix->ts_count, &ix->ts_cs, &ix->ts_ci, &ix->i8c_cs,
                      &ix->i8c_ci, &ix->i8c_count, &ix->msel, &ix->mblk, &ix->mres_s, &ix->mres_i, &ix->rows8,
                      &ix->scale8, &ix->err8, &ix->stats8})
      b->release();
    ix->afb_q.release();
    ix->afb_cs.release();
    ix->afb_ci.release();
    ix->afb_total.release();
    if (ix->afb_host) (void)hipHostFree(ix->afb_host);
    if (ix->afb_event) (void)hipEventDestroy(ix->afb_event);
    for (int t = 0; t < 4; ++t) {
      ix->tier_fail[t].release();
      ix->tier_q[t].release();
      ix->tier_s[t].release();
      ix->tier_i[t].release();
    }
  }
  delete ix;
  return MQ_OK;
}

int mq_index_size(const mq_index* ix, int64_t* n_rows) {
  clear_error();
  MQ_CHECK_ARG(ix && n_rows, "NULL argument");
  *n_rows = ix->n;
  return MQ_OK;
}

int mq_index_dim(const mq_index* ix, int* dim) {
  clear_error();
  MQ_CHECK_ARG(ix && dim, "NULL argument");
  *dim = ix->dim;
  return MQ_OK;
}

int mq_index_data(mq_index* ix, void** device_rows) {
  clear_error();
  MQ_CHECK_ARG(ix && device_rows, "NULL argument");
  *device_rows = ix->rows;
  return MQ_OK;
}

int mq_index_reset(mq_index* ix) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->n = 0;
  ix->n16 = 0;
  ix->n8 = 0;
  return MQ_OK;
}

int mq_index_add(mq_index* ix, const float* rows, int64_t n, int rows_on_device, void* stream) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(n >= 0, "negative row count");
  if (n == 0) return MQ_OK;
  MQ_CHECK_ARG(rows, "NULL rows");
  MQ_CHECK_ARG(ix->n + n < (int64_t)INT32_MAX, "index limited to 2^31-1 rows");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = reserve_rows(ix, ix->n + n, s);
  if (rc) return rc;
  const int64_t chunk =
      rows_on_device ? n : std::max<int64_t>(1, std::min<int64_t>(n, (64ll << 20) / (ix->dim * 4)));
  for (int64_t r0 = 0; r0 < n; r0 += chunk) {
    const int64_t nr = std::min(chunk, n - r0);
    const float* src = rows + r0 * ix->dim;
    if (!rows_on_device) {
      rc = ix->stage.ensure((size_t)nr * ix->dim * 4);
      if (rc) return rc;
      MQ_HIP(hipMemcpyAsync(ix->stage.p, src, (size_t)nr * ix->dim * 4, hipMemcpyHostToDevice, s));
      src = ix->stage.as<float>();
    }
    hipLaunchKernelGGL(add_rows_kernel, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, s, src,
                       ix->rows + (ix->n + r0) * ix->dim, nr, ix->dim);
    MQ_HIP(hipGetLastError());
    if (!rows_on_device) MQ_HIP(hipStreamSynchronize(s));
  }
  ix->n += n;
  return MQ_OK;
}

int mq_index_select(mq_index* src, const int64_t* rows, int64_t n, mq_index* dst) {
  clear_error();
  MQ_CHECK_ARG(src && dst, "NULL index");
  MQ_CHECK_ARG(n >= 0 && (n == 0 || rows), "bad row list");
  MQ_CHECK_ARG(src->dim == dst->dim, "dim mismatch (%d vs %d)", src->dim, dst->dim);
  MQ_CHECK_ARG(src->device == dst->device, "indexes live on different devices");
  std::unique_lock<std::mutex> l1(src->mu, std::defer_lock), l2(dst->mu, std::defer_lock);
  if (src == dst)
    l1.lock();
  else
    std::lock(l1, l2);
  for (int64_t i = 0; i < n; ++i)
    MQ_CHECK_ARG(rows[i] >= 0 && rows[i] < src->n, "row %lld out of range (n=%lld)",
                 (long long)rows[i], (long long)src->n);
  DeviceGuard dg(src->device);
  // gather straight into dst's slab when it is a different index with room (a reused
  // scratch index for filtered searches: no allocation); else into a fresh slab
  const bool in_place_slab = src != dst && dst->rows && dst->cap >= n;
  float* fresh = nullptr;
  if (n > 0) {
    int rc = src->sel.ensure((size_t)n * sizeof(int64_t));
    if (rc) return rc;
    if (!in_place_slab && hipMalloc((void**)&fresh, (size_t)n * src->dim * sizeof(float)) != hipSuccess)
      MQ_FAIL(MQ_ENOMEM, "hipMalloc of %lld rows failed", (long long)n);
    hipError_t e = hipMemcpy(src->sel.p, rows, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, nullptr,
                         src->rows, src->sel.as<int64_t>(), n, src->dim, in_place_slab ? dst->rows : fresh);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
      if (fresh) (void)hipFree(fresh);
      MQ_FAIL(MQ_EHIP, "row gather failed: %s", hipGetErrorString(e));
    }
  }
  if (!in_place_slab) {
    if (dst->rows) MQ_HIP(hipFree(dst->rows));
    dst->rows = fresh;
    dst->cap = n;
  }
  dst->n = n;
  dst->n16 = 0;
  dst->n8 = 0;
  return MQ_OK;
}

// Filtered exact search (Chroma's similarity_search(filter=), src/medical_engine.py:52):
// every row whose mask bit is unset is absent from the scan.  Paths:
//  * one query: the int8 certified screen (K9q) with the mask - masked rows do not exist
//    for its sample, appending pass or certificate;
//  * a batch of > 64 queries (k <= 16): the bf16 threshold scan (K9t) with the mask, fp32
//    re-rank and certificate, as the unfiltered batched screen;
//  * what neither certifies, and other batches: the streaming exact fp32 scan (K9s) with
//    the mask, 16 queries per launch (no gather of the allowed rows);
//  * dims the streaming scan does not take (dim % 64 != 0): the allowed rows compacted and
//    gathered into a scratch index that is released after the search.
// Synchronous.  `masked_gathers` counts the queries the screens did not certify.
int masked_stream(mq_index* ix, const float* q, int64_t nq, int k, const unsigned* bits, float* os, int64_t* oi,
                  hipStream_t s) {
  for (int64_t q0 = 0; q0 < nq; q0 += 16) {
    const int64_t nn = std::min<int64_t>(16, nq - q0);
    const int rc = scan_topk(ix, SCAN_STREAM, q + q0 * ix->dim, nn, k, os + q0 * k, oi + q0 * k, s, bits);
    if (rc) return rc;
  }
  return MQ_OK;
}

int masked_gather(mq_index* ix, const float* q, int k, const unsigned* bits, float* os, int64_t* oi,
                  hipStream_t s) {
  const int64_t n_words = (ix->n + 31) / 32;
  const int nb = (int)((n_words + 255) / 256);
  int rc = ix->msel.ensure((size_t)ix->n * sizeof(int64_t));
  if (!rc) rc = ix->mblk.ensure((size_t)(nb + 1) * sizeof(int));
  if (rc) return rc;
  int* blk = ix->mblk.as<int>();
  hipLaunchKernelGGL(mask_count_kernel, dim3(nb), dim3(256), 0, s, bits, ix->n, blk);
  hipLaunchKernelGGL(mask_scan_kernel, dim3(1), dim3(256), 0, s, blk, nb);
  hipLaunchKernelGGL(mask_compact_kernel, dim3(nb), dim3(256), 0, s, bits, ix->n, blk, ix->msel.as<int64_t>());
  MQ_HIP(hipGetLastError());
  int count = 0;
  rc = read_flag(ix, blk + nb, s, &count);
  if (rc) return rc;
  if (count == 0) return fill_padding(os, oi, k, s);
  mq_index* sub = nullptr;
  rc = mq_index_create(ix->device, ix->dim, 0, ix->dtype, &sub);
  if (rc) return rc;
  rc = reserve_rows(sub, count, s);
  if (!rc) {
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((count + 3) / 4)), dim3(256), 0, s, ix->rows,
                       ix->msel.as<int64_t>(), (int64_t)count, ix->dim, sub->rows);
    if (hipGetLastError() != hipSuccess) rc = MQ_EHIP;
  }
  sub->n = count;
  const int kk = (int)std::min<int64_t>(k, count);
  if (!rc && kk < k) rc = fill_padding(os, oi, k, s);
  if (!rc) rc = ix->out_s.ensure((size_t)k * 4);
  if (!rc) rc = ix->out_i.ensure((size_t)k * 8);
  // (kk results into scratch, then into the first kk slots)
  if (!rc) rc = search_direct(sub, q, 1, kk, ix->out_s.as<float>(), ix->out_i.as<int64_t>(), s);
  if (!rc) {
    hipLaunchKernelGGL(remap_ids_kernel, dim3(1), dim3(256), 0, s, ix->out_i.as<int64_t>(), (int64_t)kk,
                       ix->msel.as<int64_t>());
    if (hipGetLastError() != hipSuccess) rc = MQ_EHIP;
  }
  if (!rc && hipMemcpyAsync(os, ix->out_s.p, (size_t)kk * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) rc = MQ_EHIP;
  if (!rc && hipMemcpyAsync(oi, ix->out_i.p, (size_t)kk * 8, hipMemcpyDeviceToDevice, s) != hipSuccess) rc = MQ_EHIP;
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = MQ_EHIP;
  mq_index_destroy(sub);  // the gathered copy is not kept (a wide filter's copy would rival the slab)
  if (rc == MQ_EHIP) MQ_FAIL(MQ_EHIP, "masked gather search failed");
  return rc;
}

int search_masked(mq_index* ix, const float* q, int k, const unsigned* bits, float* os, int64_t* oi,
                  hipStream_t s) {
  if (ix->n == 0) return fill_padding(os, oi, k, s);
  const bool exact_kind = ix->precision == MQ_DTYPE_F32_SCREEN || ix->precision == MQ_DTYPE_F32;
  if (exact_kind && k <= kScreenMaxK && ix->i8_screen && ix->dim % 256 == 0 && ix->dim <= 1024 &&
      ix->n >= kTsMinRows && ix->n < (1ll << 31)) {
    int rc = ix->flag.ensure(sizeof(int));
    if (!rc) rc = ix->tier_fail[TIER_I8].ensure(sizeof(int64_t));
    if (!rc) rc = i8_topk(ix, q, 1, MQ_MAX_K, nullptr, nullptr, s, ix->flag.as<int>(), k, bits);
    if (rc) return rc;
    hipLaunchKernelGGL(i8_finish_kernel, dim3(1), dim3(kFinT), 0, s, q, ix->rows, ix->dim, ix->ts_cs.as<float>(),
                       ix->ts_ci.as<int>(), ix->ts_count.as<int>(), i8_lists(ix->num_cus), ix->ts_tau.as<float>(),
                       k, ix->stats8.as<unsigned>(), ix->err8.as<float>(), os, oi, ix->flag.as<int>(),
                       ix->tier_fail[TIER_I8].as<int64_t>());
    ix->tl.close(s);
    MQ_HIP(hipGetLastError());
    int n_fail = 0;
    rc = read_flag(ix, ix->flag.as<int>(), s, &n_fail);
    if (rc) return rc;
    if (n_fail == 0) return MQ_OK;
    ix->masked_gathers++;
  }
  if (stream_ok(ix)) {
    const int rc = masked_stream(ix, q, 1, k, bits, os, oi, s);
    if (rc) return rc;
    MQ_HIP(hipStreamSynchronize(s));
    return MQ_OK;
  }
  return masked_gather(ix, q, k, bits, os, oi, s);
}

int search_masked_batch(mq_index* ix, const float* q, int64_t nq, int k, const unsigned* bits, float* os,
                        int64_t* oi, hipStream_t s) {
  if (ix->n == 0) return fill_padding(os, oi, nq * k, s);
  if (nq == 1) return search_masked(ix, q, k, bits, os, oi, s);
  const bool exact_kind = ix->precision == MQ_DTYPE_F32_SCREEN || ix->precision == MQ_DTYPE_F32;
  if (!stream_ok(ix)) {  // (dim % 64 != 0: no masked scan kernel takes it)
    for (int64_t j = 0; j < nq; ++j) {
      const int rc = search_masked(ix, q + j * ix->dim, k, bits, os + j * k, oi + j * k, s);
      if (rc) return rc;
    }
    return MQ_OK;
  }
  if (!(exact_kind && k <= kScreenMaxK && thresh_ok(ix, nq) && ix->dim <= 1024)) {
    const int rc = masked_stream(ix, q, nq, k, bits, os, oi, s);
    if (rc) return rc;
    MQ_HIP(hipStreamSynchronize(s));
    return MQ_OK;
  }
  // the batched bf16 screen with the mask (search_screened's TIER_BF16, synchronous)
  const int kc = (int)std::min<int64_t>(MQ_MAX_K, ix->n);
  int rc = ensure_shadow(ix, s);
  if (!rc) rc = queries_to_bf16(ix, q, nq, s);
  if (!rc) rc = ix->coarse_s.ensure((size_t)nq * kc * sizeof(float));
  if (!rc) rc = ix->coarse_i.ensure((size_t)nq * kc * sizeof(int64_t));
  if (!rc) rc = ix->flag.ensure(sizeof(int));
  if (!rc) rc = ix->tier_fail[TIER_BF16].ensure((size_t)nq * sizeof(int64_t));
  if (rc) return rc;
  rc = thresh_topk(ix, ix->q16.as<float>(), nq, kc, ix->coarse_s.as<float>(), ix->coarse_i.as<int64_t>(), s,
                   kTsRank, nullptr, nullptr, bits);
  if (rc) return rc;
  const unsigned* stats = ix->stats16.as<unsigned>();
  hipLaunchKernelGGL(rerank_kernel, dim3((unsigned)nq), dim3(256), 0, s, q, ix->rows, ix->dim,
                     ix->coarse_i.as<int64_t>(), kc, k, os, oi, ix->coarse_s.as<float>(), VERIFY_BF16_Q16, stats);
  MQ_HIP(hipMemsetAsync(ix->flag.p, 0, sizeof(int), s));
  int64_t* fail = ix->tier_fail[TIER_BF16].as<int64_t>();
  hipLaunchKernelGGL(screen_verify_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, s, q, ix->dim,
                     ix->coarse_s.as<float>(), kc, os, k, nq, VERIFY_BF16_Q16, stats, ix->flag.as<int>(), fail,
                     nullptr);
  MQ_HIP(hipGetLastError());
  int n_fail = 0;
  rc = read_flag(ix, ix->flag.as<int>(), s, &n_fail);
  if (rc) return rc;
  if (n_fail > 0) {  // uncertified: the masked exact scan, results scattered back
    ix->masked_gathers += n_fail;
    rc = ix->tier_q[TIER_BF16].ensure((size_t)n_fail * ix->dim * sizeof(float));
    if (!rc) rc = ix->tier_s[TIER_BF16].ensure((size_t)n_fail * k * sizeof(float));
    if (!rc) rc = ix->tier_i[TIER_BF16].ensure((size_t)n_fail * k * sizeof(int64_t));
    if (rc) return rc;
    float* sq = ix->tier_q[TIER_BF16].as<float>();
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n_fail + 3) / 4)), dim3(256), 0, s, q, fail,
                       (int64_t)n_fail, ix->dim, sq);
    MQ_HIP(hipGetLastError());
    rc = masked_stream(ix, sq, n_fail, k, bits, ix->tier_s[TIER_BF16].as<float>(),
                       ix->tier_i[TIER_BF16].as<int64_t>(), s);
    if (rc) return rc;
    const int64_t total = (int64_t)n_fail * k;
    hipLaunchKernelGGL(scatter_results_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       ix->tier_s[TIER_BF16].as<float>(), ix->tier_i[TIER_BF16].as<int64_t>(), fail,
                       (int64_t)n_fail, k, os, oi);
    MQ_HIP(hipGetLastError());
  }
  MQ_HIP(hipStreamSynchronize(s));
  return MQ_OK;
}

// Device of a pointer (HIP device memory), or -1 (host / unknown).
int pointer_device(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return a.type == hipMemoryTypeDevice ? a.device : -1;
}

int mq_mask_eval(const int32_t* codes, int64_t n, const uint8_t* lut, int n_lut, uint32_t* bits, int mode,
                 void* stream) {
  clear_error();
  MQ_CHECK_ARG(n >= 0 && n_lut >= 1, "bad mask shape");
  MQ_CHECK_ARG(mode == MQ_MASK_SET || mode == MQ_MASK_AND || mode == MQ_MASK_OR, "bad mask mode %d", mode);
  if (n == 0) return MQ_OK;
  MQ_CHECK_ARG(codes && lut && bits, "NULL buffer");
  const int dev = pointer_device(bits);
  MQ_CHECK_ARG(dev >= 0 && pointer_device(codes) == dev && pointer_device(lut) == dev,
               "codes, lut and bits must be device memory of one GPU");
  DeviceGuard dg(dev);  // the launch runs on the buffers' GPU (stream: that device's)
  hipLaunchKernelGGL(mask_eval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const int*)codes, n, (const unsigned char*)lut, LutWords{}, n_lut, (unsigned*)bits, mode);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_mask_eval_bits(const int32_t* codes, int64_t n, const uint64_t* lut_words, int n_lut, uint32_t* bits,
                      int mode, void* stream) {
  clear_error();
  MQ_CHECK_ARG(n >= 0 && n_lut >= 1 && n_lut <= 256, "n_lut must be in [1, 256]");
  MQ_CHECK_ARG(mode == MQ_MASK_SET || mode == MQ_MASK_AND || mode == MQ_MASK_OR, "bad mask mode %d", mode);
  MQ_CHECK_ARG(lut_words, "NULL table");
  if (n == 0) return MQ_OK;
  MQ_CHECK_ARG(codes && bits, "NULL buffer");
  const int dev = pointer_device(bits);
  MQ_CHECK_ARG(dev >= 0 && pointer_device(codes) == dev, "codes and bits must be device memory of one GPU");
  DeviceGuard dg(dev);
  LutWords lw{};
  for (int i = 0; i < (n_lut + 63) / 64; ++i) lw.w[i] = lut_words[i];
  hipLaunchKernelGGL(mask_eval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const int*)codes, n, (const unsigned char*)nullptr, lw, n_lut, (unsigned*)bits, mode);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_mask_combine(uint32_t* dst, const uint32_t* src, int64_t n_words, int mode, void* stream) {
  clear_error();
  MQ_CHECK_ARG(n_words >= 0, "negative word count");
  MQ_CHECK_ARG(mode >= MQ_MASK_SET && mode <= MQ_MASK_CLEAR, "bad mask mode %d", mode);
  if (n_words == 0) return MQ_OK;
  MQ_CHECK_ARG(dst, "NULL dst");
  const int dev = pointer_device(dst);
  MQ_CHECK_ARG(dev >= 0 && (!src || pointer_device(src) == dev), "dst and src must be device memory of one GPU");
  DeviceGuard dg(dev);
  hipLaunchKernelGGL(mask_combine_kernel, dim3((unsigned)((n_words + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (unsigned*)dst, (const unsigned*)src, n_words, mode);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_index_search_masked_batch(mq_index* ix, const float* queries, int64_t nq, int k, const uint32_t* bits,
                                 float* out_scores, int64_t* out_ids, int io_on_device, void* stream) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(nq >= 0 && nq <= (1ll << 24), "query count %lld out of range", (long long)nq);
  MQ_CHECK_ARG(k >= 1 && k <= MQ_MAX_K, "k must be in [1, %d] (got %d)", MQ_MAX_K, k);
  if (nq == 0) return MQ_OK;
  MQ_CHECK_ARG(queries && bits && out_scores && out_ids, "NULL buffer");
  std::lock_guard<std::mutex> lk(ix->mu);
  MQ_CHECK_ARG(pointer_device(bits) == ix->device, "the mask must be device memory of the index's GPU %d",
               ix->device);
  DeviceGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  if (io_on_device) return search_masked_batch(ix, queries, nq, k, (const unsigned*)bits, out_scores, out_ids, s);
  const size_t qb = (size_t)nq * ix->dim * 4, sb = (size_t)nq * k * 4, ib = (size_t)nq * k * 8;
  int rc = ix->stage.ensure(qb);
  if (!rc) rc = ix->mres_s.ensure(sb);
  if (!rc) rc = ix->mres_i.ensure(ib);
  if (!rc) rc = ix->pin.ensure(qb + sb + ib);  // pinned staging (see mq_index_search)
  if (rc) return rc;
  unsigned char* hp = ix->pin.as<unsigned char>();
  memcpy(hp, queries, qb);
  MQ_HIP(hipMemcpyAsync(ix->stage.p, hp, qb, hipMemcpyHostToDevice, s));
  rc = search_masked_batch(ix, ix->stage.as<float>(), nq, k, (const unsigned*)bits, ix->mres_s.as<float>(),
                           ix->mres_i.as<int64_t>(), s);
  if (rc) return rc;
  MQ_HIP(hipMemcpyAsync(hp + qb, ix->mres_s.p, sb, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipMemcpyAsync(hp + qb + sb, ix->mres_i.p, ib, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipStreamSynchronize(s));
  memcpy(out_scores, hp + qb, sb);
  memcpy(out_ids, hp + qb + sb, ib);
  return MQ_OK;
}

int mq_index_search_masked(mq_index* ix, const float* query, int k, const uint32_t* bits, float* out_scores,
                           int64_t* out_ids, int io_on_device, void* stream) {
  return mq_index_search_masked_batch(ix, query, 1, k, bits, out_scores, out_ids, io_on_device, stream);
}

int mq_index_masked_gathers(const mq_index* ix, int64_t* count) {
  clear_error();
  MQ_CHECK_ARG(ix && count, "NULL argument");
  std::lock_guard<std::mutex> lk(const_cast<mq_index*>(ix)->mu);
  *count = ix->masked_gathers;
  return MQ_OK;
}

int mq_index_search(mq_index* ix, const float* queries, int64_t nq, int k, float* out_scores,
                    int64_t* out_ids, int io_on_device, void* stream) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(nq >= 0 && nq <= (1ll << 24), "query count %lld out of range", (long long)nq);
  MQ_CHECK_ARG(k >= 1 && k <= MQ_MAX_K, "k must be in [1, %d] (got %d)", MQ_MAX_K, k);
  if (nq == 0) return MQ_OK;
  MQ_CHECK_ARG(queries && out_scores && out_ids, "NULL buffer");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  if (io_on_device) return search_device(ix, queries, nq, k, out_scores, out_ids, s);
  const size_t qb = (size_t)nq * ix->dim * 4, sb = (size_t)nq * k * 4, ib = (size_t)nq * k * 8;
  int rc = ix->stage.ensure(qb);
  if (!rc) rc = ix->out_s.ensure(sb);
  if (!rc) rc = ix->out_i.ensure(ib);
  // pinned staging for the few-query path (a batch's bytes go pageable: the copy dominates
  // neither way, and the pinned buffer stays small)
  const bool pin = qb <= (1u << 20);
  if (!rc && pin) rc = ix->pin.ensure(qb + sb + ib);
  if (rc) return rc;
  unsigned char* hp = ix->pin.as<unsigned char>();
  if (pin) {
    memcpy(hp, queries, qb);
    MQ_HIP(hipMemcpyAsync(ix->stage.p, hp, qb, hipMemcpyHostToDevice, s));
  } else {
    MQ_HIP(hipMemcpyAsync(ix->stage.p, queries, qb, hipMemcpyHostToDevice, s));
  }
  rc = search_device(ix, ix->stage.as<float>(), nq, k, ix->out_s.as<float>(),
                     ix->out_i.as<int64_t>(), s);
  if (rc) return rc;
  MQ_HIP(hipMemcpyAsync(pin ? (void*)(hp + qb) : (void*)out_scores, ix->out_s.p, sb, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipMemcpyAsync(pin ? (void*)(hp + qb + sb) : (void*)out_ids, ix->out_i.p, ib, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipStreamSynchronize(s));
  if (pin) {
    memcpy(out_scores, hp + qb, sb);
    memcpy(out_ids, hp + qb + sb, ib);
  }
  return MQ_OK;
}

int mq_debug_int8_screen(mq_index* ix, const float* query, int kc, float* out_scores, int64_t* out_ids,
                         float* stats) {
  clear_error();
  MQ_CHECK_ARG(ix && query && out_scores && out_ids && stats, "NULL argument");
  MQ_CHECK_ARG(kc >= 1 && kc <= MQ_MAX_K, "kc must be in [1, %d]", MQ_MAX_K);
  MQ_CHECK_ARG(ix->dim % 256 == 0 && ix->dim <= 1024 && ix->n >= 1, "int8 screen needs dim 256..1024, rows");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  hipStream_t s = nullptr;
  int rc = ix->stage.ensure((size_t)ix->dim * 4);
  if (!rc) rc = ix->out_s.ensure((size_t)kc * 4);
  if (!rc) rc = ix->out_i.ensure((size_t)kc * 8);
  if (rc) return rc;
  MQ_HIP(hipMemcpyAsync(ix->stage.p, query, (size_t)ix->dim * 4, hipMemcpyHostToDevice, s));
  rc = i8_topk(ix, ix->stage.as<float>(), 1, kc, ix->out_s.as<float>(), ix->out_i.as<int64_t>(), s);
  ix->tl.close(s);
  if (rc) return rc;
  MQ_HIP(hipMemcpyAsync(out_scores, ix->out_s.p, (size_t)kc * 4, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipMemcpyAsync(out_ids, ix->out_i.p, (size_t)kc * 8, hipMemcpyDeviceToHost, s));
  MQ_HIP(hipMemcpyAsync(stats, ix->stats8.p, 2 * sizeof(float), hipMemcpyDeviceToHost, s));
  MQ_HIP(hipStreamSynchronize(s));
  return MQ_OK;
}

int mq_index_get(mq_index* ix, int64_t row0, int64_t n, float* out, int out_on_device,
                 void* stream) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(row0 >= 0 && n >= 0 && row0 + n <= ix->n, "rows [%lld, %lld) out of range (n=%lld)",
               (long long)row0, (long long)(row0 + n), (long long)ix->n);
  if (n == 0) return MQ_OK;
  MQ_CHECK_ARG(out, "NULL output");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  hipStream_t s = (hipStream_t)stream;
  MQ_HIP(hipMemcpyAsync(out, ix->rows + row0 * ix->dim, (size_t)n * ix->dim * 4,
                        out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
  if (!out_on_device) MQ_HIP(hipStreamSynchronize(s));
  return MQ_OK;
}

int mq_index_set_precision(mq_index* ix, int dtype) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(dtype == MQ_DTYPE_F32 || dtype == MQ_DTYPE_F32X6 || dtype == MQ_DTYPE_BF16 ||
                   dtype == MQ_DTYPE_F32_SCREEN,
               "search precision must be MQ_DTYPE_F32, _F32X6, _BF16 or _F32_SCREEN (got %d)", dtype);
  MQ_CHECK_ARG(dtype != MQ_DTYPE_BF16 || ix->dim % 64 == 0, "bf16 coarse scan needs dim %% 64 == 0");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->precision = dtype;
  return MQ_OK;
}

int mq_index_set_stream_threshold(mq_index* ix, int max_queries) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  MQ_CHECK_ARG(max_queries >= 0 && max_queries <= 16, "stream threshold must be in [0, 16] (got %d)",
               max_queries);
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->stream_max_q = max_queries;
  return MQ_OK;
}

int mq_index_set_threshold_scan(mq_index* ix, int enabled) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->thresh_scan = enabled != 0;
  return MQ_OK;
}

int mq_index_set_int8_screen(mq_index* ix, int enabled) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->i8_screen = enabled != 0;
  ix->i8_skip = 0;
  ix->i8_fail_avg = 0.0;
  return MQ_OK;
}

// Blocks until the count copy of the last asynchronous screened search has landed (that
// search's stream only - not a device-wide sync), then folds it in.
int mq_index_screen_fallbacks(const mq_index* cix, int64_t* to_direct, int64_t* to_split) {
  clear_error();
  MQ_CHECK_ARG(cix, "NULL argument");
  mq_index* ix = const_cast<mq_index*>(cix);  // the counters are folded in under the lock
  // The wait runs WITHOUT the lock: a counter read must not block searches on
  // other threads until the last asynchronous batch lands.  Take the event under the lock,
  // wait, then re-lock to fold the count in; a search recorded meanwhile re-records the
  // event, so the count is exact as of the wait (eventually consistent after it).
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    ev = ix->afb_event;
  }
  if (ev) {
    DeviceGuard dg(ix->device);
    MQ_HIP(hipEventSynchronize(ev));
  }
  std::lock_guard<std::mutex> lk(ix->mu);
  poll_async_fallbacks(ix);
  if (to_direct) *to_direct = ix->screen_fallbacks;
  if (to_split) *to_split = ix->screen_passdowns;
  return MQ_OK;
}

int mq_index_screen_skips(const mq_index* cix, int64_t* bf16_skips, int64_t* int8_skips) {
  clear_error();
  MQ_CHECK_ARG(cix, "NULL argument");
  mq_index* ix = const_cast<mq_index*>(cix);  // read under the lock, as its sibling getters
  std::lock_guard<std::mutex> lk(ix->mu);
  if (bf16_skips) *bf16_skips = ix->bf_skips;
  if (int8_skips) *int8_skips = ix->i8_skips;
  return MQ_OK;
}

int mq_index_set_async_screen(mq_index* ix, int enabled) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->async_screen = enabled != 0;
  ix->sync_left = 0;
  ix->bf_skip = 0;
  ix->bf_fail_avg = 0.0;
  return MQ_OK;
}

int mq_index_rescans(const mq_index* ix, int64_t* rescans, int64_t* remerges) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL argument");
  if (rescans) *rescans = ix->rescans;
  if (remerges) *remerges = ix->remerges;
  return MQ_OK;
}

int mq_index_set_timing(mq_index* ix, int enabled) {
  clear_error();
  MQ_CHECK_ARG(ix, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  ix->tl.drain();
  ix->tl.on = enabled != 0;
  return MQ_OK;
}

int mq_index_read_timing(mq_index* ix, float* ms, int n) {
  clear_error();
  MQ_CHECK_ARG(ix && ms && n >= 0, "bad argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  ix->tl.read(ms, n);
  return MQ_OK;
}

// rows [row0, row0 + n) as a slab file (header + rows), flushed to stable storage
static int save_rows(mq_index* ix, const char* path, int64_t row0, int64_t n) {
  FILE* f = fopen(path, "wb");
  if (!f) MQ_FAIL(MQ_EIO, "cannot open %s for writing", path);
  FileHeader h;
  memcpy(h.magic, kMagic, 8);
  h.dim = ix->dim;
  h.dtype = ix->dtype;
  h.n_rows = n;
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (ix->dim * 4));
  std::vector<float> buf;
  for (int64_t r0 = 0; ok && r0 < n; r0 += chunk) {
    const int64_t nr = std::min(chunk, n - r0);
    buf.resize((size_t)nr * ix->dim);
    if (hipMemcpy(buf.data(), ix->rows + (row0 + r0) * ix->dim, buf.size() * 4, hipMemcpyDeviceToHost) !=
        hipSuccess) {
      fclose(f);
      MQ_FAIL(MQ_EHIP, "device->host copy failed while saving");
    }
    ok = fwrite(buf.data(), 4, buf.size(), f) == buf.size();
  }
  ok = ok && fflush(f) == 0 && fsync(fileno(f)) == 0;
  ok = (fclose(f) == 0) && ok;
  if (!ok) MQ_FAIL(MQ_EIO, "short write to %s", path);
  return MQ_OK;
}

// the rows of slab file `path` placed at row `at` (0: replace the index, ix->n: append)
static int load_rows(mq_index* ix, const char* path, bool append) {
  FILE* f = fopen(path, "rb");
  if (!f) MQ_FAIL(MQ_EIO, "cannot open %s", path);
  FileHeader h;
  if (fread(&h, sizeof(h), 1, f) != 1 || memcmp(h.magic, kMagic, 8) != 0) {
    fclose(f);
    MQ_FAIL(MQ_EIO, "%s is not an mq flat index file", path);
  }
  if (h.dim != ix->dim || h.dtype != ix->dtype || h.n_rows < 0) {
    fclose(f);
    MQ_FAIL(MQ_EINVAL, "%s holds dim %d dtype %d, index has dim %d dtype %d", path, h.dim, h.dtype,
            ix->dim, ix->dtype);
  }
  const int64_t at = append ? ix->n : 0;
  if (at + h.n_rows >= (int64_t)INT32_MAX) {
    fclose(f);
    MQ_FAIL(MQ_EINVAL, "index limited to 2^31-1 rows");
  }
  if (!append) {
    ix->n = 0;
    ix->n16 = 0;
    ix->n8 = 0;
  }
  int rc = reserve_rows(ix, at + h.n_rows, nullptr);
  if (rc) {
    fclose(f);
    return rc;
  }
  const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (ix->dim * 4));
  std::vector<float> buf;
  for (int64_t r0 = 0; r0 < h.n_rows; r0 += chunk) {
    const int64_t nr = std::min(chunk, h.n_rows - r0);
    buf.resize((size_t)nr * ix->dim);
    if (fread(buf.data(), 4, buf.size(), f) != buf.size()) {
      fclose(f);
      MQ_FAIL(MQ_EIO, "%s is truncated", path);
    }
    if (hipMemcpy(ix->rows + (at + r0) * ix->dim, buf.data(), buf.size() * 4, hipMemcpyHostToDevice) !=
        hipSuccess) {
      fclose(f);
      MQ_FAIL(MQ_EHIP, "host->device copy failed while loading");
    }
  }
  fclose(f);
  ix->n = at + h.n_rows;  // rows were normalised before they were saved (the shadows extend lazily)
  return MQ_OK;
}

int mq_index_save(mq_index* ix, const char* path) {
  clear_error();
  MQ_CHECK_ARG(ix && path, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  return save_rows(ix, path, 0, ix->n);
}

int mq_index_save_rows(mq_index* ix, const char* path, int64_t row0, int64_t n) {
  clear_error();
  MQ_CHECK_ARG(ix && path, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  MQ_CHECK_ARG(row0 >= 0 && n >= 0 && row0 + n <= ix->n, "rows [%lld, %lld) outside [0, %lld)",
               (long long)row0, (long long)(row0 + n), (long long)ix->n);
  DeviceGuard dg(ix->device);
  return save_rows(ix, path, row0, n);
}

int mq_index_load(mq_index* ix, const char* path) {
  clear_error();
  MQ_CHECK_ARG(ix && path, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  return load_rows(ix, path, false);
}

int mq_index_load_append(mq_index* ix, const char* path) {
  clear_error();
  MQ_CHECK_ARG(ix && path, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard dg(ix->device);
  return load_rows(ix, path, true);
}

int mq_topk_merge_device(const float* scores, const int64_t* ids, int n_lists, int64_t nq,
                         int k_in, int k_out, float* out_scores, int64_t* out_ids, void* stream) {
  clear_error();
  MQ_CHECK_ARG(n_lists >= 1 && nq >= 0 && k_in >= 1, "bad merge shape");
  MQ_CHECK_ARG(k_out >= 1 && k_out <= MQ_MAX_K, "k_out must be in [1, %d]", MQ_MAX_K);
  if (nq == 0) return MQ_OK;
  MQ_CHECK_ARG(scores && ids && out_scores && out_ids, "NULL buffer");
  merge_dispatch<int64_t>(scores, ids, n_lists, nq, k_in, k_out, out_scores, out_ids,
                          (hipStream_t)stream);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_topk_merge_host(const float* scores, const int64_t* ids, int n_lists, int64_t nq, int k_in,
                       int k_out, float* out_scores, int64_t* out_ids) {
  clear_error();
  MQ_CHECK_ARG(n_lists >= 1 && nq >= 0 && k_in >= 1 && k_out >= 1, "bad merge shape");
  if (nq == 0) return MQ_OK;
  MQ_CHECK_ARG(scores && ids && out_scores && out_ids, "NULL buffer");
  auto better_h = [](float sa, int64_t ia, float sb, int64_t ib) {
    return sa > sb || (sa == sb && (uint64_t)ia < (uint64_t)ib);
  };
  std::vector<std::pair<float, int64_t>> pool;
  for (int64_t q = 0; q < nq; ++q) {
    pool.clear();
    for (int l = 0; l < n_lists; ++l) {
      const int64_t base = ((int64_t)l * nq + q) * k_in;
      for (int j = 0; j < k_in; ++j)
        if (ids[base + j] >= 0) pool.emplace_back(scores[base + j], ids[base + j]);
    }
    const size_t take = std::min<size_t>(pool.size(), (size_t)k_out);
    std::partial_sort(pool.begin(), pool.begin() + take, pool.end(),
                      [&](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) {
                        return better_h(a.first, a.second, b.first, b.second);
                      });
    for (int j = 0; j < k_out; ++j) {
      const bool have = (size_t)j < take;
      out_scores[q * k_out + j] = have ? pool[j].first : -INFINITY;
      out_ids[q * k_out + j] = have ? pool[j].second : -1;
    }
  }
  return MQ_OK;
}

}  // extern "C"
