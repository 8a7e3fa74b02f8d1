// encoder.hip - BERT-base encoder forward for gfx950 (K1..K7) and the mq_encoder_* ABI.
//
// Replaces the embedding model behind OllamaEmbeddings("shaw/dmeta-embedding-zh")
// (reference src/medical_engine.py:43, src/ingest_medical.py:104): token ids ->
// 12 x [self-attention + FFN] post-LN BERT layers -> CLS (or mean) pool -> L2 norm.
//
// Kernels (one forward = 1 + 7*layers + 1 launches):
//   K1 embed_ln_kernel      word + position + type-0 embedding gather, LayerNorm
//   K2 gemm (EPI_BIAS)      fused QKV projection          [M,H] x [3H,H]^T
//   K3 attention_kernel     softmax(QK^T/sqrt(dh) + mask) V, online softmax, LDS tiles
//   K4 gemm (EPI_RESID)     output projection + bias + residual, then ln_kernel
//   K5 gemm (EPI_GELU)      FFN up + bias + GELU (erf or tanh)
//   K6 gemm (EPI_RESID)     FFN down + bias + residual, then ln_kernel
//   K7 pool_kernel          CLS / masked-mean pooling + L2 normalisation
// All GEMMs run on the exact-fp32 MFMA core of gemm_f32.hpp (or its split-f32 form).
// Few token rows (a single query, B * L <= 64) take forward_rows instead: 5 launches per
// layer on the K2r / K3r kernels below, LayerNorm applied by the consuming GEMM.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "gemm_epi.hpp"
#include "gemm_f32.hpp"
#include "gemm_x6p.hpp"

namespace mq {


// LayerNorm deferred into the consumer (batched path, MQ_ENC_OPT_LN_ON_LOAD).  The
// residual GEMM (out-proj / FFN-down, EPI_RESID_STATS) writes y = A W^T + b + resid and,
// per row and per wave tile of kLnPartW columns, the partial (mean, M2) of y: stats[row][t].
// The next GEMM (FFN-up / the next layer's QKV, LN_IN) merges a row's partials into (mean,
// rstd) once per tile (Chan: M2 = sum M2_t + w sum (mean_t - mean)^2, equal counts w) and
// normalises every A element between its global load and its LDS write, (y - mean) rstd
// gamma + beta; the tiles of column 0 also store LN(y) to x, the residual input of the
// following residual GEMM.  No LayerNorm launch and no y -> x round trip.  Two-pass-class
// statistics in fp32; ln_kernel's summation order differs (results agree to rounding).
constexpr int kLnPartW = 96;   // columns per partial: the producer's wave tile (F32Tile<4,1,1,3>)
constexpr int kLnMaxParts = 8;  // partials per row: the path runs at H = 768 (BERT-base)
struct LnArgs {
  float* stats_out;       // producer: [M][nt] (mean, M2) pairs
  const float* stats_in;  // consumer: the producer's pairs for A's rows
  const float* g;         // consumer: LayerNorm gamma [K]
  const float* b;         //           beta [K]
  float* xout;            //           column-0 tiles store LN(A) rows here
  int ldx;
  int nt;                 // partials per row (K / kLnPartW)
  float eps;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ------------------------------------------------------------------ GEMM -------
// out[M,N] = epi(A[M,K] . W[N,K]^T + bias[N] (+ resid[M,N])), K % 32 == 0.
// Row strides lda / ldr / ldo (in floats) let the CLS-only last layer run on every
// L-th row of the activations without a gather.
// Persistent: gridDim.x workgroups (a multiple of 8, two per CU) walk the tiles
// t = blockIdx.x, +gridDim.x, ...; the first K-slice of the next tile is fetched during
// the last slice of the current one, so the epilogue overlaps the next tile's loads.
// Within a round, the workgroups of one XCD (blockIdx % 8 equal) take consecutive
// tiles, i.e. share A row panels in their L2.
// LN_IN: the consumer side of LnArgs, as walk_tiles_hooked hooks.  Per tile, threads t <
// BM load row m0 + t's partials with the tile's first slice (issue), merge them into
// (mean, rstd) in LDS at that iteration's store phase (prepare; two slots by tile parity),
// and every A slot is normalised on its registers before the LDS write (xform).  A slot's
// row and 16-B chunk are fixed per thread (THREADS % F4_PER_ROW == 0), so gamma / beta are
// one float4 each per slice, loaded with the slice.
// MQ_LN_DIAG (measurement builds only): 1 = the hooks stage nothing (no partial / gamma /
// beta loads, no normalisation: wrong results) - the hooked walker's own cost; 2 = loads
// kept, normalisation skipped.
#ifndef MQ_LN_DIAG
#define MQ_LN_DIAG 0
#endif
#if MQ_LN_DIAG != 0 && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_LN_DIAG computes wrong results: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
#endif

template <class T, class Coords>
struct LnInHooks {
  static constexpr int A_LOADS = T::BM * T::F4_PER_ROW / T::THREADS;
  static_assert(T::A_SLOTS && T::THREADS % T::F4_PER_ROW == 0, "A slots: fixed row chunk per thread");
  const LnArgs& ln;
  Coords& coords;
  float2* st;  // LDS [2][BM] (mean, rstd)
  int M, nk, S;
  float inv_k;
  FastDiv nkd;
  float2 part[kLnMaxParts];
  floatx4 gg[T::PF], bb[T::PF];
  float2 mr[A_LOADS];  // (mean, rstd) of this thread's A rows for the slice being stored
  template <class DC>
  __device__ __forceinline__ void issue(int s, DC) {
    if constexpr (MQ_LN_DIAG == 1) return;
    constexpr int d = DC::value;
    const int sc = s < S ? s : S - 1;
    const int i = nkd.div(sc), kt = sc - i * nk;
    const int k = kt * T::BK + (threadIdx.x % T::F4_PER_ROW) * 4;
    gg[d] = *reinterpret_cast<const floatx4*>(ln.g + k);
    bb[d] = *reinterpret_cast<const floatx4*>(ln.b + k);
    // (coords outside any per-thread branch: a tile origin computed under divergent control
    // flow turns the staging's buffer descriptors into VGPRs - waterfall loops per load)
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    // the partials of the fetched slice's tile rows, loaded with EVERY slice (64 B per
    // thread from L2; rows past BM repeat): loaded only at tile starts, the registers
    // would merge two values at the join and the copy would wait for the loads right there
    const float2* src = reinterpret_cast<const float2*>(ln.stats_in) +
                        (int64_t)min(m0 + (int)threadIdx.x % T::BM, M - 1) * kLnMaxParts;
#pragma unroll
    for (int t = 0; t < kLnMaxParts; ++t) part[t] = src[t];
  }
  __device__ __forceinline__ void prepare(int s) {
    if constexpr (MQ_LN_DIAG == 1) return;
    if (s >= S || nkd.mod(s) != 0) return;  // workgroup-uniform
    // the merge must stay here, after the slice's MFMAs: left alone the compiler folds it
    // into issue()'s equal-condition block and waits there for the partials' loads
#pragma unroll
    for (int t = 0; t < kLnMaxParts; ++t) asm volatile("" : "+v"(part[t].x), "+v"(part[t].y));
    float mean = 0.f;
#pragma unroll
    for (int t = 0; t < kLnMaxParts; ++t) mean += part[t].x;
    mean *= 1.0f / (float)kLnMaxParts;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < kLnMaxParts; ++t) {
      const float dm = part[t].x - mean;
      m2 += part[t].y + (float)kLnPartW * dm * dm;
    }
    const float rstd = 1.0f / sqrtf(m2 * inv_k + ln.eps);
    if (threadIdx.x < T::BM) st[(nkd.div(s) & 1) * T::BM + threadIdx.x] = make_float2(mean, rstd);
  }
  // at the top of the iteration that stores slice s: its rows' (mean, rstd) from LDS, read
  // under the MFMAs
  __device__ __forceinline__ void stage_in(int s) {
    if constexpr (MQ_LN_DIAG == 1) return;
    const float2* ms = st + (nkd.div(s < S ? s : S - 1) & 1) * T::BM;
#pragma unroll
    for (int a = 0; a < A_LOADS; ++a) mr[a] = ms[((int)threadIdx.x + a * T::THREADS) / T::F4_PER_ROW];
  }
  template <class DC>
  __device__ __forceinline__ void xform(Stager<T>& sg, int s, DC) {
    if constexpr (MQ_LN_DIAG != 0) return;
    constexpr int d = DC::value;
#pragma unroll
    for (int a = 0; a < A_LOADS; ++a) sg.r[a] = (sg.r[a] - mr[a].x) * mr[a].y * gg[d] + bb[d];
    const int sc = s < S ? s : S - 1;
    const int i = nkd.div(sc), kt = sc - i * nk;
    int m0;
    int64_t n0;
    coords(i, m0, n0);
    if (n0 == 0 && s < S) {  // column-0 tiles: LN(A) rows out to x (workgroup-uniform)
      const int ch = threadIdx.x % T::F4_PER_ROW;
#pragma unroll
      for (int a = 0; a < A_LOADS; ++a) {
        // rows past M were staged from row M - 1 (clamped): they store row M - 1's own values
        const int r = min(m0 + ((int)threadIdx.x + a * T::THREADS) / T::F4_PER_ROW, M - 1);
        *reinterpret_cast<floatx4*>(ln.xout + (int64_t)r * ln.ldx + kt * T::BK + ch * 4) = sg.r[a];
      }
    }
  }
};

template <class T, int EPI, bool LN_IN = false>
__global__ __launch_bounds__(T::THREADS, T::WG_PER_CU) void gemm_nt_kernel(const float* __restrict__ A, int lda,
                                                         const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ resid, int ldr,
                                                         float* __restrict__ out, int ldo, int M,
                                                         int N, int K, LnArgs ln, int rx) {
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  __shared__ float2 ln_st[LN_IN ? 2 * T::BM : 1];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int tiles_n = (N + T::BN - 1) / T::BN, tiles_m = (M + T::BM - 1) / T::BM;
  const int G = gridDim.x, per_xcd = G >> 3;
  const int xslot = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  // rx > 0: region walk (gemm_x6p.hpp region_of): this XCD group's tiles, row-major in it
  Region rg{0, tiles_m, 0, tiles_n};
  int loc = xslot, wstep = G;
  if (rx > 0) {
    rg = region_of(rx, blockIdx.x & 7, tiles_m, tiles_n);
    loc = blockIdx.x >> 3;
    wstep = per_xcd;
  }
  const int rtiles = rg.rm * rg.rn;
  const int n_tiles = loc < rtiles ? (rtiles - loc + wstep - 1) / wstep : 0;
  const FastDiv tnd(rg.rn);
  auto coords = [&](int i, int& m0, int64_t& n0) {
    const int t = i * wstep + loc;
    const int tr = tnd.div(t);
    m0 = (rg.m_lo + tr) * T::BM;
    n0 = (int64_t)(rg.n_lo + t - tr * rg.rn) * T::BN;
  };
  auto epi = [&](int i, floatx16(&acc)[T::TM][T::TN], float*) {
    int m0;
    int64_t n0l;
    coords(i, m0, n0l);
    const int n0 = (int)n0l;
    if constexpr (EPI == EPI_RESID_STATS) {
      // y = acc + bias + resid, then per row the partial (mean, M2) of y over the wave
      // tile's WN = kLnPartW columns: the 32 lanes of a lane half hold a row's columns
      // (tn-major), reduced by xor shuffles within the half.  Full tiles load the residual
      // and store y by buffer ops off the wave tile's origin with scalar row offsets (as the
      // EPI_RESID path below); a ragged last row band uses guarded plain accesses.
      static_assert(T::WN == kLnPartW, "stats partials are per kLnPartW-column wave tile");
      const int wr0 = m0 + wm * T::WM, wc0 = n0 + wn * T::WN;
      const int part = wc0 / T::WN;
      float bv[T::TN];
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn) bv[tn] = bias[wc0 + tn * 32 + (lane & 31)];
      float rv[T::TM][T::TN][16];
      const bool full = m0 + T::BM <= M;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(out + (int64_t)wr0 * ldo + wc0), (short)0, 0x7fffffff, 0x00020000);
      const int ol = (4 * (lane >> 5) * ldo + (lane & 31)) * 4;
      if (full) {
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(resid + (int64_t)wr0 * ldr + wc0), (short)0, 0x7fffffff, 0x00020000);
        const int rl = (4 * (lane >> 5) * ldr + (lane & 31)) * 4;
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e)
              rv[tm][tn][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  rr, rl, (acc_row(tm, e, 0) * ldr + tn * 32) * 4, 0));
      } else {
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int row = min(wr0 + acc_row(tm, e, lane), M - 1);
              rv[tm][tn][e] = resid[(int64_t)row * ldr + wc0 + tn * 32 + (lane & 31)];
            }
      }
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = wr0 + acc_row(tm, e, lane);
          float v[T::TN], sum = 0.f;
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn) {
            v[tn] = acc[tm][tn][e] + bv[tn] + rv[tm][tn][e];
            sum += v[tn];
          }
          if (full) {
#pragma unroll
            for (int tn = 0; tn < T::TN; ++tn)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[tn]), ro, ol, (acc_row(tm, e, 0) * ldo + tn * 32) * 4, 0);
          } else if (row < M) {
#pragma unroll
            for (int tn = 0; tn < T::TN; ++tn) out[(int64_t)row * ldo + wc0 + tn * 32 + (lane & 31)] = v[tn];
          }
#pragma unroll
          for (int off = 16; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
          const float mean = sum * (1.0f / T::WN);
          float m2 = 0.f;
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn) m2 += (v[tn] - mean) * (v[tn] - mean);
#pragma unroll
          for (int off = 16; off > 0; off >>= 1) m2 += __shfl_xor(m2, off);
          if ((lane & 31) == 0 && row < M)
            reinterpret_cast<float2*>(ln.stats_out)[(int64_t)row * ln.nt + part] = make_float2(mean, m2);
        }
      return;
    }
    if (m0 + T::BM <= M && n0 + T::BN <= N) {
      // full tile: every bias / residual load goes out before the first use, so the
      // tile pays one memory round trip (the guarded loop below waits per element).
      // Residual loads and output stores are buffer ops off the wave tile's origin: one
      // lane offset (column, lane half's row quad) in a VGPR, each register's row offset
      // row(e) * ld a scalar soffset - no per-element address arithmetic.
      const int wr0 = m0 + wm * T::WM, wc0 = n0 + wn * T::WN;
      float bv[T::TN];
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn) bv[tn] = bias[wc0 + tn * 32 + (lane & 31)];
      float rv[T::TM][T::TN][16];
      if constexpr (EPI == EPI_RESID) {
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(resid + (int64_t)wr0 * ldr + wc0), (short)0, 0x7fffffff, 0x00020000);
        const int rl = (4 * (lane >> 5) * ldr + (lane & 31)) * 4;
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
            for (int e = 0; e < 16; ++e)
              rv[tm][tn][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                  rr, rl, (acc_row(tm, e, 0) * ldr + tn * 32) * 4, 0));
      }
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(out + (int64_t)wr0 * ldo + wc0), (short)0, 0x7fffffff, 0x00020000);
      const int ol = (4 * (lane >> 5) * ldo + (lane & 31)) * 4;
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            float v = acc[tm][tn][e] + bv[tn];
            if (EPI == EPI_GELU_ERF) v = gelu_erf(v);
            if (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
            if (EPI == EPI_RESID) v += rv[tm][tn][e];
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ro, ol, (acc_row(tm, e, 0) * ldo + tn * 32) * 4, 0);
          }
      return;
    }
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn) {
      const int col = n0 + wn * T::WN + tn * 32 + (lane & 31);
      if (col >= N) continue;
      const float b = bias[col];
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = m0 + wm * T::WM + acc_row(tm, e, lane);
          if (row >= M) continue;
          float v = acc[tm][tn][e] + b;
          if (EPI == EPI_GELU_ERF) v = gelu_erf(v);
          if (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
          if (EPI == EPI_RESID) v += resid[(int64_t)row * ldr + col];
          out[(int64_t)row * ldo + col] = v;
        }
    }
  };
  if constexpr (LN_IN) {
    LnInHooks<T, decltype(coords)> hk{ln, coords, ln_st, M, K / T::BK, n_tiles * (K / T::BK), 1.0f / (float)K,
                                      FastDiv(K / T::BK)};
    walk_tiles_hooked<T>(lds, n_tiles, TileOperands{A, lda, M, W, K, N, K}, coords, epi, hk);
  } else {
    walk_tiles<T>(lds, n_tiles, TileOperands{A, lda, M, W, K, N, K}, coords, epi);
  }
}

// ------------------------------------------- K4 / K6: residual GEMM + LayerNorm ---
// x = LN(A W^T + bias + resid) with the LayerNorm in the epilogue: a workgroup owns 32 FULL
// rows (BN = N = H, T = F32Tile<1, 8, 1, H / 256, ..., BK 16>: 8 waves x 32 x (H/8)
// columns, 16-deep slices so the 32 + H row image double-buffers in LDS), so each row's
// mean and variance are block reductions - no y round trip through HBM and no LayerNorm
// launch (24 per batched step).  Two-pass statistics over the fp32 sums as ln_kernel
// computes them (the summation order differs: results agree to rounding).  `out` may be
// `resid` (each element is read and written by the same thread, and a workgroup owns its
// rows); the strided CLS-only layer, whose compact output rows alias other residual rows,
// keeps the two-launch path.  Persistent: workgroups walk row blocks t = blockIdx.x + i G.
template <class T>
__global__ __launch_bounds__(T::THREADS, 1) void gemm_resid_ln_kernel(
    const float* __restrict__ A, int lda, const float* __restrict__ W, const float* __restrict__ bias,
    const float* resid, const float* __restrict__ lng, const float* __restrict__ lnb, float eps, float* out,
    int M, int K) {
  constexpr int H = T::BN;
  static_assert(T::WAVES_M == 1 && T::TM == 1 && T::BM == 32, "32-row full-width tiles");
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  __shared__ float red[2][T::WAVES_N][32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int total = (M + 31) / 32;
  const int n_tiles = blockIdx.x < total ? (total - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
  auto coords = [&](int i, int& m0, int64_t& n0) {
    m0 = (blockIdx.x + i * gridDim.x) * 32;
    n0 = 0;
  };
  // this lane's columns: wave w, tile tn, lane & 31; bias / gamma / beta held for the launch
  float bv[T::TN], gv[T::TN], ev[T::TN];
#pragma unroll
  for (int tn = 0; tn < T::TN; ++tn) {
    const int col = wave * T::WN + tn * 32 + (lane & 31);
    bv[tn] = bias[col];
    gv[tn] = lng[col];
    ev[tn] = lnb[col];
  }
  auto epi = [&](int i, floatx16(&acc)[T::TM][T::TN], float*) {
    const int m0 = (blockIdx.x + i * gridDim.x) * 32;
    // v = acc + bias + resid (rows past M read row M - 1 and are never stored)
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn) {
      const int col = wave * T::WN + tn * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = min(m0 + acc_row(0, e, lane), M - 1);
        acc[0][tn][e] = acc[0][tn][e] + bv[tn] + resid[(int64_t)row * H + col];
      }
    }
    // row sums: this lane's T::TN columns, then the 32 lanes of its half (same rows), then
    // the waves through LDS; element e of lane half h is row (e&3) + 8(e>>2) + 4h
    auto row_reduce = [&](int pass, auto&& val) {
      float p[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float t = 0.f;
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn) t += val(tn, e);
        p[e] = t;
      }
#pragma unroll
      for (int off = 1; off < 32; off <<= 1)
#pragma unroll
        for (int e = 0; e < 16; ++e) p[e] += __shfl_xor(p[e], off);
      if ((lane & 31) == 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[pass][wave][acc_row(0, e, lane)] = p[e];
    };
    row_reduce(0, [&](int tn, int e) { return acc[0][tn][e]; });
    __syncthreads();
    float mean[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rr = acc_row(0, e, lane);
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < T::WAVES_N; ++w) t += red[0][w][rr];
      mean[e] = t * (1.0f / H);
    }
    row_reduce(1, [&](int tn, int e) {
      const float d = acc[0][tn][e] - mean[e];
      return d * d;
    });
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rr = acc_row(0, e, lane);
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < T::WAVES_N; ++w) t += red[1][w][rr];
      const float rstd = 1.0f / sqrtf(t * (1.0f / H) + eps);
      const int row = m0 + rr;
      if (row < M) {
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn) {
          const int col = wave * T::WN + tn * 32 + (lane & 31);
          out[(int64_t)row * H + col] = (acc[0][tn][e] - mean[e]) * rstd * gv[tn] + ev[tn];
        }
      }
    }
    // (the next tile's reductions reuse red[]: its first write follows a block barrier
    // inside the slice loop, after every wave has read this tile's sums)
  };
  walk_tiles<T>(lds, n_tiles, TileOperands{A, lda, M, W, K, H, K}, coords, epi);
}

// ---------------------------------------------------------- split-K GEMM ------
// For few rows (single queries, the CLS-only last layer) the direct GEMM leaves most
// CUs idle.  Split K into S chunks: workgroup (tile, s) multiplies its tile over
// K-chunk s and stores an fp32 partial slab[s][M][N]; splitk_reduce_kernel then sums
// the S slabs IN ORDER (bitwise reproducible) and applies bias / GELU / residual.
template <class T>
__global__ __launch_bounds__(256, 2) void gemm_splitk_kernel(const float* __restrict__ A, int lda,
                                                             const float* __restrict__ W, int M,
                                                             int N, int K, int S,
                                                             float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int tiles_n = (N + T::BN - 1) / T::BN;
  const int tile = blockIdx.x / S, sidx = blockIdx.x % S;
  const int Kc = K / S;
  const int m0 = (tile / tiles_n) * T::BM;
  const int n0 = (tile % tiles_n) * T::BN;
  auto coords = [&](int, int& mm0, int64_t& nn0) {
    mm0 = m0;
    nn0 = n0;
  };
  float* dst = slab + (int64_t)sidx * M * N;
  auto epi = [&](int, floatx16(&acc)[T::TM][T::TN], float*) {
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn) {
      const int col = n0 + wn * T::WN + tn * 32 + (lane & 31);
      if (col >= N) continue;
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = m0 + wm * T::WM + acc_row(tm, e, lane);
          if (row < M) dst[(int64_t)row * N + col] = acc[tm][tn][e];
        }
    }
  };
  walk_tiles<T>(lds, 1, TileOperands{A + (int64_t)sidx * Kc, lda, M, W + (int64_t)sidx * Kc, K, N, Kc},
                coords, epi);
}

// sum_{s<S} p[s * plane] (float4), left to right; the loads go out 8, then 4 at a time
// so a deep split does not serialise on load latency (same additions, same order: the
// sum starts from -0.0f, the exact additive identity; S = 12 and 16, the split factors
// of K = 768 and 3072, take no single-load round trip).
__device__ __forceinline__ floatx4 sum_slabs(const float* __restrict__ p, int64_t plane, int S) {
  floatx4 v = {-0.f, -0.f, -0.f, -0.f};
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    floatx4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const floatx4*>(p + (s + u) * plane);
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  if (s + 4 <= S) {
    floatx4 t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const floatx4*>(p + (s + u) * plane);
#pragma unroll
    for (int u = 0; u < 4; ++u) v += t[u];
    s += 4;
  }
  for (; s < S; ++s) v += *reinterpret_cast<const floatx4*>(p + s * plane);
  return v;
}

template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int S,
                                                            int M, int N,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ resid, int ldr,
                                                            float* __restrict__ out, int ldo) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index, N % 4 == 0
  const int64_t n4 = N / 4;
  if (i4 >= (int64_t)M * n4) return;
  const int row = (int)(i4 / n4), c = (int)(i4 % n4) * 4;
  const int64_t plane = (int64_t)M * N;
  floatx4 v = sum_slabs(slab + (int64_t)row * N + c, plane, S);
  v += *reinterpret_cast<const floatx4*>(bias + c);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (EPI == EPI_GELU_ERF) v[j] = gelu_erf(v[j]);
    if (EPI == EPI_GELU_TANH) v[j] = gelu_tanh(v[j]);
  }
  if (EPI == EPI_RESID) v += *reinterpret_cast<const floatx4*>(resid + (int64_t)row * ldr + c);
  *reinterpret_cast<floatx4*>(out + (int64_t)row * ldo + c) = v;
}

// ------------------------------------------------------- K1 / LayerNorm ------
template <int VPL>
__device__ __forceinline__ void ln_row_store(floatx4 (&x)[VPL], const float* __restrict__ g,
                                             const float* __restrict__ b, float eps,
                                             float* __restrict__ dst, int lane) {
  constexpr int H = VPL * 256;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += x[i].x + x[i].y + x[i].z + x[i].w;
  const float mean = wave_sum(s) * (1.0f / H);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    x[i] -= mean;
    v += x[i].x * x[i].x + x[i].y * x[i].y + x[i].z * x[i].z + x[i].w * x[i].w;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(v) * (1.0f / H) + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (i * 64 + lane) * 4;
    const floatx4 gg = *reinterpret_cast<const floatx4*>(g + c);
    const floatx4 bb = *reinterpret_cast<const floatx4*>(b + c);
    *reinterpret_cast<floatx4*>(dst + c) = x[i] * rstd * gg + bb;
  }
}

// Split-K reduction of a residual projection fused with the LayerNorm after it (few-row
// path: saves a launch and the y round trip per LN): x = LN(sum_s slab[s] + bias +
// resid), slabs summed in order (the LN's reductions are block-wide, so the result
// matches splitk_reduce_kernel<EPI_RESID> + ln_kernel to rounding).  A block reads its
// whole row before writing it, so dst may alias resid row for row (stride H).
template <int VPL>
__global__ __launch_bounds__(256) void splitk_reduce_ln_kernel(
    const float* __restrict__ slab, int S, int M, const float* __restrict__ bias,
    const float* resid, int ldr, const float* __restrict__ g, const float* __restrict__ b,
    float eps, float* dst) {
  // one 256-thread block per row (the few-row path has few rows: 4 waves per row keep
  // 4x more slab loads in flight than a wave per row); thread t owns columns t + 256 i
  constexpr int H = VPL * 256;
  __shared__ float part[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row = blockIdx.x;
  const int64_t plane = (int64_t)M * H;
  float x[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = t + 256 * i;
    const float* p = slab + (int64_t)row * H + c;
    float v = -0.f;  // as sum_slabs: 8 then 4 loads in flight, same order
    int sl = 0;
    for (; sl + 8 <= S; sl += 8) {
      float u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = p[(sl + j) * plane];
#pragma unroll
      for (int j = 0; j < 8; ++j) v += u[j];
    }
    if (sl + 4 <= S) {
      float u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = p[(sl + j) * plane];
#pragma unroll
      for (int j = 0; j < 4; ++j) v += u[j];
      sl += 4;
    }
    for (; sl < S; ++sl) v += p[sl * plane];
    x[i] = v + bias[c] + resid[(int64_t)row * ldr + c];
  }
  auto block_sum = [&](float v) {
    v = wave_sum(v);
    if (lane == 0) part[wave] = v;
    __syncthreads();
    const float r = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    return r;
  };
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) sum += x[i];
  const float mean = block_sum(sum) * (1.0f / H);
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    x[i] -= mean;
    var += x[i] * x[i];
  }
  const float rstd = 1.0f / sqrtf(block_sum(var) * (1.0f / H) + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = t + 256 * i;
    dst[(int64_t)row * H + c] = x[i] * rstd * g[c] + b[c];
  }
}

// Row statistics of one LayerNorm row held as ln_row_store holds it (same sums in the
// same order, so mean / rstd are bitwise those of ln_kernel).
template <int VPL>
__device__ __forceinline__ void ln_row_stats(const floatx4 (&x)[VPL], float eps, float& mean,
                                             float& rstd) {
  constexpr int H = VPL * 256;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += x[i].x + x[i].y + x[i].z + x[i].w;
  mean = wave_sum(s) * (1.0f / H);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const floatx4 d = x[i] - mean;
    v += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
  }
  rstd = 1.0f / sqrtf(wave_sum(v) * (1.0f / H) + eps);
}

// Wave sum with DPP lane moves inside each 16-lane row (xor 1, xor 2, half-row mirror, row
// mirror) and two cross-row shuffles: 2 LDS-crossbar round trips instead of wave_sum's 6
// (the few-row path's LayerNorm runs on the critical path of every launch).
__device__ __forceinline__ float dpp_add(float v, int ctrl_id) {
  int t;
  switch (ctrl_id) {  // dpp_ctrl must be an immediate
    case 0: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false); break;   // quad xor 1
    case 1: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false); break;   // quad xor 2
    case 2: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false); break;  // row half mirror
    default: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false); break; // row mirror
  }
  return v + __int_as_float(t);
}
__device__ __forceinline__ float wave_sum_fast(float v) {
  v = dpp_add(v, 0);
  v = dpp_add(v, 1);
  v = dpp_add(v, 2);
  v = dpp_add(v, 3);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int VPL>
__device__ __forceinline__ void ln_row_stats_fast(const floatx4 (&x)[VPL], float eps, float& mean,
                                                  float& rstd) {
  constexpr int H = VPL * 256;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += x[i].x + x[i].y + x[i].z + x[i].w;
  mean = wave_sum_fast(s) * (1.0f / H);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const floatx4 d = x[i] - mean;
    v += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
  }
  rstd = 1.0f / sqrtf(wave_sum_fast(v) * (1.0f / H) + eps);
}

// ------------------------------------------------------- few-row GEMM (K2r) ----
// A single query is M = L <= 64 token rows: the tiled GEMM leaves the chip idle and the
// split-K path pays a second launch for its ordered slab reduction (~5 us each, 4 per
// layer).  Here one 1024-thread workgroup owns a 16 x 16 output tile over the FULL depth:
// its 16 waves each multiply one contiguous K range (NB x 256 / 16 deep) on
// v_mfma_f32_16x16x4_f32 and the 16 partial tiles are summed in wave order through LDS
// (bitwise reproducible), then bias / GELU / residual.  Grid (N / 16, ceil(M / 16)):
// 288 workgroups for QKV, 384 for FFN-up, 96 for the two H-wide projections at M = 32.
// Lane (c = l & 15, kq = l >> 4) loads float4s of row c of the A and W tiles at
// k0 + 4 kq; MFMA step t multiplies element t, i.e. logical k index kq <-> k0 + 4 kq + t
// in both operands.
// LN_IN: A holds pre-LayerNorm rows (the last residual sum, K = H = 256 VPL); wave w
// first computes row r0 + w's mean / rstd (as ln_kernel) and A is normalised while it is
// loaded, so no LayerNorm launch sits between the GEMMs.  The column-0 workgroups also
// store the normalised rows to ln_out: the residual input of the next projection.
#ifndef MQ_ROWS_DBG
#define MQ_ROWS_DBG 0  // measurement builds only: 1 no weight loads, 2 no row loads, 4 no MFMA
#endif
#if MQ_ROWS_DBG != 0 && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_ROWS_DBG computes wrong results: only a measurement build (-DMQ_MEASUREMENT_BUILD) may set it"
#endif
// Measurement builds with -DMQ_KTRACE: thread 0 of each workgroup of the few-row kernels
// stamps the 100 MHz wall clock at phase boundaries into mq_ktrace[workgroup][slot]
// (read back by mq_debug_ktrace_read, tools/ktrace.py).  Compiled out otherwise.
#if defined(MQ_KTRACE) && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_KTRACE is a measurement build option (-DMQ_MEASUREMENT_BUILD)"
#endif
#ifdef MQ_KTRACE
// region 0 QKV, 1 FFN-up, 2 FFN-down / out-proj (rows_gemm_kernel by epilogue), 3 K3o
constexpr int kTraceSlots = 8, kTraceWgs = 1024, kTraceRegions = 4;
__device__ long long mq_ktrace[kTraceRegions * kTraceWgs * kTraceSlots];
#define KTRACE_R(region, slot)                                                                 \
  do {                                                                                        \
    if (threadIdx.x == 0) {                                                                   \
      const int wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);           \
      if (wg_ < kTraceWgs) mq_ktrace[((region) * kTraceWgs + wg_) * kTraceSlots + (slot)] = wall_clock64(); \
    }                                                                                         \
  } while (0)
#else
#define KTRACE_R(region, slot) \
  do {                         \
  } while (0)
#endif
// Measurement builds with -DMQ_ROWS_REPEAT: every few-row launch runs twice back to back
// (all five are idempotent), so a kernel trace shows each launch cold and with its
// weights warm in L2 / MALL - what a next-phase weight prefetch could at best recover.
#if defined(MQ_ROWS_REPEAT) && !defined(MQ_MEASUREMENT_BUILD)
#error "MQ_ROWS_REPEAT is a measurement build option (-DMQ_MEASUREMENT_BUILD)"
#endif
#ifdef MQ_ROWS_REPEAT
#define ROWS_REP for (int rep_ = 0; rep_ < 2; ++rep_)
#else
#define ROWS_REP
#endif
// A weight fragment of the few-row kernels: default cache policy, or non-temporal for the
// layers past the handle's `resident_layers` (MQ_ENC_OPT_RESIDENT_LAYERS), so that
// back-to-back single queries keep the first layers' weights in the 256 MB MALL instead
// of cycling all 340 MB through it (a cyclic sweep larger than the cache hits nothing).
// Buffer loads off the matrix base (byte offsets < 2^31): the policy is an immediate of the
// intrinsic, so the two forms stay two instructions (a plain load and a nontemporal-hinted
// one under a runtime branch get merged into one plain load).
__device__ __forceinline__ floatx4 load_w(__amdgpu_buffer_rsrc_t w, int byte_off, int nt) {
  return __builtin_bit_cast(floatx4, nt ? __builtin_amdgcn_raw_buffer_load_b128(w, byte_off, 0, 2)
                                        : __builtin_amdgcn_raw_buffer_load_b128(w, byte_off, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w_rsrc(const float* W) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 0x7fffffff, 0x00020000);
}
// Fragment image ("frag16") of a [R][C] fp32 matrix for the few-row kernels: per 16-row x
// 16-column block (block (rb, cb), cb fastest) 1 KB in the lane order of one
// v_mfma_f32_16x16x4_f32 operand load - lane l = c + 16 kq holds the float4 at row
// 16 rb + c, columns 16 cb + 4 kq .. + 3.  One wave-instruction then moves 1 KB of whole
// lines, where the row-major operand loads moved 16 rows x 64 B (16 half lines) each;
// profiles/r6/engine_probe.jsonl: 5.76 -> 3.37 us for FFN-down's per-workgroup bytes.
// The weights are imaged once at load (mq_encoder_load_weights); FFN-up writes its output
// in this layout for FFN-down (FL_O / FL_A).
// FL_OT (with FL_O): the blocks of the last third of the columns (QKV's V) are stored
// transposed - the frag16 of V^T - so attention's P V reads V^T fragments whole
// FL_ACC: the K splits add into ONE output plane (a no-return device-scope atomic add per
// element into a zeroed buffer) instead of writing a plane each.  With exactly two addends
// per element, 0 + a + b and 0 + b + a are the same float (addition commutes), so the result
// is bitwise the p0 + p1 the consumer summed before - and the consumer reads one plane.
enum RowsFlags { FL_A = 1, FL_O = 2, FL_OT = 4, FL_ACC = 8 };  // A / output in frag16 (weights always are)
__device__ __forceinline__ int64_t frag16_offset(int64_t row, int col, int cols) {  // in floats
  return ((row >> 4) * (cols >> 4) + (col >> 4)) * 256 + ((row & 15) + 16 * ((col & 15) >> 2)) * 4 + (col & 3);
}
__global__ __launch_bounds__(256) void frag16_image_kernel(const float* __restrict__ W, int R, int C,
                                                           floatx4* __restrict__ img) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one float4 of the image
  if (idx >= (int64_t)R * C / 4) return;
  const int lane = (int)(idx & 63);
  const int64_t blk = idx >> 6;
  const int cbs = C >> 4;
  const int64_t rb = blk / cbs;
  const int cb = (int)(blk - rb * cbs);
  img[idx] = *reinterpret_cast<const floatx4*>(W + (rb * 16 + (lane & 15)) * C + cb * 16 + 4 * (lane >> 4));
}

constexpr int kRT = 16;      // rows = columns per output tile
constexpr int kRWaves = 16;  // waves per workgroup, one K range each
constexpr int kRowsMax = 256; // token rows up to which a forward may take this path
constexpr int kRowsDefault = 64;  // ... and does by default (MQ_ROWS_MAX overrides)

// W is the weights' frag16 image (ldw = the full depth); FL & FL_A: A (no LayerNorm input)
// in frag16 with lda columns; FL & FL_O: out in frag16 with ldo columns.
template <int EPI, bool LN_IN, int VPL, int NB, int S_IN, int RT, int FL = 0>
__global__ __launch_bounds__(1024) void rows_gemm_kernel(
    const float* __restrict__ A, int lda, int64_t a_plane, int M, const float* __restrict__ lng,
    const float* __restrict__ lnb, float eps, float* __restrict__ ln_out,
    const float* __restrict__ W, int ldw, const float* __restrict__ bias,
    const float* __restrict__ resid, int ldr, float* __restrict__ out, int ldo, int64_t o_plane,
    const int* __restrict__ ids, int L, int vocab, const float* __restrict__ pos,
    const float* __restrict__ typ, int nt_w, float* __restrict__ zbuf, int64_t zn) {
  static_assert(!(LN_IN && (FL & FL_A)), "a LayerNorm input is read row-major");
  static_assert(!((FL & FL_ACC) && (FL & FL_O)), "accumulated output is row-major");
  // zbuf: zn floats (a multiple of 4) this launch zeroes for a LATER launch's FL_ACC adds
  if (zbuf) {
    const int64_t nwg = (int64_t)gridDim.x * gridDim.y * gridDim.z;
    const int64_t wg = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    for (int64_t i = wg * 1024 + threadIdx.x; i < zn / 4; i += nwg * 1024)
      reinterpret_cast<floatx4*>(zbuf)[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int K = NB * 256;  // depth of this workgroup's K split (blockIdx.z)
  // 16-deep blocks per load batch: all of them while the operands fit the 128 VGPRs of a
  // 1024-thread workgroup (one memory round trip), else batches
  constexpr int CH = RT == 1 ? (NB <= 12 ? NB : 8) : (NB <= 6 ? NB : 4);
  static_assert(NB % CH == 0, "the load batch must divide NB");
  static_assert(!LN_IN || NB == VPL, "LayerNorm input needs K == H");
  static_assert(RT >= 1 && RT * kRT * kRT <= 1024, "one epilogue thread per output element");
  // LN_IN: the RT x 16 normalised rows, row stride K + 4 floats (a 16-lane ds_read_b128
  // group reads 16 rows at one k: 16 distinct 16-B bank groups)
  constexpr int AS = K + 4;
  __shared__ __attribute__((aligned(16))) float arows[LN_IN ? RT * kRT * AS : 4];
  __shared__ float part[kRWaves][RT][kRT * kRT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, kq = lane >> 4;
  const int n0 = blockIdx.x * kRT, r0 = blockIdx.y * kRT * RT;
  const int kb0 = wave * (K / kRWaves);  // this wave's K range
  const int ks = blockIdx.z;  // K split: columns [ks K, (ks + 1) K) of A and W
  const __amdgpu_buffer_rsrc_t wr = w_rsrc(W);
  // this lane's weight fragment: block (n0 / 16, (ks K + kb0) / 16 + j) of the image, 1 KB apart
  const int kblk0 = (ks * K + kb0) >> 4;
  const int wo4 = (((n0 >> 4) * (ldw >> 4) + kblk0) * 64 + lane) * 16;

  KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 0);
  floatx4 wv[CH], av[RT][CH];
  // the first batch of weights is in flight before anything else (the LayerNorm pass
  // below waits on its own row loads only).  All RT row tiles share each weight
  // fragment: the launch streams W once.
#pragma unroll
  for (int j = 0; j < CH; ++j)
    wv[j] = (MQ_ROWS_DBG & 1) ? floatx4{1e-3f, 1e-3f, 1e-3f, 1e-3f} : load_w(wr, wo4 + 1024 * j, nt_w);
  // Everything else this launch reads from memory goes out now too, under the weight
  // loads: the epilogue's bias / residual element (thread t < 256 RT finishes element
  // t % 256 of row tile t / 256) and the LayerNorm's gamma / beta.  Loaded where they are
  // used, each would add a dependent memory round trip to the launch's critical path
  // (after the partial-tile reduction, after the row statistics).  FL_O: thread t's element
  // is position t % 256 of the tile's frag16 block (lane (t % 256) / 4), so each wave
  // stores 256 contiguous bytes.
  const int et = threadIdx.x, ert = et / (kRT * kRT), ep = et % (kRT * kRT);
  const bool vt = (FL & FL_OT) && n0 >= 2 * (ldo / 3);  // a V block of QKV, stored as V^T
  const int ee = !(FL & FL_O) ? ep
                 : vt ? ((4 * (ep >> 6) + (ep & 3)) * kRT + ((ep >> 2) & 15))
                      : (((ep >> 2) & 15) * kRT + 4 * (ep >> 6) + (ep & 3));  // [row][col] in the tile
  const int erow = r0 + ert * kRT + ee / kRT, ecol = n0 + ee % kRT;
  float ebias = 0.f, eres = 0.f;
  if (ert < RT && ks == 0 && erow < M) {
    ebias = bias[ecol];
    if (EPI == EPI_RESID) eres = resid[(int64_t)erow * ldr + ecol];
  }
  floatx4 lgv[LN_IN ? VPL : 1], lbv[LN_IN ? VPL : 1];
  if (LN_IN) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      lgv[i] = *reinterpret_cast<const floatx4*>(lng + (i * 64 + lane) * 4);
      lbv[i] = *reinterpret_cast<const floatx4*>(lnb + (i * 64 + lane) * 4);
    }
  }
  if (LN_IN) {
    // wave w normalises rows r0 + w + 16 rt (one row per wave per row tile)
    floatx4 x[RT][VPL];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int rr = min(r0 + rt * kRT + wave, M - 1);
      const float* src = A + (int64_t)rr * lda;
      if constexpr (MQ_ROWS_DBG & 2) {
#pragma unroll
        for (int i = 0; i < VPL; ++i) x[rt][i] = floatx4{0.1f * lane, 0.2f, 0.3f, 0.4f * wave};
      } else if constexpr (S_IN == 0) {
        // layer 0: the row is the embedding sum word[id] + pos[p] + type[0] (as
        // embed_ln_kernel; A = the word table), normalised with the embedding LayerNorm
        int id = ids[rr];
        id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
          const int cc = (i * 64 + lane) * 4;
          x[rt][i] = *reinterpret_cast<const floatx4*>(A + (int64_t)id * K + cc) +
                     *reinterpret_cast<const floatx4*>(pos + (int64_t)(rr % L) * K + cc) +
                     *reinterpret_cast<const floatx4*>(typ + cc);
        }
      } else {
        // the row is the sum of S_IN split-K planes of the producing GEMM, added in order
        floatx4 p[S_IN][VPL];
#pragma unroll
        for (int z = 0; z < S_IN; ++z)
#pragma unroll
          for (int i = 0; i < VPL; ++i)
            p[z][i] = *reinterpret_cast<const floatx4*>(src + z * a_plane + (i * 64 + lane) * 4);
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
          x[rt][i] = p[0][i];
#pragma unroll
          for (int z = 1; z < S_IN; ++z) x[rt][i] += p[z][i];
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float mu, rs;
      ln_row_stats_fast<VPL>(x[rt], eps, mu, rs);
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int cc = (i * 64 + lane) * 4;
        x[rt][i] = (x[rt][i] - mu) * rs * lgv[i] + lbv[i];
        *reinterpret_cast<floatx4*>(&arows[(rt * kRT + wave) * AS + cc]) = x[rt][i];
      }
    }
    KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 1);
    // LDS-only barrier: the weight loads stay in flight across it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 2);
    // the normalised rows out, 16 columns per workgroup of this row group (not all of
    // them from one workgroup: the slowest workgroup sets the launch's duration)
    if (ln_out && ert < RT) {
      const int rr = ert * kRT + ee / kRT, cc = ee % kRT;
      if (r0 + rr < M)
        for (int c0 = blockIdx.x * kRT; c0 < K; c0 += gridDim.x * kRT)
          ln_out[(int64_t)(r0 + rr) * K + c0 + cc] = arows[rr * AS + c0 + cc];
    }
  }

  floatx4 acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < NB; b += CH) {
    if (b > 0) {
#pragma unroll
      for (int j = 0; j < CH; ++j) wv[j] = load_w(wr, wo4 + 1024 * (b + j), nt_w);
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float* arow = A + (int64_t)min(r0 + rt * kRT + c, M - 1) * lda + ks * K + kb0 + 4 * kq;
      // frag16 A: row block (r0 / 16 + rt) (rows past M in the last block are never
      // written; they only feed output rows past M, which are not stored)
      const floatx4* afr = reinterpret_cast<const floatx4*>(A) +
                           ((int64_t)((r0 >> 4) + rt) * (lda >> 4) + kblk0) * 64 + lane;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        if (LN_IN)
          av[rt][j] = *reinterpret_cast<const floatx4*>(&arows[(rt * kRT + c) * AS + kb0 + 16 * (b + j) + 4 * kq]);
        else if (MQ_ROWS_DBG & 2)
          av[rt][j] = floatx4{0.1f, 0.2f, 0.3f, 0.4f};
        else if (FL & FL_A)
          av[rt][j] = afr[(b + j) * 64];
        else
          av[rt][j] = *reinterpret_cast<const floatx4*>(arow + 16 * (b + j));
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          if (MQ_ROWS_DBG & 4)
            acc[rt][t] += av[rt][j][t] * wv[j][t];
          else
            acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rt][j][t], wv[j][t], acc[rt], 0, 0, 0);
        }
      }
    }
  }
  KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 3);
  // accumulator element j is (row 4 kq + j, column c) of this wave's partial tile
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[wave][rt][(4 * kq + j) * kRT + c] = acc[rt][j];
  __syncthreads();
  KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 4);
  if (ert >= RT) return;
  float v = part[0][ert][ee];
#pragma unroll
  for (int w = 1; w < kRWaves; ++w) v += part[w][ert][ee];
  if (erow >= M) return;
  if (ks == 0) {  // split 0 carries bias / residual; GELU needs an unsplit K
    v += ebias;
    if (EPI == EPI_GELU_ERF) v = gelu_erf(v);
    if (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
    if (EPI == EPI_RESID) v += eres;
  }
  if (FL & FL_O)
    out[ks * o_plane + (((int64_t)((r0 >> 4) + ert) * (ldo >> 4) + blockIdx.x) << 8) + ep] = v;
  else if (FL & FL_ACC)
    (void)atomicAdd(out + (int64_t)erow * ldo + ecol, v);
  else
    out[ks * o_plane + (int64_t)erow * ldo + ecol] = v;
  KTRACE_R(EPI == EPI_BIAS ? 0 : EPI == EPI_RESID ? 2 : 1, 5);
}

// One wave per row of H = 256*VPL floats held in registers (two-pass mean/variance).
template <int VPL>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int* __restrict__ ids, int M, int L, int vocab, const float* __restrict__ word,
    const float* __restrict__ pos, const float* __restrict__ typ, const float* __restrict__ g,
    const float* __restrict__ b, float eps, float* __restrict__ out) {
  constexpr int H = VPL * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  int id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // never gather out of bounds
  const int p = row % L;
  floatx4 x[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = (i * 64 + lane) * 4;
    x[i] = *reinterpret_cast<const floatx4*>(word + (int64_t)id * H + c) +
           *reinterpret_cast<const floatx4*>(pos + (int64_t)p * H + c) +
           *reinterpret_cast<const floatx4*>(typ + c);
  }
  ln_row_store<VPL>(x, g, b, eps, out + (int64_t)row * H, lane);
}

// RPW rows per wave, loaded together and reduced with interleaved shuffle chains (the
// per-row arithmetic is ln_row_store's, so results are bitwise those of one row per wave).
template <int VPL, int RPW>
__global__ __launch_bounds__(256) void ln_kernel(const float* __restrict__ src, int M,
                                                 const float* __restrict__ g,
                                                 const float* __restrict__ b, float eps,
                                                 float* __restrict__ dst) {
  constexpr int H = VPL * 256;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= M) return;
  floatx4 x[RPW][VPL];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      x[r][i] = *reinterpret_cast<const floatx4*>(src + (int64_t)min(row0 + r, M - 1) * H + (i * 64 + lane) * 4);
  float s[RPW], v[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    s[r] = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) s[r] += x[r][i].x + x[r][i].y + x[r][i].z + x[r][i].w;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int r = 0; r < RPW; ++r) s[r] += __shfl_xor(s[r], off);
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const float mean = s[r] * (1.0f / H);
    v[r] = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      x[r][i] -= mean;
      v[r] += x[r][i].x * x[r][i].x + x[r][i].y * x[r][i].y + x[r][i].z * x[r][i].z + x[r][i].w * x[r][i].w;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int r = 0; r < RPW; ++r) v[r] += __shfl_xor(v[r], off);
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    if (row0 + r >= M) break;
    const float rstd = 1.0f / sqrtf(v[r] * (1.0f / H) + eps);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = (i * 64 + lane) * 4;
      const floatx4 gg = *reinterpret_cast<const floatx4*>(g + c);
      const floatx4 bb = *reinterpret_cast<const floatx4*>(b + c);
      *reinterpret_cast<floatx4*>(dst + (int64_t)(row0 + r) * H + c) = x[r][i] * rstd * gg + bb;
    }
  }
}

// ------------------------------------------------------------ K3 attention ----
// One 64-thread workgroup (one wave) per (sequence, head, 32-query tile); dh = 64.
// Scores are computed TRANSPOSED on the f32 MFMA: S^T[key][query] = K . Q^T, so keys
// sit in the accumulator registers and queries on the lanes; the softmax over keys is
// then 16 in-register values + one cross-half exchange per query, and S^T is already
// the B operand of O^T[d][query] = V^T . P^T (no transpose, no LDS for P).
// Operand k-order: lane half h carries head dims 32h..32h+31 for QK^T (one contiguous
// 128-B read per row per lane), and key (s&3) + 8(s>>2) + 4h at PV step s (the
// accumulator row map).  Online softmax across 32-key tiles; masked keys weigh 0.
// NS > 1 (few (sequence, head, query tile) triples with many keys: a long single query, the
// CLS-only last layer): NS waves per workgroup split the key tiles (wave w takes tiles w,
// w + NS, ...), each with its own running max / sum / O^T, merged through LDS at the end in
// wave order: O = sum_w e^(m_w - m) O_w / sum_w e^(m_w - m) l_w (the same softmax; the
// rescaling order differs from one wave walking every tile, results agree to rounding).
constexpr int kDh = 64;

// HB > 1 (NS = 1): one workgroup per (sequence, query tile) with one wave per head, so a
// sequence's Q / K / V rows are read by waves issued together, whole 9 KB rows at a time
// (one wave per workgroup read 256-B head slices of rows 9 KB apart, ~4 TB/s).
template <int NS, int HB = 1>
__global__ __launch_bounds__(64 * NS * HB, NS == 1 && HB == 1 ? 3 : 1) void attention_kernel(const float* __restrict__ qkv,
                                                            const int* __restrict__ mask, int L,
                                                            int H, int heads, int q_tiles,
                                                            float scale, float* __restrict__ ctx) {
  // one LDS tile per wave, used in turn to stage Q, each key tile's K, and the output:
  // [32][68] rows for staging (a 16-lane ds_read_b128 group hits 16 distinct bank groups),
  // [32][65] for the output
  constexpr int kSt = kDh + 4;
  static_assert(HB == 1 || NS == 1, "heads per block or key splits");
  __shared__ __attribute__((aligned(16))) float tiles[NS * HB][32 * kSt];
  __shared__ float wmax[NS > 1 ? NS : 1][32], wsum[NS > 1 ? NS : 1][32];
  const int wv = NS > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  const int hw = HB > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  float* tile = tiles[NS > 1 ? wv : hw];
  float(*obuf)[kDh + 1] = reinterpret_cast<float(*)[kDh + 1]>(tile);
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int hgroups = heads / HB;
  const int qt = blockIdx.x % q_tiles, h = ((blockIdx.x / q_tiles) % hgroups) * HB + hw;
  const int bseq = blockIdx.x / (q_tiles * hgroups);
  const int q0 = qt * 32;
  const int64_t row0 = (int64_t)bseq * L;
  const int ld = 3 * H;
  // Q / K tiles arrive by whole-line loads (4 rows x 256 B per wave-instruction) through
  // LDS; read lane-strided straight from HBM (64 lines per instruction) the tiles were
  // fetched ~2x (PMC), the lines evicted between the 8 instructions that share them.
  auto stage = [&](int row_base, int col) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = 4 * i + (lane >> 4);
      const float* src = qkv + (row0 + min(row_base + rr, L - 1)) * ld + col + (lane & 15) * 4;
      *reinterpret_cast<floatx4*>(&tile[rr * kSt + (lane & 15) * 4]) = *reinterpret_cast<const floatx4*>(src);
    }
  };

  float qf[32];
  stage(q0, h * kDh);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(&tile[r * kSt + hh * 32 + 4 * i]) * scale;
    qf[4 * i] = v.x;
    qf[4 * i + 1] = v.y;
    qf[4 * i + 2] = v.z;
    qf[4 * i + 3] = v.w;
  }
  float m_run = -INFINITY, l_run = 0.f;
  floatx16 o0, o1;
#pragma unroll
  for (int e = 0; e < 16; ++e) o0[e] = o1[e] = 0.f;

  for (int k0 = wv * 32; k0 < L; k0 += 32 * NS) {
    const int kr = min(k0 + r, L - 1);
    const bool kvalid = (k0 + r < L) && mask[row0 + kr] != 0;
    const unsigned long long kbits = __ballot(kvalid);  // bit j = key k0 + j usable
    float kf[32];
    stage(k0, H + h * kDh);  // (one wave per tile: its LDS reads of the last tile precede these writes)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(&tile[r * kSt + hh * 32 + 4 * i]);
      kf[4 * i] = v.x;
      kf[4 * i + 1] = v.y;
      kf[4 * i + 2] = v.z;
      kf[4 * i + 3] = v.w;
    }
    floatx16 st;
#pragma unroll
    for (int e = 0; e < 16; ++e) st[e] = 0.f;
#pragma unroll
    for (int sidx = 0; sidx < 32; ++sidx) st = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[sidx], qf[sidx], st, 0, 0, 0);

    float tmax = -INFINITY;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = (e & 3) + 8 * (e >> 2) + 4 * hh;
      st[e] = ((kbits >> key) & 1ull) ? st[e] : -INFINITY;
      tmax = fmaxf(tmax, st[e]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = (m_new == -INFINITY) ? 1.f : expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      st[e] = (st[e] == -INFINITY) ? 0.f : expf(st[e] - m_new);
      psum += st[e];
    }
    psum += __shfl_xor(psum, 32);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    o0 *= alpha;
    o1 *= alpha;
    // (V staged through this LDS tile by whole-line loads instead, in flight under the
    // softmax, measured slower: attention 0.298 -> 0.327 ms per step, r6)
    const float* vbase = qkv + row0 * ld + 2 * H + h * kDh + r;
#pragma unroll
    for (int sidx = 0; sidx < 16; ++sidx) {
      const int key = min(k0 + (sidx & 3) + 8 * (sidx >> 2) + 4 * hh, L - 1);
      const float v0 = vbase[(int64_t)key * ld];
      const float v1 = vbase[(int64_t)key * ld + 32];
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, st[sidx], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, st[sidx], o1, 0, 0, 0);
    }
  }
  const int nrows = min(32, L - q0);
  if constexpr (NS == 1) {
    // O^T (d on registers, query on lanes) -> LDS [query][d] -> coalesced row stores
    const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int d = (e & 3) + 8 * (e >> 2) + 4 * hh;
      obuf[r][d] = o0[e] * inv;
      obuf[r][d + 32] = o1[e] * inv;
    }
    __syncthreads();
    for (int q = 0; q < nrows; ++q) ctx[(row0 + q0 + q) * H + h * kDh + lane] = obuf[q][lane];
  } else {
    if (hh == 0) wmax[wv][r] = m_run;
    __syncthreads();  // also: every wave is past its last K-tile reads of its own tile
    float m = -INFINITY;
#pragma unroll
    for (int w = 0; w < NS; ++w) m = fmaxf(m, wmax[w][r]);
    const float sc = m_run == -INFINITY ? 0.f : expf(m_run - m);
    if (hh == 0) wsum[wv][r] = l_run * sc;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int d = (e & 3) + 8 * (e >> 2) + 4 * hh;
      obuf[r][d] = o0[e] * sc;
      obuf[r][d + 32] = o1[e] * sc;
    }
    __syncthreads();
    // 32 x 64 outputs over 64 NS threads, partials summed in wave order
    for (int i = threadIdx.x; i < 32 * kDh; i += 64 * NS) {
      const int q = i / kDh, d = i % kDh;
      if (q >= nrows) break;
      float o = 0.f, l = 0.f;
#pragma unroll
      for (int w = 0; w < NS; ++w) {
        o += reinterpret_cast<const float(*)[kDh + 1]>(tiles[w])[q][d];
        l += wsum[w][q];
      }
      ctx[(row0 + q0 + q) * H + h * kDh + d] = l > 0.f ? o * (1.0f / l) : 0.f;
    }
  }
}

// K3 launch: one wave per (sequence, head, query tile) when those fill the chip, else NS
// waves per triple splitting the key tiles (a 256-token single query: 96 waves -> 768).
void launch_attention(int B, int L, int heads, int qt, int H, float scale, const float* qkv,
                      const int* mask, float* ctx, hipStream_t s) {
  const int triples = B * heads * qt, key_tiles = (L + 31) / 32;
  const dim3 grid(triples);
  // (6 or 4 heads per workgroup, 2-3 workgroups per CU: 0.386 / 0.337 vs 0.305 ms per step,
  // same box, r6)
  if (key_tiles == 1 && heads == 12 && triples >= 12 * 256)  // BERT-base batches: 12 heads per workgroup
    hipLaunchKernelGGL((attention_kernel<1, 12>), dim3(B * qt), dim3(768), 0, s, qkv, mask, L, H, heads, qt, scale,
                       ctx);
  else if (key_tiles >= 8 && triples <= 256)
    hipLaunchKernelGGL(attention_kernel<8>, grid, dim3(512), 0, s, qkv, mask, L, H, heads, qt, scale, ctx);
  else if (key_tiles >= 4 && triples <= 512)
    hipLaunchKernelGGL(attention_kernel<4>, grid, dim3(256), 0, s, qkv, mask, L, H, heads, qt, scale, ctx);
  else if (key_tiles >= 2 && triples <= 1024)
    hipLaunchKernelGGL(attention_kernel<2>, grid, dim3(128), 0, s, qkv, mask, L, H, heads, qt, scale, ctx);
  else
    hipLaunchKernelGGL(attention_kernel<1>, grid, dim3(64), 0, s, qkv, mask, L, H, heads, qt, scale, ctx);
}

// K3 for the few-row forward (L <= 64 keys, one sequence's latency): one 512-thread
// workgroup per (sequence, head, 32-query tile).  Wave w = (key quarter kw = w >> 1,
// query half qh = w & 1) computes its 16 x 16 block of S^T = K Q^T on
// v_mfma_f32_16x16x4_f32 (dh = 64 in two 8-step chains), the softmax max and sum over
// all keys are shared through LDS, and the wave multiplies its 16 keys' P^T (the S^T
// accumulator is already the B operand) by V^T into a partial O^T; the four key
// quarters' partials are summed in order.  Masking, scale and exp as attention_kernel;
// the MFMA chain per SIMD is a quarter of the one-wave kernel's.
__global__ __launch_bounds__(512) void attention_rows_kernel(const float* __restrict__ qkv,
                                                             const int* __restrict__ mask, int L,
                                                             int H, int heads, int q_tiles,
                                                             float scale, float* __restrict__ ctx) {
  __shared__ float smax[2][4][16], ssum[2][4][16];
  __shared__ float opart[2][4][16][kDh + 1];  // [qh][kw][query][d]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kw = w >> 1, qh = w & 1;
  const int c = lane & 15, g = lane >> 4;
  const int qt = blockIdx.x % q_tiles, h = (blockIdx.x / q_tiles) % heads;
  const int bseq = blockIdx.x / (q_tiles * heads);
  const int64_t row0 = (int64_t)bseq * L;
  const int ld = 3 * H;
  const int q = qt * 32 + qh * 16 + c;  // this lane's query (B-operand column)
  const int key = kw * 16 + c;          // this lane's key (A-operand row)

  // operands: lane (c, g) holds d = 16 s + 4 g + t at MFMA step (s, t) in both
  floatx4 qf[4], kf[4];
  {
    const float* qs = qkv + (row0 + min(q, L - 1)) * ld + h * kDh + 4 * g;
    const float* ks = qkv + (row0 + min(key, L - 1)) * ld + H + h * kDh + 4 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = *reinterpret_cast<const floatx4*>(qs + 16 * s) * scale;
      kf[s] = *reinterpret_cast<const floatx4*>(ks + 16 * s);
    }
  }
  // V^T operand of the PV step: d = 16 db + c, key = kw * 16 + 4 g + t
  float vf[4][4];
  {
    const float* vs = qkv + row0 * ld + 2 * H + h * kDh + c;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kk = min(kw * 16 + 4 * g + t, L - 1);
#pragma unroll
      for (int db = 0; db < 4; ++db) vf[db][t] = vs[(int64_t)kk * ld + 16 * db];
    }
  }
  const bool kvalid = key < L && mask[row0 + min(key, L - 1)] != 0;
  const unsigned kbits = (unsigned)(__ballot(kvalid) & 0xFFFFull);  // bit k: key kw*16+k usable

  floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s][t], qf[s][t], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s + 2][t], qf[s + 2][t], s1, 0, 0, 0);
    }
  // accumulator j = S^T[key kw*16 + 4g + j][query c]
  floatx4 st = s0 + s1;
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    st[j] = ((kbits >> (4 * g + j)) & 1u) ? st[j] : -INFINITY;
    mx = fmaxf(mx, st[j]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  if (g == 0) smax[qh][kw][c] = mx;
  __syncthreads();
  const float m = fmaxf(fmaxf(smax[qh][0][c], smax[qh][1][c]), fmaxf(smax[qh][2][c], smax[qh][3][c]));
  float ls = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    st[j] = (st[j] == -INFINITY) ? 0.f : expf(st[j] - m);
    ls += st[j];
  }
  ls += __shfl_xor(ls, 16);
  ls += __shfl_xor(ls, 32);
  if (g == 0) ssum[qh][kw][c] = ls;
  floatx4 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    o[db] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) o[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[db][t], st[t], o[db], 0, 0, 0);
  }
  // o[db][j] = O^T[d = 16 db + 4 g + j][query c] over this wave's 16 keys
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int j = 0; j < 4; ++j) opart[qh][kw][c][16 * db + 4 * g + j] = o[db][j];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = e * 512 + (int)threadIdx.x;  // (query of the tile, d), d fastest
    const int q32 = idx >> 6, d = idx & 63;
    const int qq = q32 >> 4, qc = q32 & 15;
    const float v = ((opart[qq][0][qc][d] + opart[qq][1][qc][d]) + opart[qq][2][qc][d]) + opart[qq][3][qc][d];
    const float l = ((ssum[qq][0][qc] + ssum[qq][1][qc]) + ssum[qq][2][qc]) + ssum[qq][3][qc];
    const int qrow = qt * 32 + q32;
    if (qrow < L) ctx[(row0 + qrow) * H + h * kDh + d] = v * (l > 0.f ? 1.0f / l : 0.f);
  }
}

// K3o: attention + output projection of the few-row forward in ONE launch (L <= 64 keys;
// one attention launch per layer fewer).  Workgroup (column tile, query tile, head group):
// 8 waves; waves 0..HG-1 each run one head of the group for the tile's <= 16 queries of
// one sequence (all its keys), as attention_rows_kernel does on v_mfma_f32_16x16x4_f32 but
// with the whole key range in one wave (softmax max / sum by two cross-lane-group
// shuffles, no LDS exchange), and leave ctx[query][head group's 64 HG dims] in LDS; then
// all 8 waves multiply it by the group's K slice of Wo^T for the tile's 32 output columns
// (2 column blocks x 4 K quarters, partial tiles summed in order through LDS).  Group g
// writes output plane g (planes = heads / HG; the next FFN-up sums them while it
// normalises, as QKV sums FFN-down's split-K planes); plane 0 carries bias + residual.
// The attention of a query tile is recomputed by each of the H / 32 column tiles: HG heads
// x 16 queries x L keys of f32 MFMA per workgroup (~1.5 us at L = 32), cheaper than the
// separate launch and its boundary it replaces.
// Rows: output row r of the projection is query position q = r % rps of sequence
// b = r / rps (rps = L, or 1 for the CLS-only last layer: query 0, compact rows).
constexpr int kOpCols = 32;  // output columns per workgroup

// QF: qkv in frag16 with V^T blocks (QKV's FL_O | FL_OT; needs L % 16 == 0, so every
// sequence starts a 16-row block): Q, K and V^T fragments load as whole 1 KB blocks.
// ACC: the head groups add into ONE zeroed output plane (two groups: FL_ACC's argument).
template <int HG, int NKB, bool QF = false, bool ACC = false>
__global__ __launch_bounds__(512) void attn_oproj_rows_kernel(
    const float* __restrict__ qkv, const int* __restrict__ mask, int L, int H, int rps, int qtiles,
    float scale, const float* __restrict__ Wo, const float* __restrict__ bo,
    const float* __restrict__ resid, int ldr, float* __restrict__ out, int64_t o_plane, int nt_w) {
  // NKB = ceil(L / 16) key blocks (compile time: every operand load below is issued before
  // the first MFMA, one memory round trip for the whole launch)
  constexpr int KG = HG * kDh;     // K depth of this group's slice of the projection
  constexpr int CS = KG + 4;       // LDS row stride of ctx (conflict-free ds_read_b128)
  constexpr int KQ = KG / 4;       // K per quarter
  constexpr int NJ = KQ / 16;      // float4 per lane per operand in a quarter
  __shared__ __attribute__((aligned(16))) float ctx[16 * CS];
  __shared__ float part[8][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.y / qtiles, q0 = (blockIdx.y % qtiles) * 16;
  const int grp = blockIdx.z, h0 = grp * HG;
  const int n0 = blockIdx.x * kOpCols;
  const int64_t srow0 = (int64_t)b * L;  // first qkv row of the sequence
  const int ld = 3 * H;

  KTRACE_R(3, 0);
  // projection operands of phase B, in flight from the start: wave w = (column block cb,
  // K quarter kqr); lane (c, g) holds W[n0 + 16 cb + c][k] at k = kqr KQ + 16 j + 4 g + t
  const int cb = w & 1, kqr = w >> 1;
  floatx4 wv[NJ];
  {  // Wo's frag16 image: block ((n0 + 16 cb) / 16, (h0 kDh + kqr KQ) / 16 + j)
    const __amdgpu_buffer_rsrc_t wr = w_rsrc(Wo);
    const int wo4 = ((((n0 >> 4) + cb) * (H >> 4) + ((h0 * kDh + kqr * KQ) >> 4)) * 64 + lane) * 16;
#pragma unroll
    for (int j = 0; j < NJ; ++j) wv[j] = load_w(wr, wo4 + 1024 * j, nt_w);
  }
  // epilogue element of threads < 512: column block et >> 8, row (et & 255) / 16
  const int et = threadIdx.x, ecb = et >> 8, erow_t = (et & 255) >> 4, ecol = n0 + ecb * 16 + (et & 15);
  const int qrow = q0 + erow_t;  // query position of the element's row within the sequence
  const int64_t orow = (int64_t)b * rps + qrow;
  float ebias = 0.f, eres = 0.f;
  if (grp == 0 && qrow < rps) {
    ebias = bo[ecol];
    eres = resid[orow * ldr + ecol];
  }

  if (w < HG) {
    const int h = h0 + w;
    // operands, all requested up front: Q (d = 16 s + 4 g + t for query c; rps == 1:
    // query 0), K per key block (key 16 kb + c), V^T per key block (key 16 kb + 4 g + t,
    // d = 16 db + c), the key mask
    const int qpos = rps == 1 ? 0 : min(q0 + c, L - 1);
    floatx4 qf[4], kf[NKB][4];
    float vf[NKB][4][4];
    if constexpr (QF) {
      // block (row block, column block) of the [rows][3H] frag16 image; lane = (c, g)
      const floatx4* f4 = reinterpret_cast<const floatx4*>(qkv);
      const int cbs = ld >> 4;
      const int64_t rb0 = srow0 >> 4;
      auto blk = [&](int64_t rb, int cb) { return f4 + (rb * cbs + cb) * 64 + lane; };
      // (rps == 1: rows c of block 0 - query 0 is row c = 0, the only one stored)
#pragma unroll
      for (int sI = 0; sI < 4; ++sI) qf[sI] = *blk(rb0 + (q0 >> 4), ((h * kDh) >> 4) + sI);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int sI = 0; sI < 4; ++sI) kf[kb][sI] = *blk(rb0 + kb, ((H + h * kDh) >> 4) + sI);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int db = 0; db < 4; ++db) {  // V^T block: (d = 16 db + c, key = 16 kb + 4 g + t)
          const floatx4 v = *blk(rb0 + kb, ((2 * H + h * kDh) >> 4) + db);
#pragma unroll
          for (int t = 0; t < 4; ++t) vf[kb][db][t] = v[t];
        }
    } else {
      const float* qs = qkv + (srow0 + qpos) * ld + h * kDh + 4 * g;
#pragma unroll
      for (int sI = 0; sI < 4; ++sI) qf[sI] = *reinterpret_cast<const floatx4*>(qs + 16 * sI);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const float* ks = qkv + (srow0 + min(kb * 16 + c, L - 1)) * ld + H + h * kDh + 4 * g;
#pragma unroll
        for (int sI = 0; sI < 4; ++sI) kf[kb][sI] = *reinterpret_cast<const floatx4*>(ks + 16 * sI);
      }
      const float* vs = qkv + srow0 * ld + 2 * H + h * kDh + c;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int64_t kk = min(kb * 16 + 4 * g + t, L - 1);
#pragma unroll
          for (int db = 0; db < 4; ++db) vf[kb][db][t] = vs[kk * ld + 16 * db];
        }
    }
    const bool kval = lane < L && mask[srow0 + min(lane, L - 1)] != 0;
    const unsigned long long kbits = __ballot(kval);  // bit k: key k usable
#pragma unroll
    for (int sI = 0; sI < 4; ++sI) qf[sI] *= scale;
    KTRACE_R(3, 1);  // operands landed
    floatx4 st[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[kb][0][t], qf[0][t], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[kb][2][t], qf[2][t], a1, 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[kb][1][t], qf[1][t], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[kb][3][t], qf[3][t], a1, 0, 0, 0);
      }
      st[kb] = a0 + a1;  // st[kb][j] = S^T[key 16 kb + 4 g + j][query c]
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kb * 16 + 4 * g + j;
        st[kb][j] = ((kbits >> key) & 1ull) ? st[kb][j] : -INFINITY;
        mx = fmaxf(mx, st[kb][j]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st[kb][j] = (st[kb][j] == -INFINITY) ? 0.f : expf(st[kb][j] - mx);
        ls += st[kb][j];
      }
    ls += __shfl_xor(ls, 16);
    ls += __shfl_xor(ls, 32);
    const float inv = ls > 0.f ? 1.0f / ls : 0.f;
    // O^T[d][query] = V^T P^T: A = V[key 16 kb + 4 g + t][d = 16 db + c], B = st[kb][t]
    floatx4 o[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      o[db] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int t = 0; t < 4; ++t) o[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[kb][db][t], st[kb][t], o[db], 0, 0, 0);
    }
    // o[db][j] = O^T[d = 16 db + 4 g + j][query c]
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int j = 0; j < 4; ++j) ctx[c * CS + w * kDh + 16 * db + 4 * g + j] = o[db][j] * inv;
    KTRACE_R(3, 2);  // attention done (wave 0)
  }
  __syncthreads();
  KTRACE_R(3, 3);
  // phase B: partial [16 rows][16 cols] of column block cb over K quarter kqr, as two
  // interleaved accumulation chains (one chain of NJ * 4 dependent MFMAs waits out each
  // one's latency)
  floatx4 acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const floatx4 av = *reinterpret_cast<const floatx4*>(&ctx[c * CS + kqr * KQ + 16 * j + 4 * g]);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc2[j & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], wv[j][t], acc2[j & 1], 0, 0, 0);
  }
  const floatx4 acc = acc2[0] + acc2[1];
  KTRACE_R(3, 4);
  // acc[j] = (row 4 g + j, column c) of the partial
#pragma unroll
  for (int j = 0; j < 4; ++j) part[w][(4 * g + j) * 16 + c] = acc[j];
  __syncthreads();
  KTRACE_R(3, 5);
  const int e = et & 255;
  float v = part[ecb][e];
#pragma unroll
  for (int q = 1; q < 4; ++q) v += part[ecb + 2 * q][e];
  if (qrow >= rps) return;
  if (grp == 0) v = (v + ebias) + eres;
  if (ACC)
    (void)atomicAdd(out + orow * H + ecol, v);
  else
    out[grp * o_plane + orow * H + ecol] = v;
  KTRACE_R(3, 6);
}

// --------------------------------------------------------------- K7 pool -----
// One wave per sequence: CLS row (or masked mean over rows), then x / max(||x||, 1e-12).
template <int VPL>
__global__ __launch_bounds__(256) void pool_kernel(const float* __restrict__ hs,
                                                   const int* __restrict__ mask, int B, int L,
                                                   int pooling, float* __restrict__ out) {
  constexpr int H = VPL * 256;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  floatx4 x[VPL];
  if (pooling == MQ_POOL_MEAN) {
    float cnt = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) x[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < L; ++r) {
      if (!mask[(int64_t)b * L + r]) continue;
      cnt += 1.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i)
        x[i] += *reinterpret_cast<const floatx4*>(hs + ((int64_t)b * L + r) * H + (i * 64 + lane) * 4);
    }
    const float inv = 1.0f / fmaxf(cnt, 1.f);
#pragma unroll
    for (int i = 0; i < VPL; ++i) x[i] *= inv;
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      x[i] = *reinterpret_cast<const floatx4*>(hs + (int64_t)b * L * H + (i * 64 + lane) * 4);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) ss += x[i].x * x[i].x + x[i].y * x[i].y + x[i].z * x[i].z + x[i].w * x[i].w;
  const float inv = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
#pragma unroll
  for (int i = 0; i < VPL; ++i)
    *reinterpret_cast<floatx4*>(out + (int64_t)b * H + (i * 64 + lane) * 4) = x[i] * inv;
}

// K7 for the few-row path, whose last layer leaves pre-LayerNorm rows as `planes`
// split-K planes (`plane` floats apart, summed in order): LN (g, be) of the pooled rows,
// then pool and L2-normalise as pool_kernel.  `rows` = rows per sequence in hs (1: the
// compact CLS rows of the pruned last layer).
template <int VPL>
__global__ __launch_bounds__(256) void ln_pool_kernel(const float* __restrict__ hs, int planes,
                                                      int64_t plane, const int* __restrict__ mask,
                                                      int B, int L, int rows, int pooling,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ be, float eps,
                                                      float* __restrict__ out) {
  constexpr int H = VPL * 256;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  auto ln_row = [&](const float* src, floatx4 (&x)[VPL]) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) x[i] = *reinterpret_cast<const floatx4*>(src + (i * 64 + lane) * 4);
    for (int z = 1; z < planes; ++z)
#pragma unroll
      for (int i = 0; i < VPL; ++i) x[i] += *reinterpret_cast<const floatx4*>(src + z * plane + (i * 64 + lane) * 4);
    float mu, rs;
    ln_row_stats<VPL>(x, eps, mu, rs);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = (i * 64 + lane) * 4;
      x[i] = (x[i] - mu) * rs * *reinterpret_cast<const floatx4*>(g + c) +
             *reinterpret_cast<const floatx4*>(be + c);
    }
  };
  floatx4 x[VPL];
  if (pooling == MQ_POOL_MEAN) {
    float cnt = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) x[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < L; ++r) {
      if (!mask[(int64_t)b * L + r]) continue;
      cnt += 1.f;
      floatx4 y[VPL];
      ln_row(hs + ((int64_t)b * rows + r) * H, y);
#pragma unroll
      for (int i = 0; i < VPL; ++i) x[i] += y[i];
    }
    const float inv = 1.0f / fmaxf(cnt, 1.f);
#pragma unroll
    for (int i = 0; i < VPL; ++i) x[i] *= inv;
  } else {
    ln_row(hs + (int64_t)b * rows * H, x);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) ss += x[i].x * x[i].x + x[i].y * x[i].y + x[i].z * x[i].z + x[i].w * x[i].w;
  const float inv = 1.0f / fmaxf(sqrtf(wave_sum(ss)), 1e-12f);
#pragma unroll
  for (int i = 0; i < VPL; ++i)
    *reinterpret_cast<floatx4*>(out + (int64_t)b * H + (i * 64 + lane) * 4) = x[i] * inv;
}

}  // namespace mq

// ================================================================ host side =====
using namespace mq;

namespace {

struct Buf {
  float* p = nullptr;
  size_t n = 0;  // floats
  int ensure(size_t need) {
    if (need <= n) return MQ_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc((void**)&p, need * sizeof(float)) != hipSuccess)
      MQ_FAIL(MQ_ENOMEM, "hipMalloc(%zu floats) failed", need);
    n = need;
    return MQ_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct LayerW {
  const float *wqkv, *bqkv, *wo, *bo, *ln1g, *ln1b, *w1, *b1, *w2, *b2, *ln2g, *ln2b;
  // W3 plane images of the four projection weights (gemm_x6p.hpp), built when the split-f32
  // precision is selected; null otherwise
  const unsigned char *wqkv3 = nullptr, *wo3 = nullptr, *w13 = nullptr, *w23 = nullptr;
  // frag16 images of the same four (the few-row kernels' weight operands)
  const float *wqkvf = nullptr, *wof = nullptr, *w1f = nullptr, *w2f = nullptr;
};

int64_t weight_count(const mq_bert_config& c) {
  const int64_t H = c.hidden, F = c.ffn;
  const int64_t per_layer = 3 * H * H + 3 * H + H * H + H + 2 * H + F * H + F + H * F + H + 2 * H;
  return ((int64_t)c.vocab_size + c.max_positions + c.type_vocab) * H + 2 * H + c.layers * per_layer;
}

}  // namespace


namespace {

struct GemmArgs {
  float* slab;  // split-K workspace (may be null: never split)
  size_t slab_floats;
  const float* A;
  int lda;
  const float* W;
  const float* bias;
  const float* resid;
  int ldr;
  float* out;
  int ldo;
  int M, N, K;
  int nt = 0;  // few-row split-K launches: weights load non-temporally (layers past resident_layers)
  const void* W3 = nullptr;  // split-f32: W's W3 plane image (K2p, gemm_x6p.hip)
};

template <class T, int EPI, bool LN_IN = false>
void launch_gemm_t(const GemmArgs& g, int num_cus, hipStream_t s, const LnArgs& ln = LnArgs{}) {
  const int tiles = ((g.M + T::BM - 1) / T::BM) * ((g.N + T::BN - 1) / T::BN);
  // persistent grid: the workgroups that fit the CUs at once, a multiple of 8
  const int grid = (std::min(tiles, T::WG_PER_CU * num_cus) + 7) / 8 * 8;
  const int tiles_m = (g.M + T::BM - 1) / T::BM, tiles_n = (g.N + T::BN - 1) / T::BN;
  const int rx = region_pick_rx(tiles_m, tiles_n, (double)T::BM * g.K * 4, (double)T::BN * g.K * 4, grid);
  hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, LN_IN>), dim3(grid), dim3(T::THREADS), 0, s, g.A, g.lda, g.W,
                     g.bias, g.resid, g.ldr, g.out, g.ldo, g.M, g.N, g.K, ln, rx);
}

using GemmBig = F32Tile<2, 2, 2, 2>;    // 128 x 128
using GemmT96 = F32Tile<4, 1, 1, 3>;    // 128 x 96
using GemmMid = F32Tile<2, 2, 2, 1>;    // 128 x 64
using GemmSmall = F32Tile<1, 4, 1, 1>;  // 32 x 128  (few rows)

// Pick the tile whose launch wastes the least: every CU runs two workgroups at a time,
// so a grid that is not a multiple of 2*CUs idles part of the chip in its last round
// (M = 8192: N = 768 -> 128x96 gives exactly 512 tiles; 2304 -> 1536).  Cost model:
// rounds * tile area / relative tile efficiency.
using X6Big = F32Tile<2, 2, 2, 2, true>;  // 128 x 128, split-f32
using X6T96 = F32Tile<4, 1, 1, 3, true>;  // 128 x 96
using X6Mid = F32Tile<2, 2, 2, 1, true>;  // 128 x 64

// Tile codes (also the mq_debug_gemm_f32 `tile` argument): 0-3 exact f32 128x128 /
// 128x96 / 128x64 / 32x128, 4 split-K (host path only), 5-7 split-f32 128x128 / 128x96
// / 128x64, 8 / 9 exact / split-f32 128x192 with 8-wave workgroups (one per CU; measured
// within run-to-run noise of the 4-wave tiles, kept as a test of the 8-wave walker).
template <int EPI>
void launch_gemm_tile(const GemmArgs& g, int tile, int num_cus, hipStream_t s) {
  switch (tile) {
    case 0: launch_gemm_t<GemmBig, EPI>(g, num_cus, s); return;
    case 1: launch_gemm_t<GemmT96, EPI>(g, num_cus, s); return;
    case 2: launch_gemm_t<GemmMid, EPI>(g, num_cus, s); return;
    case 5: launch_gemm_t<X6Big, EPI>(g, num_cus, s); return;
    case 6: launch_gemm_t<X6T96, EPI>(g, num_cus, s); return;
    case 7: launch_gemm_t<X6Mid, EPI>(g, num_cus, s); return;
    case 8: launch_gemm_t<F32Tile<4, 2, 1, 3>, EPI>(g, num_cus, s); return;         // 128x192, 8 waves
    case 9: launch_gemm_t<F32Tile<4, 2, 1, 3, true>, EPI>(g, num_cus, s); return;   // x6 128x192
    default: launch_gemm_t<GemmSmall, EPI>(g, num_cus, s); return;
  }
}

// Split-K factor for a GEMM that would under-fill the chip (0 = run it directly):
// enough chunks for ~2 workgroups per CU, each chunk a multiple of 32 deep.
int splitk_factor(const GemmArgs& g, int num_cus, int cap = 16, int tiles_max = 0) {
  if (!g.slab || g.N % 4 != 0) return 0;
  const int64_t tiles = (int64_t)((g.M + 31) / 32) * ((g.N + 127) / 128);  // 32 x 128 tiles
  const int64_t slots = 2 * (int64_t)num_cus;
  // split only grids of at most tiles_max direct tiles (0: one tile per CU)
  if (tiles > (tiles_max > 0 ? tiles_max : num_cus) || g.M > 256) return 0;
  const int slices = g.K / kBK;
  // At most 16 chunks: deeper splits fill more CUs but the slab traffic and the ordered
  // reduction grow with S (single query, L=32: encoder p50 0.74 ms at 16 vs 0.88 ms at
  // 64, 0.80 ms at 8).  MQ_ENC_OPT_SPLITK_MAX overrides it.
  int best = 1;
  for (int s = 1; s <= slices && s <= cap; ++s)
    if (slices % s == 0 && tiles * s <= slots && (size_t)s * g.M * g.N <= g.slab_floats) best = s;
  return best >= 2 ? best : 0;
}

// The split-K partial GEMM on the 32 x 128 tile (g.nt: non-temporal weight loads).
void launch_splitk_gemm(const GemmArgs& g, int S, hipStream_t s) {
  auto go = [&](auto tile) {
    using T = decltype(tile);
    const int tiles = ((g.M + T::BM - 1) / T::BM) * ((g.N + T::BN - 1) / T::BN);
    hipLaunchKernelGGL((gemm_splitk_kernel<T>), dim3(tiles * S), dim3(256), 0, s, g.A, g.lda, g.W, g.M, g.N, g.K,
                       S, g.slab);
  };
  if (g.nt)
    go(F32Tile<1, 4, 1, 1, false, 2, false, 0, true>{});
  else
    go(F32Tile<1, 4, 1, 1>{});
}

template <int EPI>
void launch_splitk(const GemmArgs& g, int S, hipStream_t s) {
  launch_splitk_gemm(g, S, s);
  const int64_t n4 = (int64_t)g.M * g.N / 4;
  hipLaunchKernelGGL((splitk_reduce_kernel<EPI>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                     s, g.slab, S, g.M, g.N, g.bias, g.resid, g.ldr, g.out, g.ldo);
}

template <int EPI>
void launch_gemm(const GemmArgs& g, int num_cus, hipStream_t s, bool x6 = false, int splitk_cap = 16,
                 int splitk_tiles = 0) {
  const int S = splitk_factor(g, num_cus, splitk_cap, splitk_tiles);
  if (S) {
    launch_splitk<EPI>(g, S, s);
    return;
  }
  // split-f32 pays where its tiles fill the chip; a GEMM of fewer rows (a long single
  // query: M = 512 is 48 K2p tiles on 256 CUs) runs the exact-f32 tiles instead - narrower
  // tiles spread further, and exact f32 is at least as accurate (L = 512 single query:
  // 3.09-3.16 ms p50 on either split-f32 path, 2.45 on exact f32)
  if (x6 && (int64_t)((g.M + 127) / 128) * ((g.N + 191) / 192) < num_cus) x6 = false;
  if (x6 && g.W3) {  // split-f32 on the pre-split weights (K2p)
    launch_gemm_x6p(X6pArgs{g.A, g.lda, g.W3, g.bias, g.resid, g.ldr, g.out, g.ldo, g.M, g.N, g.K}, EPI, -1, num_cus,
                    s);
    return;
  }
  if (x6) {  // split-f32 tiles (both operands split while staged): same waste model over 128x{128,96,64}
    const int bns[3] = {128, 96, 64};
    const double effs[3] = {1.0, 0.96, 0.9};
    const int64_t slots = 2 * (int64_t)num_cus;
    int best = 0;
    double best_cost = 1e300;
    for (int i = 0; i < 3; ++i) {
      const int64_t tiles = (int64_t)((g.M + 127) / 128) * ((g.N + bns[i] - 1) / bns[i]);
      const double cost = (double)((tiles + slots - 1) / slots) * 128 * bns[i] / effs[i];
      if (cost < best_cost) {
        best_cost = cost;
        best = i;
      }
    }
    launch_gemm_tile<EPI>(g, 5 + best, num_cus, s);
    return;
  }
  struct Cand {
    int bm, bn;
    double eff;
  };
  const Cand cands[4] = {{128, 128, 1.0}, {128, 96, 0.96}, {128, 64, 0.9}, {32, 128, 0.55}};
  const int64_t slots = 2 * (int64_t)num_cus;
  int best = 0;
  double best_cost = 1e300;
  for (int i = 0; i < 4; ++i) {
    const int64_t tiles = (int64_t)((g.M + cands[i].bm - 1) / cands[i].bm) * ((g.N + cands[i].bn - 1) / cands[i].bn);
    const int64_t rounds = (tiles + slots - 1) / slots;
    const double cost = (double)rounds * cands[i].bm * cands[i].bn / cands[i].eff;
    if (cost < best_cost) {
      best_cost = cost;
      best = i;
    }
  }
  launch_gemm_tile<EPI>(g, best, num_cus, s);
}

// LayerNorm deferred into the consumer (LnArgs): the producer is the 128x96 tile (its wave
// tile is the partial width), the consumer the 128x128 or 128x96 tile by launch_gemm's
// waste model over those two.
void launch_gemm_stats(const GemmArgs& g, const LnArgs& ln, int num_cus, hipStream_t s) {
  launch_gemm_t<GemmT96, EPI_RESID_STATS>(g, num_cus, s, ln);
}

template <int EPI>
void launch_gemm_ln_in(const GemmArgs& g, const LnArgs& ln, int num_cus, hipStream_t s) {
  const int64_t slots = 2 * (int64_t)num_cus;
  auto cost = [&](int bn, double eff) {
    const int64_t tiles = (int64_t)((g.M + 127) / 128) * ((g.N + bn - 1) / bn);
    return (double)((tiles + slots - 1) / slots) * 128 * bn / eff;
  };
  if (cost(128, 1.0) <= cost(96, 0.96))
    launch_gemm_t<GemmBig, EPI, true>(g, num_cus, s, ln);
  else
    launch_gemm_t<GemmT96, EPI, true>(g, num_cus, s, ln);
}

// Stage labels for the optional per-kernel-class event timeline.
enum Stage { ST_EMBED = 0, ST_QKV, ST_ATTN, ST_OPROJ, ST_LN, ST_FFN_UP, ST_FFN_DOWN, ST_POOL, ST_N };


}  // namespace

struct mq_encoder {
  int device = 0;
  PinBuf pin;  // pinned staging of the host-pointer embed path (few tokens)
  mq_bert_config cfg{};
  int precision = MQ_DTYPE_F32;
  bool loaded = false;
  Buf weights;
  const float *word = nullptr, *pos = nullptr, *typ = nullptr, *eg = nullptr, *eb = nullptr;
  std::vector<LayerW> layers;
  Buf x, y, qkv, ctx, ffn, io_out, slab;  // (+ lnst below)
  Buf w3;  // split-f32: every layer's W3 plane images (LayerW::*3 point into it)
  Buf wfrag;  // every layer's frag16 weight images (LayerW::*f point into it), built at load
  int* io_ids = nullptr;
  int* io_mask = nullptr;
  size_t io_tokens = 0;
  Timeline tl;
  int num_cus = 256;
  // Replayed forwards: one hipGraph per (B, L, precision, buffer set), captured on a
  // private stream from io_ids/io_mask to io_out and launched on the caller's stream.
  struct Graph {
    int B = 0, L = 0, precision = 0;
    std::vector<const void*> bufs;
    hipGraphExec_t exec = nullptr;
    uint64_t last_use = 0;
  };
  std::vector<Graph> graphs;
  // tuning options (mq_encoder_set_option)
  bool fuse_attn_oproj = true;  // few-row forward: K3o (attention + output projection)
  int rows_max = kRowsDefault;  // few-row forward up to this many token rows (0 = off)
  int rows_splits = 0;          // few-row FFN-down K splits (0 = automatic)
  int splitk_max = 16;          // deepest split-K of the tiled path's few-row GEMMs
  int splitk_tiles = 0;         // split-K only grids of <= this many 32x128 tiles (0 = num_cus)
  int ln_rows_per_wave = 4;     // batched LayerNorm kernel: rows per wave
  bool fused_ln = false;        // batched residual GEMMs: LayerNorm in the epilogue (full-row tiles;
                                // measured slower, kept as an option: DESIGN.md §4)
  int resident_layers = 8;      // few-row forward: layers whose weights load with the default
                                // cache policy (8 x 28 MB of BERT-base fit the 256 MB MALL);
                                // later layers' loads are non-temporal
  bool ln_on_load = false;      // batched forward: LayerNorm applied by the consuming GEMM (LnArgs;
                                // measured slower: the consumers' staging VALU)
  Buf lnst;                     // its per-row partials, two sets of [M][H / kLnPartW] (mean, M2)
  bool x6_presplit = true;      // split-f32 batched GEMMs on the W3 images (K2p)
  bool rows_planes = false;     // few-row forward: keep the two-plane hand-offs (no FL_ACC merge)
  bool use_graphs = false;  // eager measured faster for one query (0.628 vs 0.645 ms: the
                            // graph path stages ids / mask / out through its own buffers)
  uint64_t graph_clock = 0;
  hipStream_t cap_stream = nullptr;
  std::mutex mu;
};

namespace {

// Split-f32 precision: split every layer's four projection weights once into their W3
// plane images (gemm_x6p.hpp; 6 B per weight, 510 MB for BERT-base), which the batched
// GEMMs (K2p) multiply without re-splitting them.  No-op unless the precision is F32X6 and
// weights are loaded, or when the images exist.  Synchronous.
int build_w3(mq_encoder* e) {
  if (e->precision != MQ_DTYPE_F32X6 || !e->loaded || e->layers.empty() || e->layers[0].wqkv3) return MQ_OK;
  const mq_bert_config& c = e->cfg;
  const int H = c.hidden, F = c.ffn;
  const size_t per = w3_bytes(3 * H, H) + w3_bytes(H, H) + w3_bytes(F, H) + w3_bytes(H, F);
  DeviceGuard dg(e->device);
  int rc = e->w3.ensure((per * e->layers.size() + 3) / 4);
  if (rc) return rc;
  unsigned char* p = reinterpret_cast<unsigned char*>(e->w3.p);
  for (LayerW& w : e->layers) {
    auto one = [&](const float* W, int n, int k, const unsigned char*& dst) {
      launch_split_w3(W, n, k, p, nullptr);
      dst = p;
      p += w3_bytes(n, k);
    };
    one(w.wqkv, 3 * H, H, w.wqkv3);
    one(w.wo, H, H, w.wo3);
    one(w.w1, F, H, w.w13);
    one(w.w2, H, F, w.w23);
  }
  MQ_HIP(hipGetLastError());
  MQ_HIP(hipStreamSynchronize(nullptr));
  return MQ_OK;
}

// The frag16 images of every layer's four projection weights (the few-row kernels' layout,
// rows_gemm_kernel / attn_oproj_rows_kernel; 4 B per weight, 340 MB for BERT-base beside the
// row-major blob the batched GEMMs read).  Synchronous.
int build_frag16(mq_encoder* e) {
  const mq_bert_config& c = e->cfg;
  const int64_t H = c.hidden, F = c.ffn;
  const int64_t per = 3 * H * H + H * H + F * H + H * F;
  DeviceGuard dg(e->device);
  int rc = e->wfrag.ensure((size_t)(per * (int64_t)e->layers.size()));
  if (rc) return rc;
  float* p = e->wfrag.p;
  for (LayerW& w : e->layers) {
    auto one = [&](const float* W, int64_t r, int64_t k, const float*& dst) {
      const int64_t n4 = r * k / 4;
      hipLaunchKernelGGL(frag16_image_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, nullptr, W, (int)r,
                         (int)k, reinterpret_cast<floatx4*>(p));
      dst = p;
      p += r * k;
    };
    one(w.wqkv, 3 * H, H, w.wqkvf);
    one(w.wo, H, H, w.wof);
    one(w.w1, F, H, w.w1f);
    one(w.w2, H, F, w.w2f);
  }
  MQ_HIP(hipGetLastError());
  MQ_HIP(hipStreamSynchronize(nullptr));
  return MQ_OK;
}

template <int EPI>
void gemm(mq_encoder* e, const GemmArgs& g, int stage, hipStream_t s) {
  e->tl.mark(s, stage);
  GemmArgs a = g;
  if (!e->x6_presplit) a.W3 = nullptr;
  launch_gemm<EPI>(a, e->num_cus, s, e->precision == MQ_DTYPE_F32X6, e->splitk_max, e->splitk_tiles);
}

// Residual projection + LayerNorm: x = LN(A W^T + b + resid), through y (g.out) on the
// tiled path; on the split-K (few-row) path the slab reduction, residual and LN run as
// one kernel writing x directly (bit-identical).  The fused form needs resid rows at
// stride H (a wave overwrites only the row it has read).
template <int VPL>
void gemm_resid_ln(mq_encoder* e, const GemmArgs& g, const float* lng, const float* lnb, float* x,
                   int stage, hipStream_t s) {
  const int H = VPL * 256;
  const unsigned rb = (unsigned)((g.M + 3) / 4);
  const int S = splitk_factor(g, e->num_cus, e->splitk_max, e->splitk_tiles);
  if constexpr (VPL <= 3) {  // (the 32 + H row image of hidden 1024 does not double-buffer in LDS)
    // full-row tiles with the LayerNorm in the epilogue: exact f32, unit-stride residual
    // rows written in place (the strided CLS-only layer's compact output would overwrite
    // residual rows other workgroups still read)
    if (!S && e->fused_ln && e->precision == MQ_DTYPE_F32 && g.ldr == H && g.N == H && g.resid == x) {
      using T = F32Tile<1, 8, 1, VPL, false, 2, false, 16>;
      e->tl.mark(s, stage);
      const int tiles = (g.M + 31) / 32;
      hipLaunchKernelGGL((gemm_resid_ln_kernel<T>), dim3(std::min(tiles, e->num_cus)), dim3(T::THREADS), 0, s,
                         g.A, g.lda, g.W, g.bias, g.resid, lng, lnb, e->cfg.ln_eps, x, g.M, g.K);
      return;
    }
  }
  if (S && g.ldr == H && g.N == H) {
    e->tl.mark(s, stage);
    launch_splitk_gemm(g, S, s);
    e->tl.mark(s, ST_LN);
    hipLaunchKernelGGL((splitk_reduce_ln_kernel<VPL>), dim3((unsigned)g.M), dim3(256), 0, s, g.slab, S,
                       g.M, g.bias, g.resid, g.ldr, lng, lnb, e->cfg.ln_eps, x);
    return;
  }
  gemm<EPI_RESID>(e, g, stage, s);
  e->tl.mark(s, ST_LN);
  const int rpw = e->ln_rows_per_wave;  // MQ_ENC_OPT_LN_ROWS_PER_WAVE: 1 / 2 / 4
  if (rpw == 4)
    hipLaunchKernelGGL((ln_kernel<VPL, 4>), dim3((unsigned)((g.M + 15) / 16)), dim3(256), 0, s, g.out, g.M, lng,
                       lnb, e->cfg.ln_eps, x);
  else if (rpw == 1)
    hipLaunchKernelGGL((ln_kernel<VPL, 1>), dim3(rb), dim3(256), 0, s, g.out, g.M, lng, lnb, e->cfg.ln_eps, x);
  else
    hipLaunchKernelGGL((ln_kernel<VPL, 2>), dim3((unsigned)((g.M + 7) / 8)), dim3(256), 0, s, g.out, g.M, lng,
                       lnb, e->cfg.ln_eps, x);
}

// One forward.  With CLS pooling the last layer only needs the CLS rows after its
// attention: its QKV projection runs on all tokens (keys / values), attention on the
// first 32-query tile, and the output projection, LayerNorms and FFN on the B CLS
// rows (strided views of the activations) - identical CLS outputs, ~8% less work.
template <int VPL>
int forward_vpl(mq_encoder* e, const int* ids, const int* mask, int B, int L, float* out,
                hipStream_t s) {
  const mq_bert_config& c = e->cfg;
  const int M = B * L, H = c.hidden, F = c.ffn;
  const unsigned row_blocks = (unsigned)((M + 3) / 4);
  const float scale = 1.0f / sqrtf((float)(H / c.heads));
  const int q_tiles = (L + 31) / 32;
  e->tl.mark(s, ST_EMBED);
  hipLaunchKernelGGL((embed_ln_kernel<VPL>), dim3(row_blocks), dim3(256), 0, s, ids, M, L,
                     c.vocab_size, e->word, e->pos, e->typ, e->eg, e->eb, c.ln_eps, e->x.p);
  // LayerNorm deferred into the consumers (LnArgs) on the full-M layers: exact f32, rows
  // enough for the tiled path, hidden a whole number of kLnPartW-column partials
  const int nt = H / kLnPartW;
  const bool lnl = e->ln_on_load && !e->fused_ln && e->precision == MQ_DTYPE_F32 && M > 256 &&
                   H == kLnPartW * kLnMaxParts && e->lnst.n >= (size_t)4 * M * nt;
  float* st1 = e->lnst.p;                          // out-proj -> FFN-up
  float* st2 = lnl ? e->lnst.p + (size_t)2 * M * nt : nullptr;  // FFN-down -> next QKV
  bool y_pending = false;  // x holds LN2's input y (+ st2) instead of the LayerNorm output
  const LayerW* prev = nullptr;
  auto ln_args = [&](const float* stats, const float* g, const float* b) {
    LnArgs a{};
    a.stats_in = stats;
    a.g = g;
    a.b = b;
    a.xout = e->x.p;
    a.ldx = H;
    a.nt = nt;
    a.eps = c.ln_eps;
    return a;
  };
  auto stats_out = [&](float* stats) {
    LnArgs a{};
    a.stats_out = stats;
    a.nt = nt;
    return a;
  };
  for (size_t li = 0; li < e->layers.size(); ++li) {
    const LayerW& w = e->layers[li];
    const bool cls_only = c.pooling == MQ_POOL_CLS && li + 1 == e->layers.size();
    // rows this layer carries past attention: all M tokens, or the B CLS rows
    const int rows = cls_only ? B : M;
    const int stride = cls_only ? L * H : H;  // row stride of x / ctx views
    // QKV input: x, or (deferred LN2 of the previous layer) y normalised while staged,
    // the column-0 tiles writing LN2(y) to x for the residual and the CLS-row Q GEMM
    const float* qkv_in = y_pending ? e->y.p : e->x.p;
    // few rows (single queries past the few-row limit): the layers past resident_layers
    // stream their weights non-temporally in the split-K GEMMs (as forward_rows does)
    const int lnt = M <= 256 && (int)li >= e->resident_layers ? 1 : 0;
    auto qkv_gemm = [&](GemmArgs g) {
      g.nt = lnt;
      if (y_pending) {
        e->tl.mark(s, ST_QKV);
        launch_gemm_ln_in<EPI_BIAS>(g, ln_args(st2, prev->ln2g, prev->ln2b), e->num_cus, s);
      } else {
        gemm<EPI_BIAS>(e, g, ST_QKV, s);
      }
    };
    if (cls_only && L > 1) {
      // only the CLS rows need queries: K and V for every token ([M, 2H] into qkv columns
      // H..3H), Q for the B CLS rows (every L-th row of x into row b*L of qkv)
      GemmArgs kv{e->slab.p, e->slab.n, qkv_in, H, w.wqkv + (int64_t)H * H, w.bqkv + H, nullptr, 0, e->qkv.p + H,
                  3 * H, M, 2 * H, H};
      if (w.wqkv3) kv.W3 = w.wqkv3 + w3_row_offset(H, H);
      qkv_gemm(kv);
      GemmArgs q{e->slab.p, e->slab.n, e->x.p, L * H, w.wqkv, w.bqkv, nullptr, 0, e->qkv.p, L * 3 * H, B, H, H, lnt};
      q.W3 = w.wqkv3;
      gemm<EPI_BIAS>(e, q, ST_QKV, s);
    } else {
      GemmArgs qkv{e->slab.p, e->slab.n, qkv_in, H, w.wqkv, w.bqkv, nullptr, 0, e->qkv.p, 3 * H, M, 3 * H, H};
      qkv.W3 = w.wqkv3;
      qkv_gemm(qkv);
    }
    y_pending = false;
    e->tl.mark(s, ST_ATTN);
    const int qt = cls_only ? 1 : q_tiles;
    launch_attention(B, L, c.heads, qt, H, scale, e->qkv.p, mask, e->ctx.p, s);
    const bool lnl_layer = lnl && !cls_only;
    // x = LN1(x + ctx Wo^T + bo)  (compact [rows, H], through y) - or, deferred, y + partials
    GemmArgs oproj{e->slab.p, e->slab.n, e->ctx.p, stride, w.wo, w.bo, e->x.p, stride, e->y.p, H, rows, H, H, lnt};
    oproj.W3 = w.wo3;
    if (lnl_layer) {
      e->tl.mark(s, ST_OPROJ);
      launch_gemm_stats(oproj, stats_out(st1), e->num_cus, s);
    } else {
      gemm_resid_ln<VPL>(e, oproj, w.ln1g, w.ln1b, e->x.p, ST_OPROJ, s);
    }
    GemmArgs up{e->slab.p, e->slab.n, lnl_layer ? e->y.p : e->x.p, H, w.w1, w.b1, nullptr, 0, e->ffn.p, F,
                rows, F, H, lnt};
    up.W3 = w.w13;
    if (lnl_layer) {  // FFN-up normalises y (LN1) while staging; its column-0 tiles write x
      e->tl.mark(s, ST_FFN_UP);
      if (c.gelu == MQ_GELU_TANH)
        launch_gemm_ln_in<EPI_GELU_TANH>(up, ln_args(st1, w.ln1g, w.ln1b), e->num_cus, s);
      else
        launch_gemm_ln_in<EPI_GELU_ERF>(up, ln_args(st1, w.ln1g, w.ln1b), e->num_cus, s);
    } else if (c.gelu == MQ_GELU_TANH) {
      gemm<EPI_GELU_TANH>(e, up, ST_FFN_UP, s);
    } else {
      gemm<EPI_GELU_ERF>(e, up, ST_FFN_UP, s);
    }
    GemmArgs down{e->slab.p, e->slab.n, e->ffn.p, F, w.w2, w.b2, e->x.p, H, e->y.p, H, rows, H, F, lnt};
    down.W3 = w.w23;
    if (lnl_layer && li + 1 < e->layers.size()) {  // LN2 deferred into the next layer's QKV
      e->tl.mark(s, ST_FFN_DOWN);
      launch_gemm_stats(down, stats_out(st2), e->num_cus, s);
      y_pending = true;
    } else {
      gemm_resid_ln<VPL>(e, down, w.ln2g, w.ln2b, e->x.p, ST_FFN_DOWN, s);
    }
    prev = &w;
  }
  e->tl.mark(s, ST_POOL);
  const bool pruned = c.pooling == MQ_POOL_CLS;  // x holds [B, H] CLS rows
  hipLaunchKernelGGL((pool_kernel<VPL>), dim3((B + 3) / 4), dim3(256), 0, s, e->x.p, mask, B,
                     pruned ? 1 : L, c.pooling, out);
  e->tl.close(s);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// ------------------------------------------------------- few-row forward ------
struct RowsArgs {
  const float* A;
  int lda;
  int64_t a_plane;  // LN_IN: floats between the summed input planes
  const float* W;
  int ldw;
  const float* bias;
  const float* resid;
  int ldr;
  float* out;
  int ldo;
  int64_t o_plane;  // floats between the output planes of a K split
  int M, N, K;      // K: full depth (ldw >= K)
  int splits;       // K splits (grid.z), each writing one output plane
  // LN_IN with s_in = 0: A is the word-embedding table, rows gathered by token id
  const int* ids = nullptr;
  int L = 1, vocab = 0;
  const float* pos = nullptr;
  const float* typ = nullptr;
  int nt_w = 0;  // weights loaded non-temporally (layers past resident_layers)
  float* zbuf = nullptr;  // zn floats this launch zeroes for a later launch's FL_ACC adds
  int64_t zn = 0;
};

// Row tiles per workgroup: two for the LayerNorm-input GEMMs when M > 16 (the launch then
// streams each weight panel once instead of once per 16-row tile: QKV 10.5 -> 9.0 us,
// FFN-up 10.1 -> 8.6 us at M = 32), unless the normalised rows would not fit LDS (hidden
// 1024).  The plain GEMMs keep one: with half the workgroups their per-CU bytes, not the
// chip's, bound them (FFN-down 7.8 -> 10.9 us with two).
template <int EPI, bool LN_IN, int VPL, int NB, int S_IN, int RT, int FL>
void launch_rows_rt(const RowsArgs& g, const float* lng, const float* lnb, float eps, float* ln_out,
                    hipStream_t s) {
  hipLaunchKernelGGL((rows_gemm_kernel<EPI, LN_IN, VPL, NB, S_IN, RT, FL>),
                     dim3(g.N / kRT, (g.M + kRT * RT - 1) / (kRT * RT), g.splits), dim3(64 * kRWaves), 0, s,
                     g.A, g.lda, g.a_plane, g.M, lng, lnb, eps, ln_out, g.W, g.ldw, g.bias, g.resid, g.ldr,
                     g.out, g.ldo, g.o_plane, g.ids, g.L, g.vocab, g.pos, g.typ, g.nt_w, g.zbuf, g.zn);
}

template <int EPI, bool LN_IN, int VPL, int NB, int S_IN, int FL = 0>
void launch_rows_nb(const RowsArgs& g, const float* lng, const float* lnb, float eps, float* ln_out,
                    hipStream_t s) {
  constexpr bool two_fit = LN_IN && (size_t)(2 * kRT * (NB * 256 + 4) + kRWaves * 2 * kRT * kRT) * 4 <= 160 * 1024;
  if constexpr (two_fit) {
    if (g.M > kRT) {
      launch_rows_rt<EPI, LN_IN, VPL, NB, S_IN, 2, FL>(g, lng, lnb, eps, ln_out, s);
      return;
    }
  }
  launch_rows_rt<EPI, LN_IN, VPL, NB, S_IN, 1, FL>(g, lng, lnb, eps, ln_out, s);
}

// Per-split depths the few-row kernel is instantiated for (K / 256 blocks per wave).
bool rows_nb_ok(int nb) { return nb >= 1 && (nb <= 4 || nb == 6 || nb == 8 || nb == 12 || nb == 16); }

// K splits for a depth-K projection: the fewest with per-split depth <= 1536, at most 4.
// More splits put more workgroups on the weights but add planes the consumer sums (at
// K = 3072, encoder p50: one split 13.9 us per FFN-down launch; two 0.474 ms, three 0.495,
// four 0.493 - FFN-down 8.9 / 9.2 / 7.1 us, the next QKV 9.2 / 10.0 / 11.0 us).
int rows_splits(int K, int forced = 0) {  // forced: MQ_ENC_OPT_ROWS_SPLITS, used when it divides K / 256
  const int nb = K / 256;
  if (forced >= 1 && forced <= 4 && nb % forced == 0 && rows_nb_ok(nb / forced)) return forced;
  for (int sp = 1; sp <= 4; ++sp)
    if (nb % sp == 0 && nb / sp <= 6 && rows_nb_ok(nb / sp)) return sp;
  return 1;
}

template <int EPI, int NB, int FL>
void launch_rows_plain(const RowsArgs& g, hipStream_t s) {
  launch_rows_nb<EPI, false, 1, NB, 1, FL>(g, nullptr, nullptr, 0.f, nullptr, s);
}

// No LayerNorm on A: any instantiated per-split depth; FL_A: A in frag16 (FFN-up's output).
template <int EPI, int FL = 0>
void launch_rows(const RowsArgs& g, hipStream_t s) {
  switch (g.K / g.splits / 256) {
    case 1: launch_rows_plain<EPI, 1, FL>(g, s); return;
    case 2: launch_rows_plain<EPI, 2, FL>(g, s); return;
    case 3: launch_rows_plain<EPI, 3, FL>(g, s); return;
    case 4: launch_rows_plain<EPI, 4, FL>(g, s); return;
    case 6: launch_rows_plain<EPI, 6, FL>(g, s); return;
    case 8: launch_rows_plain<EPI, 8, FL>(g, s); return;
    case 12: launch_rows_plain<EPI, 12, FL>(g, s); return;
    default: launch_rows_plain<EPI, 16, FL>(g, s); return;
  }
}

// A = LN(sum of s_in planes) with K == H, the normalised rows also to ln_out (may be null);
// s_in = 0: A = LN(embedding sum) gathered by token id (g.ids, g.pos, g.typ).
template <int EPI, int VPL, int FL = 0>
void launch_rows_ln(const RowsArgs& g, int s_in, const float* lng, const float* lnb, float eps,
                    float* ln_out, hipStream_t s) {
  switch (s_in) {
    case 0: launch_rows_nb<EPI, true, VPL, VPL, 0, FL>(g, lng, lnb, eps, ln_out, s); return;
    case 1: launch_rows_nb<EPI, true, VPL, VPL, 1, FL>(g, lng, lnb, eps, ln_out, s); return;
    case 2: launch_rows_nb<EPI, true, VPL, VPL, 2, FL>(g, lng, lnb, eps, ln_out, s); return;
    case 3: launch_rows_nb<EPI, true, VPL, VPL, 3, FL>(g, lng, lnb, eps, ln_out, s); return;
    default: launch_rows_nb<EPI, true, VPL, VPL, 4, FL>(g, lng, lnb, eps, ln_out, s); return;
  }
}

template <int HG, bool QF, bool ACC>
void launch_attn_oproj_hg(int nkb, dim3 grid, hipStream_t s, const float* qkv, const int* mask, int L, int H,
                          int rps, int qtiles, float scale, const float* wo, const float* bo, const float* resid,
                          int ldr, float* out, int64_t o_plane, int nt_w) {
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(512), 0, s, qkv, mask, L, H, rps, qtiles, scale, wo, bo, resid, ldr, out,
                       o_plane, nt_w);
  };
  switch (nkb) {
    case 1: go(attn_oproj_rows_kernel<HG, 1, QF, ACC>); break;
    case 2: go(attn_oproj_rows_kernel<HG, 2, QF, ACC>); break;
    case 3: go(attn_oproj_rows_kernel<HG, 3, QF, ACC>); break;
    default: go(attn_oproj_rows_kernel<HG, 4, QF, ACC>); break;
  }
}

// acc: the two head-group planes added into one zeroed plane (hg = heads / 2 only)
void launch_attn_oproj(int hg, bool qf, bool acc, int nkb, dim3 grid, hipStream_t s, const float* qkv,
                       const int* mask, int L, int H, int rps, int qtiles, float scale, const float* wo,
                       const float* bo, const float* resid, int ldr, float* out, int64_t o_plane, int nt_w) {
  auto go = [&](auto hgc, auto qfc, auto accc) {
    launch_attn_oproj_hg<decltype(hgc)::value, decltype(qfc)::value, decltype(accc)::value>(
        nkb, grid, s, qkv, mask, L, H, rps, qtiles, scale, wo, bo, resid, ldr, out, o_plane, nt_w);
  };
  if (hg == 6) {
    if (qf && acc) go(IC<6>{}, std::true_type{}, std::true_type{});
    else if (qf) go(IC<6>{}, std::true_type{}, std::false_type{});
    else if (acc) go(IC<6>{}, std::false_type{}, std::true_type{});
    else go(IC<6>{}, std::false_type{}, std::false_type{});
  } else {
    if (qf && acc) go(IC<4>{}, std::true_type{}, std::true_type{});
    else if (qf) go(IC<4>{}, std::true_type{}, std::false_type{});
    else if (acc) go(IC<4>{}, std::false_type{}, std::true_type{});
    else go(IC<4>{}, std::false_type{}, std::false_type{});
  }
}

// Heads per output plane of the fused attention + output projection (K3o), 0 = run
// attention and the projection as two launches (keys past 64, or a head count neither
// 6 nor 4 divides).  6 at BERT-base (12 heads: two planes).
int oproj_heads_per_plane(const mq_encoder* e, int L) {
  const mq_bert_config& c = e->cfg;
  if (!e->fuse_attn_oproj || L > 64 || c.hidden != c.heads * kDh || c.hidden % kOpCols) return 0;
  return c.heads % 6 == 0 ? 6 : c.heads % 4 == 0 ? 4 : 0;
}

// Few-row forward (B * L <= kRowsMax): 5 launches per layer instead of 9, 5 L + 1 in all.  Between
// layers the activations stay pre-LayerNorm, as the FFN-down's split-K planes in `slab`;
// the next GEMM sums and normalises them on load (K2r LN_IN) and materialises the
// normalised rows in x for the residual:
//   QKV   qkv = LN2'(sum slab) Wqkv^T + b  (x = LN2'(...); layer 0: LN of the gathered
//         embedding sum, so the forward has no separate embedding launch)
//   attn  ctx
//   oproj y = ctx Wo^T + bo + x
//   up    ffn = GELU(LN1(y) W1^T + b1)     (x = LN1(y))
//   down  slab[z] = ffn[:, Kz] W2[:, Kz]^T (+ b2 + x for z = 0)
// and ln_pool applies the last LN2 to the pooled rows.  The CLS-only last layer carries
// the B CLS rows past attention as forward_vpl does.
template <int VPL>
int forward_rows(mq_encoder* e, const int* ids, const int* mask, int B, int L, float* out,
                 hipStream_t s) {
  const mq_bert_config& c = e->cfg;
  const int M = B * L, H = c.hidden, F = c.ffn;
  const float eps = c.ln_eps;
  const float scale = 1.0f / sqrtf((float)(H / c.heads));
  const int q_tiles = (L + 31) / 32;
  const int dsplit = rows_splits(F, e->rows_splits);
  const int hg = oproj_heads_per_plane(e, L);
  // QKV -> K3o through frag16 (Q, K, V^T blocks) when every sequence starts a 16-row block
  const bool qf = hg != 0 && L % 16 == 0 && (3 * H) % 48 == 0;
  // two-addend plane merges (FL_ACC): FFN-down's two K splits and K3o's two head groups add
  // into one zeroed plane, so QKV and FFN-up read one plane of rows instead of two (the
  // buffer each zeroes: the slab by FFN-up, y by QKV, a launch ahead of the adds)
  const bool dacc = dsplit == 2 && !e->rows_planes;
  const bool yacc = hg != 0 && c.heads / hg == 2 && !e->rows_planes;
  int prev_rows = M;
  for (size_t li = 0; li < e->layers.size(); ++li) {
    const LayerW& w = e->layers[li];
    const bool cls_only = c.pooling == MQ_POOL_CLS && li + 1 == e->layers.size();
    const int rows = cls_only ? B : M;
    const int stride = cls_only ? L * H : H;
    const int nt = (int)li >= e->resident_layers ? 1 : 0;  // this layer's weights bypass MALL
    e->tl.mark(s, ST_QKV);
    RowsArgs qkv{e->slab.p, H, (int64_t)prev_rows * H, w.wqkvf, H, w.bqkv, nullptr, 0, e->qkv.p, 3 * H, 0, M, 3 * H, H, 1};
    qkv.nt_w = nt;
    if (li == 0) {  // the embedding gather + LayerNorm run inside the first QKV launch
      qkv.A = e->word;
      qkv.a_plane = 0;
      qkv.ids = ids;
      qkv.L = L;
      qkv.vocab = c.vocab_size;
      qkv.pos = e->pos;
      qkv.typ = e->typ;
    }
    const LayerW* pl = li ? &e->layers[li - 1] : nullptr;
    const float* lg = pl ? pl->ln2g : e->eg;
    const float* lb = pl ? pl->ln2b : e->eb;
    const int s_in = pl ? (dacc ? 1 : dsplit) : 0;
    if (yacc) {  // K3o of this layer adds into y
      qkv.zbuf = e->y.p;
      qkv.zn = (int64_t)rows * H;
    }
    if (qf)  // K3o reads Q, K, V^T as whole frag16 blocks
      ROWS_REP launch_rows_ln<EPI_BIAS, VPL, FL_O | FL_OT>(qkv, s_in, lg, lb, eps, e->x.p, s);
    else
      ROWS_REP launch_rows_ln<EPI_BIAS, VPL>(qkv, s_in, lg, lb, eps, e->x.p, s);
    const int qt = cls_only ? 1 : q_tiles;
    int y_planes = 1;
    if (hg) {  // attention + output projection in one launch (K3o), hg heads per plane
      e->tl.mark(s, ST_OPROJ);
      const int rps = cls_only ? 1 : L, qtiles = (rps + 15) / 16;
      y_planes = c.heads / hg;
      const dim3 grid(H / kOpCols, B * qtiles, y_planes);
      if (yacc) y_planes = 1;
      ROWS_REP launch_attn_oproj(hg, qf, yacc, (L + 15) / 16, grid, s, e->qkv.p, mask, L, H, rps, qtiles, scale, w.wof, w.bo, e->x.p,
                                 stride, e->y.p, (int64_t)rows * H, nt);
    } else {
      e->tl.mark(s, ST_ATTN);
      if (L <= 64)
        hipLaunchKernelGGL(attention_rows_kernel, dim3(B * c.heads * qt), dim3(512), 0, s, e->qkv.p, mask, L,
                           H, c.heads, qt, scale, e->ctx.p);
      else
        launch_attention(B, L, c.heads, qt, H, scale, e->qkv.p, mask, e->ctx.p, s);
      e->tl.mark(s, ST_OPROJ);
      RowsArgs oproj{e->ctx.p, stride, 0, w.wof, H, w.bo, e->x.p, stride, e->y.p, H, 0, rows, H, H, 1};
      oproj.nt_w = nt;
      launch_rows<EPI_RESID>(oproj, s);
    }
    e->tl.mark(s, ST_FFN_UP);
    // FFN-up writes the GELU rows in frag16 for FFN-down's A operand
    RowsArgs up{e->y.p, H, (int64_t)rows * H, w.w1f, H, w.b1, nullptr, 0, e->ffn.p, F, 0, rows, F, H, 1};
    up.nt_w = nt;
    if (dacc) {  // FFN-down of this layer adds into the slab
      up.zbuf = e->slab.p;
      up.zn = (int64_t)rows * H;
    }
    if (c.gelu == MQ_GELU_TANH)
      ROWS_REP launch_rows_ln<EPI_GELU_TANH, VPL, FL_O>(up, y_planes, w.ln1g, w.ln1b, eps, e->x.p, s);
    else
      ROWS_REP launch_rows_ln<EPI_GELU_ERF, VPL, FL_O>(up, y_planes, w.ln1g, w.ln1b, eps, e->x.p, s);
    e->tl.mark(s, ST_FFN_DOWN);
    RowsArgs down{e->ffn.p, F, 0, w.w2f, F, w.b2, e->x.p, H, e->slab.p, H, (int64_t)rows * H, rows, H, F, dsplit};
    down.nt_w = nt;
    if (dacc)
      ROWS_REP launch_rows<EPI_RESID, FL_A | FL_ACC>(down, s);
    else
      ROWS_REP launch_rows<EPI_RESID, FL_A>(down, s);
    prev_rows = rows;
  }
  e->tl.mark(s, ST_POOL);
  const LayerW& last = e->layers.back();
  const int pool_rows = c.pooling == MQ_POOL_CLS ? 1 : L;  // slab holds [B, H] CLS rows or [M, H]
  hipLaunchKernelGGL((ln_pool_kernel<VPL>), dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, e->slab.p, dacc ? 1 : dsplit,
                     (int64_t)prev_rows * H, mask, B, L, pool_rows, c.pooling, last.ln2g, last.ln2b, eps, out);
  e->tl.close(s);
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

// The few-row forward serves B * L <= rows_max token rows (MQ_ENC_OPT_ROWS_MAX, default
// 64: a single query up to 64 tokens; 0 turns it off).
bool use_rows_path(const mq_encoder* e, int B, int L) {
  const mq_bert_config& c = e->cfg;
  const int sp = rows_splits(c.ffn, e->rows_splits);
  // slab holds the FFN-down planes: splits x rows x H floats
  return (int64_t)B * L <= e->rows_max && !e->layers.empty() && c.ffn % 256 == 0 &&
         rows_nb_ok(c.ffn / 256 / sp) && (size_t)sp * B * L * c.hidden <= e->slab.n &&
         e->layers[0].wqkvf != nullptr;  // (the frag16 weight images)
}

}  // namespace

namespace {

int forward(mq_encoder* e, const int* ids, const int* mask, int B, int L, float* out,
            hipStream_t s) {
  const bool rows = use_rows_path(e, B, L);
  switch (e->cfg.hidden) {
    case 256: return rows ? forward_rows<1>(e, ids, mask, B, L, out, s) : forward_vpl<1>(e, ids, mask, B, L, out, s);
    case 512: return rows ? forward_rows<2>(e, ids, mask, B, L, out, s) : forward_vpl<2>(e, ids, mask, B, L, out, s);
    case 768: return rows ? forward_rows<3>(e, ids, mask, B, L, out, s) : forward_vpl<3>(e, ids, mask, B, L, out, s);
    default: return rows ? forward_rows<4>(e, ids, mask, B, L, out, s) : forward_vpl<4>(e, ids, mask, B, L, out, s);
  }
}

constexpr size_t kMaxGraphs = 6;

// Replay the forward io_ids/io_mask -> io_out for (B, L) as one hipGraph launch on s,
// capturing it first if no cached graph matches the shape, precision and buffers.
int launch_graph(mq_encoder* e, int B, int L, hipStream_t s) {
  const std::vector<const void*> bufs = {e->weights.p, e->x.p,   e->y.p,      e->qkv.p,
                                         e->ctx.p,     e->ffn.p, e->slab.p,   e->io_out.p,
                                         e->io_ids,    e->io_mask,  e->w3.p,   e->wfrag.p};
  mq_encoder::Graph* hit = nullptr;
  for (auto& g : e->graphs)
    if (g.B == B && g.L == L && g.precision == e->precision && g.bufs == bufs) hit = &g;
  if (!hit) {
    if (!e->cap_stream) MQ_HIP(hipStreamCreateWithFlags(&e->cap_stream, hipStreamNonBlocking));
    // drop graphs that reference freed buffers, then the least recently used
    for (size_t i = 0; i < e->graphs.size();) {
      if (e->graphs[i].bufs != bufs) {
        (void)hipGraphExecDestroy(e->graphs[i].exec);
        e->graphs.erase(e->graphs.begin() + i);
      } else {
        ++i;
      }
    }
    if (e->graphs.size() >= kMaxGraphs) {
      auto lru = std::min_element(e->graphs.begin(), e->graphs.end(),
                                  [](const auto& a, const auto& b) { return a.last_use < b.last_use; });
      (void)hipGraphExecDestroy(lru->exec);
      e->graphs.erase(lru);
    }
    hipGraph_t graph = nullptr;
    MQ_HIP(hipStreamBeginCapture(e->cap_stream, hipStreamCaptureModeThreadLocal));
    const int rc = forward(e, e->io_ids, e->io_mask, B, L, e->io_out.p, e->cap_stream);
    const hipError_t end = hipStreamEndCapture(e->cap_stream, &graph);
    if (rc) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    if (end != hipSuccess) MQ_FAIL(MQ_EHIP, "graph capture failed: %s", hipGetErrorString(end));
    mq_encoder::Graph g;
    g.B = B;
    g.L = L;
    g.precision = e->precision;
    g.bufs = bufs;
    const hipError_t inst = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (inst != hipSuccess) MQ_FAIL(MQ_EHIP, "graph instantiate failed: %s", hipGetErrorString(inst));
    e->graphs.push_back(g);
    hit = &e->graphs.back();
  }
  hit->last_use = ++e->graph_clock;
  MQ_HIP(hipGraphLaunch(hit->exec, s));
  return MQ_OK;
}

}  // namespace

extern "C" {

int64_t mq_encoder_weight_count(const mq_bert_config* cfg) {
  if (!cfg) return -1;
  return weight_count(*cfg);
}

int mq_encoder_create(int device, const mq_bert_config* cfg, mq_encoder** out) {
  clear_error();
  MQ_CHECK_ARG(out && cfg, "NULL argument");
  *out = nullptr;
  const mq_bert_config& c = *cfg;
  MQ_CHECK_ARG(c.hidden == 256 || c.hidden == 512 || c.hidden == 768 || c.hidden == 1024,
               "hidden must be 256/512/768/1024 (got %d)", c.hidden);
  MQ_CHECK_ARG(c.heads > 0 && c.hidden / c.heads == kDh && c.hidden % c.heads == 0,
               "head dim must be %d (hidden %d, heads %d)", kDh, c.hidden, c.heads);
  MQ_CHECK_ARG(c.ffn > 0 && c.ffn % kBK == 0, "ffn must be a positive multiple of %d", kBK);
  MQ_CHECK_ARG(c.layers >= 1 && c.vocab_size > 0 && c.max_positions > 0 && c.type_vocab > 0,
               "bad config");
  MQ_CHECK_ARG(c.gelu == MQ_GELU_ERF || c.gelu == MQ_GELU_TANH, "bad gelu variant");
  MQ_CHECK_ARG(c.pooling == MQ_POOL_CLS || c.pooling == MQ_POOL_MEAN, "bad pooling");
  DeviceGuard dg(device);
  if (!dg.ok) MQ_FAIL(MQ_EHIP, "hipSetDevice(%d) failed", device);
  auto e = std::make_unique<mq_encoder>();
  e->device = device;
  e->cfg = c;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      cus > 0)
    e->num_cus = cus;
  *out = e.release();
  return MQ_OK;
}

int mq_encoder_destroy(mq_encoder* e) {
  clear_error();
  if (!e) return MQ_OK;
  {
    DeviceGuard dg(e->device);
    for (Buf* b : {&e->weights, &e->x, &e->y, &e->qkv, &e->ctx, &e->ffn, &e->io_out, &e->slab, &e->w3, &e->wfrag,
                   &e->lnst})
      b->release();
    if (e->io_ids) (void)hipFree(e->io_ids);
    if (e->io_mask) (void)hipFree(e->io_mask);
    e->pin.release();
    for (auto& g : e->graphs) (void)hipGraphExecDestroy(g.exec);
    if (e->cap_stream) (void)hipStreamDestroy(e->cap_stream);
  }
  delete e;
  return MQ_OK;
}

int mq_encoder_load_weights(mq_encoder* e, const float* blob, int64_t n_floats) {
  clear_error();
  MQ_CHECK_ARG(e && blob, "NULL argument");
  const mq_bert_config& c = e->cfg;
  const int64_t need = weight_count(c);
  MQ_CHECK_ARG(n_floats == need, "weight blob has %lld floats, config needs %lld",
               (long long)n_floats, (long long)need);
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg(e->device);
  int rc = e->weights.ensure((size_t)need);
  if (rc) return rc;
  MQ_HIP(hipMemcpy(e->weights.p, blob, (size_t)need * 4, hipMemcpyHostToDevice));
  const int64_t H = c.hidden, F = c.ffn;
  const float* p = e->weights.p;
  auto take = [&](int64_t n) {
    const float* r = p;
    p += n;
    return r;
  };
  e->word = take((int64_t)c.vocab_size * H);
  e->pos = take((int64_t)c.max_positions * H);
  e->typ = take((int64_t)c.type_vocab * H);
  e->eg = take(H);
  e->eb = take(H);
  e->layers.clear();
  for (int l = 0; l < c.layers; ++l) {
    LayerW w;
    w.wqkv = take(3 * H * H);
    w.bqkv = take(3 * H);
    w.wo = take(H * H);
    w.bo = take(H);
    w.ln1g = take(H);
    w.ln1b = take(H);
    w.w1 = take(F * H);
    w.b1 = take(F);
    w.w2 = take(H * F);
    w.b2 = take(H);
    w.ln2g = take(H);
    w.ln2b = take(H);
    e->layers.push_back(w);
  }
  e->loaded = true;
  if (H % 16 == 0 && F % 16 == 0) {  // (the few-row path needs them: use_rows_path checks)
    rc = build_frag16(e);
    if (rc) return rc;
  }
  return build_w3(e);  // (re)split the new weights when the split-f32 precision is selected
}

int mq_encoder_set_precision(mq_encoder* e, int dtype) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  MQ_CHECK_ARG(dtype == MQ_DTYPE_F32 || dtype == MQ_DTYPE_F32X6,
               "encoder precision must be MQ_DTYPE_F32 or MQ_DTYPE_F32X6 (got %d)", dtype);
  std::lock_guard<std::mutex> lk(e->mu);
  e->precision = dtype;
  return build_w3(e);
}

int mq_debug_gemm_f32(const float* A, const float* W, const float* bias, const float* resid,
                      float* out, int M, int N, int K, int epi, int tile, void* stream) {
  clear_error();
  MQ_CHECK_ARG(A && W && bias && out && (epi != EPI_RESID || resid), "NULL buffer");
  MQ_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % kBK == 0, "bad shape M=%d N=%d K=%d", M, N, K);
  MQ_CHECK_ARG(epi >= 0 && epi <= 3 && tile >= 0 && tile <= 9, "bad epi/tile");
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  GemmArgs g{nullptr, 0, A, K, W, bias, resid, N, out, N, M, N, K};
  hipStream_t s = (hipStream_t)stream;
  if (tile == 4) {  // split-K path (test hook: allocates its own slab)
    MQ_CHECK_ARG(N % 4 == 0, "split-K needs N %% 4 == 0");
    const int slices = K / kBK;
    int S = 1;
    for (int c = 2; c <= slices && c <= 64; ++c)
      if (slices % c == 0) S = c;
    float* slab = nullptr;
    if (hipMalloc((void**)&slab, (size_t)S * M * N * 4) != hipSuccess)
      MQ_FAIL(MQ_ENOMEM, "slab allocation failed");
    g.slab = slab;
    g.slab_floats = (size_t)S * M * N;
    switch (epi) {
      case EPI_BIAS: launch_splitk<EPI_BIAS>(g, S, s); break;
      case EPI_GELU_ERF: launch_splitk<EPI_GELU_ERF>(g, S, s); break;
      case EPI_GELU_TANH: launch_splitk<EPI_GELU_TANH>(g, S, s); break;
      default: launch_splitk<EPI_RESID>(g, S, s); break;
    }
    const hipError_t err = hipStreamSynchronize(s);
    (void)hipFree(slab);
    if (err != hipSuccess) MQ_FAIL(MQ_EHIP, "split-K GEMM failed: %s", hipGetErrorString(err));
    return MQ_OK;
  }
  switch (epi) {
    case EPI_BIAS: launch_gemm_tile<EPI_BIAS>(g, tile, cus, s); break;
    case EPI_GELU_ERF: launch_gemm_tile<EPI_GELU_ERF>(g, tile, cus, s); break;
    case EPI_GELU_TANH: launch_gemm_tile<EPI_GELU_TANH>(g, tile, cus, s); break;
    default: launch_gemm_tile<EPI_RESID>(g, tile, cus, s); break;
  }
  MQ_HIP(hipGetLastError());
  return MQ_OK;
}

int mq_encoder_set_graphs(mq_encoder* e, int enabled) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  std::lock_guard<std::mutex> lk(e->mu);
  e->use_graphs = enabled != 0;
  return MQ_OK;
}

int mq_encoder_set_option(mq_encoder* e, int option, int value) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  std::lock_guard<std::mutex> lk(e->mu);
  switch (option) {
    case MQ_ENC_OPT_ROWS_MAX:
      MQ_CHECK_ARG(value >= 0 && value <= kRowsMax, "rows_max must be in [0, %d] (got %d)", kRowsMax, value);
      e->rows_max = value;
      break;
    case MQ_ENC_OPT_ROWS_SPLITS:
      MQ_CHECK_ARG(value >= 0 && value <= 4, "rows_splits must be in [0, 4] (got %d)", value);
      e->rows_splits = value;
      break;
    case MQ_ENC_OPT_SPLITK_MAX:
      MQ_CHECK_ARG(value >= 2 && value <= 64, "splitk_max must be in [2, 64] (got %d)", value);
      e->splitk_max = value;
      break;
    case MQ_ENC_OPT_LN_ROWS_PER_WAVE:
      MQ_CHECK_ARG(value == 1 || value == 2 || value == 4, "ln_rows_per_wave must be 1, 2 or 4 (got %d)", value);
      e->ln_rows_per_wave = value;
      break;
    case MQ_ENC_OPT_FUSE_ATTN_OPROJ:
      MQ_CHECK_ARG(value == 0 || value == 1, "fuse_attn_oproj must be 0 or 1 (got %d)", value);
      e->fuse_attn_oproj = value != 0;
      break;
    case MQ_ENC_OPT_FUSED_LN:
      MQ_CHECK_ARG(value == 0 || value == 1, "fused_ln must be 0 or 1 (got %d)", value);
      e->fused_ln = value != 0;
      break;
    case MQ_ENC_OPT_RESIDENT_LAYERS:
      MQ_CHECK_ARG(value >= 0 && value <= 1024, "resident_layers must be in [0, 1024] (got %d)", value);
      e->resident_layers = value;
      break;
    case MQ_ENC_OPT_LN_ON_LOAD:
      MQ_CHECK_ARG(value == 0 || value == 1, "ln_on_load must be 0 or 1 (got %d)", value);
      e->ln_on_load = value != 0;
      break;
    case MQ_ENC_OPT_SPLITK_TILES:
      MQ_CHECK_ARG(value >= 0 && value <= 4096, "splitk_tiles must be in [0, 4096] (got %d)", value);
      e->splitk_tiles = value;
      break;
    case MQ_ENC_OPT_X6_PRESPLIT:
      MQ_CHECK_ARG(value == 0 || value == 1, "x6_presplit must be 0 or 1 (got %d)", value);
      e->x6_presplit = value != 0;
      break;
    case MQ_ENC_OPT_ROWS_PLANES:
      MQ_CHECK_ARG(value == 0 || value == 1, "rows_planes must be 0 or 1 (got %d)", value);
      e->rows_planes = value != 0;
      break;
    default:
      MQ_FAIL(MQ_EINVAL, "unknown encoder option %d", option);
  }
  // captured forwards bake the old choices in
  for (auto& g : e->graphs) (void)hipGraphExecDestroy(g.exec);
  e->graphs.clear();
  return MQ_OK;
}

int mq_encoder_get_option(const mq_encoder* e, int option, int* value) {
  clear_error();
  MQ_CHECK_ARG(e && value, "NULL argument");
  switch (option) {
    case MQ_ENC_OPT_ROWS_MAX: *value = e->rows_max; break;
    case MQ_ENC_OPT_ROWS_SPLITS: *value = e->rows_splits; break;
    case MQ_ENC_OPT_SPLITK_MAX: *value = e->splitk_max; break;
    case MQ_ENC_OPT_LN_ROWS_PER_WAVE: *value = e->ln_rows_per_wave; break;
    case MQ_ENC_OPT_FUSE_ATTN_OPROJ: *value = e->fuse_attn_oproj ? 1 : 0; break;
    case MQ_ENC_OPT_FUSED_LN: *value = e->fused_ln ? 1 : 0; break;
    case MQ_ENC_OPT_LN_ON_LOAD: *value = e->ln_on_load ? 1 : 0; break;
    case MQ_ENC_OPT_RESIDENT_LAYERS: *value = e->resident_layers; break;
    case MQ_ENC_OPT_SPLITK_TILES: *value = e->splitk_tiles; break;
    case MQ_ENC_OPT_X6_PRESPLIT: *value = e->x6_presplit ? 1 : 0; break;
    case MQ_ENC_OPT_ROWS_PLANES: *value = e->rows_planes ? 1 : 0; break;
    default: MQ_FAIL(MQ_EINVAL, "unknown encoder option %d", option);
  }
  return MQ_OK;
}

int mq_encoder_set_timing(mq_encoder* e, int enabled) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg(e->device);
  e->tl.drain();
  e->tl.on = enabled != 0;
  return MQ_OK;
}

int mq_encoder_read_timing(mq_encoder* e, float* ms, int n) {
  clear_error();
  MQ_CHECK_ARG(e && ms && n >= 0, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg(e->device);
  e->tl.read(ms, n);
  return MQ_OK;
}

int mq_encoder_embed(mq_encoder* e, const int32_t* ids, const int32_t* mask, int B, int L,
                     float* out, int io_on_device, void* stream) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  MQ_CHECK_ARG(B >= 0 && L >= 1, "bad shape B=%d L=%d", B, L);
  MQ_CHECK_ARG(L <= e->cfg.max_positions, "L=%d exceeds max_positions %d", L, e->cfg.max_positions);
  if (B == 0) return MQ_OK;
  MQ_CHECK_ARG(ids && mask && out, "NULL buffer");
  MQ_CHECK_ARG((int64_t)B * L < (1ll << 31) / 4096, "batch too large");
  if (!e->loaded) MQ_FAIL(MQ_ESTATE, "encoder weights not loaded");
  std::lock_guard<std::mutex> lk(e->mu);
  DeviceGuard dg(e->device);
  hipStream_t s = (hipStream_t)stream;
  const mq_bert_config& c = e->cfg;
  const size_t M = (size_t)B * L;
  if (e->tl.used > 4096) e->tl.drain();  // bound the event pool while timing
  int rc = MQ_OK;
  // split-K slabs: up to 2*CUs partial tiles of 32 x 128 floats
  rc = e->slab.ensure((size_t)2 * e->num_cus * 32 * 128);
  if (rc) return rc;
  // y also holds the few-row forward's output-projection planes (<= 4 of M rows)
  const size_t ln_parts = e->ln_on_load && M > 256 ? (size_t)4 * M * std::max(1, c.hidden / kLnPartW) : 0;
  for (auto bn : {std::make_pair(&e->x, M * c.hidden), std::make_pair(&e->y, (M <= (size_t)kRowsMax ? 4 : 1) * M * c.hidden),
                  std::make_pair(&e->ctx, M * c.hidden), std::make_pair(&e->qkv, M * 3 * c.hidden),
                  // (the few-row FFN output is frag16: whole 16-row blocks)
                  std::make_pair(&e->ffn, (M + 15) / 16 * 16 * c.ffn), std::make_pair(&e->lnst, ln_parts)}) {
    rc = bn.first->ensure(bn.second);
    if (rc) return rc;
  }
  const bool graph = e->use_graphs && !e->tl.on;
  const int* dids = ids;
  const int* dmask = mask;
  float* dout = out;
  if (!io_on_device || graph) {  // stage through the encoder's own io buffers
    if (e->io_tokens < M) {
      if (e->io_ids) (void)hipFree(e->io_ids);
      if (e->io_mask) (void)hipFree(e->io_mask);
      e->io_ids = e->io_mask = nullptr;
      e->io_tokens = 0;
      if (hipMalloc((void**)&e->io_ids, M * 4) != hipSuccess ||
          hipMalloc((void**)&e->io_mask, M * 4) != hipSuccess)
        MQ_FAIL(MQ_ENOMEM, "hipMalloc(io) failed");
      e->io_tokens = M;
    }
    rc = e->io_out.ensure((size_t)B * c.hidden);
    if (rc) return rc;
    const hipMemcpyKind kind = io_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (!io_on_device && M * 8 + (size_t)B * c.hidden * 4 <= (1u << 20)) {
      // few tokens (single queries): ids and mask through pinned staging, one DMA each
      rc = e->pin.ensure(M * 8 + (size_t)B * c.hidden * 4);
      if (rc) return rc;
      memcpy(e->pin.as<unsigned char>(), ids, M * 4);
      memcpy(e->pin.as<unsigned char>() + M * 4, mask, M * 4);
      MQ_HIP(hipMemcpyAsync(e->io_ids, e->pin.p, M * 4, kind, s));
      MQ_HIP(hipMemcpyAsync(e->io_mask, e->pin.as<unsigned char>() + M * 4, M * 4, kind, s));
    } else {
      MQ_HIP(hipMemcpyAsync(e->io_ids, ids, M * 4, kind, s));
      MQ_HIP(hipMemcpyAsync(e->io_mask, mask, M * 4, kind, s));
    }
    dids = e->io_ids;
    dmask = e->io_mask;
    dout = e->io_out.p;
  }
  if (graph) {
    rc = launch_graph(e, B, L, s);
  } else {
    rc = forward(e, dids, dmask, B, L, dout, s);
  }
  if (rc) return rc;
  if (io_on_device && dout != out)
    MQ_HIP(hipMemcpyAsync(out, dout, (size_t)B * c.hidden * 4, hipMemcpyDeviceToDevice, s));
  if (!io_on_device) {
    const size_t ob = (size_t)B * c.hidden * 4;
    if (M * 8 + ob <= (1u << 20)) {  // (the pinned staging above)
      unsigned char* hp = e->pin.as<unsigned char>() + M * 8;
      MQ_HIP(hipMemcpyAsync(hp, dout, ob, hipMemcpyDeviceToHost, s));
      MQ_HIP(hipStreamSynchronize(s));
      memcpy(out, hp, ob);
    } else {
      MQ_HIP(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, s));
      MQ_HIP(hipStreamSynchronize(s));
    }
  }
  return MQ_OK;
}

#ifdef MQ_KTRACE
// Measurement builds: copy (and clear) the few-row kernels' phase stamps, [4][1024][8] int64.
int mq_debug_ktrace_read(long long* out, int n) {
  const int total = kTraceRegions * kTraceWgs * kTraceSlots;
  if (!out || n < total) return MQ_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mq_ktrace), total * sizeof(long long)) != hipSuccess) return MQ_EHIP;
  std::vector<long long> zero(total, 0);
  if (hipMemcpyToSymbol(HIP_SYMBOL(mq_ktrace), zero.data(), total * sizeof(long long)) != hipSuccess) return MQ_EHIP;
  return MQ_OK;
}
#endif

}  // extern "C"
