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
// All GEMMs run on the exact-fp32 MFMA core of gemm_f32.hpp.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "gemm_f32.hpp"

namespace mq {

enum Epi { EPI_BIAS = 0, EPI_GELU_ERF = 1, EPI_GELU_TANH = 2, EPI_RESID = 3 };

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  return 0.5f * x * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ------------------------------------------------------------------ GEMM -------
// out[M,N] = epi(A[M,K] . W[N,K]^T + bias[N] (+ resid[M,N])), K % 32 == 0.
template <class T, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const float* __restrict__ A,
                                                         const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ resid,
                                                         float* __restrict__ out, int M, int N,
                                                         int K) {
  __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE_FLOATS];
  float* stage0 = lds;
  float* stage1 = lds + T::STAGE_FLOATS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const int tiles_n = (N + T::BN - 1) / T::BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);  // neighbours share the A panel on one XCD
  const int m0 = (wg / tiles_n) * T::BM, n0 = (wg % tiles_n) * T::BN;
  const int nk = K / kBK;

  floatx16 acc[T::TM][T::TN];
  zero_acc<T>(acc);
  Stager<T> st;
  st.load(A, K, M, m0, W, K, N, n0, 0, tid);
  st.store(stage0, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) st.load(A, K, M, m0, W, K, N, n0, (kt + 1) * kBK, tid);
    mma_slice<T>((kt & 1) ? stage1 : stage0, acc, wm, wn, lane);
    if (more) st.store((kt & 1) ? stage0 : stage1, tid);
    __syncthreads();
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
        const int64_t o = (int64_t)row * N + col;
        if (EPI == EPI_GELU_ERF) v = gelu_erf(v);
        if (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
        if (EPI == EPI_RESID) v += resid[o];
        out[o] = v;
      }
  }
}

// ------------------------------------------------------- K1 / LayerNorm ------
// One wave per row of H = 256*VPL floats held in registers (two-pass mean/variance).
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

template <int VPL>
__global__ __launch_bounds__(256) void ln_kernel(const float* __restrict__ src, int M,
                                                 const float* __restrict__ g,
                                                 const float* __restrict__ b, float eps,
                                                 float* __restrict__ dst) {
  constexpr int H = VPL * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  floatx4 x[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
    x[i] = *reinterpret_cast<const floatx4*>(src + (int64_t)row * H + (i * 64 + lane) * 4);
  ln_row_store<VPL>(x, g, b, eps, dst + (int64_t)row * H, lane);
}

// ------------------------------------------------------------ K3 attention ----
// Block = (64-query tile, head, sequence); dh = 64.  K/V tiles of 64 keys staged in
// LDS; each of 4 lanes per query row owns 16 keys for QK^T and 16 output dims for PV.
// Online softmax (running max / sum) in fp32; masked keys contribute exactly 0.
constexpr int kAttQ = 64, kAttK = 64, kDh = 64;

__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ qkv,
                                                        const int* __restrict__ mask, int L,
                                                        int H, float scale,
                                                        float* __restrict__ ctx) {
  __shared__ float qs[kAttQ][kDh + 1];
  __shared__ float ks[kAttK][kDh + 1];
  __shared__ float vs[kAttK][kDh + 4];
  __shared__ float ps[kAttQ][kAttK + 1];
  __shared__ int ms[kAttK];

  const int q0 = blockIdx.x * kAttQ, h = blockIdx.y, bseq = blockIdx.z;
  const int tid = threadIdx.x, qi = tid >> 2, part = tid & 3;
  const int64_t row0 = (int64_t)bseq * L;
  const int ld = 3 * H;

  // Q tile -> LDS (pre-scaled)
  for (int e = tid; e < kAttQ * (kDh / 4); e += 256) {
    const int r = e / (kDh / 4), c4 = e % (kDh / 4);
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (q0 + r < L)
      v = *reinterpret_cast<const floatx4*>(qkv + (row0 + q0 + r) * ld + h * kDh + c4 * 4);
    qs[r][c4 * 4 + 0] = v.x * scale;
    qs[r][c4 * 4 + 1] = v.y * scale;
    qs[r][c4 * 4 + 2] = v.z * scale;
    qs[r][c4 * 4 + 3] = v.w * scale;
  }

  float m_run = -INFINITY, l_run = 0.f;
  float o[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = 0.f;

  for (int k0 = 0; k0 < L; k0 += kAttK) {
    __syncthreads();  // previous tile fully consumed (and Q visible on the first pass)
    for (int e = tid; e < kAttK * (kDh / 4); e += 256) {
      const int r = e / (kDh / 4), c4 = e % (kDh / 4);
      floatx4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (k0 + r < L) {
        const float* base = qkv + (row0 + k0 + r) * ld + h * kDh + c4 * 4;
        kv = *reinterpret_cast<const floatx4*>(base + H);
        vv = *reinterpret_cast<const floatx4*>(base + 2 * H);
      }
      ks[r][c4 * 4 + 0] = kv.x;
      ks[r][c4 * 4 + 1] = kv.y;
      ks[r][c4 * 4 + 2] = kv.z;
      ks[r][c4 * 4 + 3] = kv.w;
      *reinterpret_cast<floatx4*>(&vs[r][c4 * 4]) = vv;
    }
    if (tid < kAttK) ms[tid] = (k0 + tid < L) ? mask[row0 + k0 + tid] : 0;
    __syncthreads();

    // scores for keys part*16 .. part*16+15
    float s[16];
    float tmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int kj = part * 16 + j;
      float acc = 0.f;
#pragma unroll 16
      for (int d = 0; d < kDh; ++d) acc = fmaf(qs[qi][d], ks[kj][d], acc);
      s[j] = ms[kj] ? acc : -INFINITY;
      tmax = fmaxf(tmax, s[j]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 1));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 2));
    const float m_new = fmaxf(m_run, tmax);
    // fully masked so far: keep everything at zero
    const float alpha = (m_new == -INFINITY) ? 1.f : expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float p = (s[j] == -INFINITY) ? 0.f : expf(s[j] - m_new);
      psum += p;
      ps[qi][part * 16 + j] = p;
    }
    psum += __shfl_xor(psum, 1);
    psum += __shfl_xor(psum, 2);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] *= alpha;
    for (int j = 0; j < kAttK; ++j) {
      const float p = ps[qi][j];
      const float* vr = &vs[j][part * 16];
#pragma unroll
      for (int d = 0; d < 16; ++d) o[d] = fmaf(p, vr[d], o[d]);
    }
  }
  if (q0 + qi < L) {
    const float inv = l_run > 0.f ? 1.0f / l_run : 0.f;
    float* dst = ctx + (row0 + q0 + qi) * H + h * kDh + part * 16;
#pragma unroll
    for (int d = 0; d < 16; d += 4) {
      floatx4 v = {o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv};
      *reinterpret_cast<floatx4*>(dst + d) = v;
    }
  }
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
};

int64_t weight_count(const mq_bert_config& c) {
  const int64_t H = c.hidden, F = c.ffn;
  const int64_t per_layer = 3 * H * H + 3 * H + H * H + H + 2 * H + F * H + F + H * F + H + 2 * H;
  return ((int64_t)c.vocab_size + c.max_positions + c.type_vocab) * H + 2 * H + c.layers * per_layer;
}

}  // namespace

struct mq_encoder {
  int device = 0;
  mq_bert_config cfg{};
  int precision = MQ_DTYPE_F32;
  bool loaded = false;
  Buf weights;
  const float *word = nullptr, *pos = nullptr, *typ = nullptr, *eg = nullptr, *eb = nullptr;
  std::vector<LayerW> layers;
  Buf x, y, qkv, ctx, ffn, io_out;
  int* io_ids = nullptr;
  int* io_mask = nullptr;
  size_t io_tokens = 0;
  std::mutex mu;
};

namespace {

template <class T, int EPI>
void launch_gemm_t(const float* A, const float* W, const float* bias, const float* resid, float* out,
                   int M, int N, int K, hipStream_t s) {
  const int tiles = ((M + T::BM - 1) / T::BM) * ((N + T::BN - 1) / T::BN);
  hipLaunchKernelGGL((gemm_nt_kernel<T, EPI>), dim3(tiles), dim3(256), 0, s, A, W, bias, resid,
                     out, M, N, K);
}

using GemmBig = F32Tile<2, 2, 2, 2>;    // 128 x 128
using GemmMid = F32Tile<2, 2, 2, 1>;    // 128 x 64  (N = hidden: 3x the blocks)
using GemmSmall = F32Tile<1, 4, 1, 1>;  // 32 x 128  (few tokens)

template <int EPI>
void launch_gemm(const float* A, const float* W, const float* bias, const float* resid, float* out,
                 int M, int N, int K, int num_cus, hipStream_t s) {
  const int64_t big_tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (M <= 64)
    launch_gemm_t<GemmSmall, EPI>(A, W, bias, resid, out, M, N, K, s);
  else if (big_tiles < 2 * num_cus)
    launch_gemm_t<GemmMid, EPI>(A, W, bias, resid, out, M, N, K, s);
  else
    launch_gemm_t<GemmBig, EPI>(A, W, bias, resid, out, M, N, K, s);
}

template <int VPL>
int forward_vpl(mq_encoder* e, const int* ids, const int* mask, int B, int L, float* out,
                hipStream_t s) {
  const mq_bert_config& c = e->cfg;
  const int M = B * L, H = c.hidden, F = c.ffn;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device);
  const unsigned row_blocks = (unsigned)((M + 3) / 4);
  hipLaunchKernelGGL((embed_ln_kernel<VPL>), dim3(row_blocks), dim3(256), 0, s, ids, M, L,
                     c.vocab_size, e->word, e->pos, e->typ, e->eg, e->eb, c.ln_eps, e->x.p);
  const float scale = 1.0f / sqrtf((float)(H / c.heads));
  for (const LayerW& w : e->layers) {
    launch_gemm<EPI_BIAS>(e->x.p, w.wqkv, w.bqkv, nullptr, e->qkv.p, M, 3 * H, H, cus, s);
    hipLaunchKernelGGL(attention_kernel, dim3((L + kAttQ - 1) / kAttQ, c.heads, B), dim3(256), 0,
                       s, e->qkv.p, mask, L, H, scale, e->ctx.p);
    launch_gemm<EPI_RESID>(e->ctx.p, w.wo, w.bo, e->x.p, e->y.p, M, H, H, cus, s);
    hipLaunchKernelGGL((ln_kernel<VPL>), dim3(row_blocks), dim3(256), 0, s, e->y.p, M, w.ln1g,
                       w.ln1b, c.ln_eps, e->x.p);
    if (c.gelu == MQ_GELU_TANH)
      launch_gemm<EPI_GELU_TANH>(e->x.p, w.w1, w.b1, nullptr, e->ffn.p, M, F, H, cus, s);
    else
      launch_gemm<EPI_GELU_ERF>(e->x.p, w.w1, w.b1, nullptr, e->ffn.p, M, F, H, cus, s);
    launch_gemm<EPI_RESID>(e->ffn.p, w.w2, w.b2, e->x.p, e->y.p, M, H, F, cus, s);
    hipLaunchKernelGGL((ln_kernel<VPL>), dim3(row_blocks), dim3(256), 0, s, e->y.p, M, w.ln2g,
                       w.ln2b, c.ln_eps, e->x.p);
  }
  hipLaunchKernelGGL((pool_kernel<VPL>), dim3((B + 3) / 4), dim3(256), 0, s, e->x.p, mask, B, L,
                     c.pooling, out);
  MQ_HIP(hipGetLastError());
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
  *out = e.release();
  return MQ_OK;
}

int mq_encoder_destroy(mq_encoder* e) {
  clear_error();
  if (!e) return MQ_OK;
  {
    DeviceGuard dg(e->device);
    for (Buf* b : {&e->weights, &e->x, &e->y, &e->qkv, &e->ctx, &e->ffn, &e->io_out}) b->release();
    if (e->io_ids) (void)hipFree(e->io_ids);
    if (e->io_mask) (void)hipFree(e->io_mask);
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
  return MQ_OK;
}

int mq_encoder_set_precision(mq_encoder* e, int dtype) {
  clear_error();
  MQ_CHECK_ARG(e, "NULL encoder");
  MQ_CHECK_ARG(dtype == MQ_DTYPE_F32, "only the f32 encoder path is implemented (got %d)", dtype);
  e->precision = dtype;
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
  int rc = MQ_OK;
  for (auto bn : {std::make_pair(&e->x, M * c.hidden), std::make_pair(&e->y, M * c.hidden),
                  std::make_pair(&e->ctx, M * c.hidden), std::make_pair(&e->qkv, M * 3 * c.hidden),
                  std::make_pair(&e->ffn, M * c.ffn)}) {
    rc = bn.first->ensure(bn.second);
    if (rc) return rc;
  }
  const int* dids = ids;
  const int* dmask = mask;
  float* dout = out;
  if (!io_on_device) {
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
    MQ_HIP(hipMemcpyAsync(e->io_ids, ids, M * 4, hipMemcpyHostToDevice, s));
    MQ_HIP(hipMemcpyAsync(e->io_mask, mask, M * 4, hipMemcpyHostToDevice, s));
    dids = e->io_ids;
    dmask = e->io_mask;
    dout = e->io_out.p;
  }
  switch (c.hidden) {
    case 256: rc = forward_vpl<1>(e, dids, dmask, B, L, dout, s); break;
    case 512: rc = forward_vpl<2>(e, dids, dmask, B, L, dout, s); break;
    case 768: rc = forward_vpl<3>(e, dids, dmask, B, L, dout, s); break;
    default: rc = forward_vpl<4>(e, dids, dmask, B, L, dout, s); break;
  }
  if (rc) return rc;
  if (!io_on_device) {
    MQ_HIP(hipMemcpyAsync(out, dout, (size_t)B * c.hidden * 4, hipMemcpyDeviceToHost, s));
    MQ_HIP(hipStreamSynchronize(s));
  }
  return MQ_OK;
}

}  // extern "C"
