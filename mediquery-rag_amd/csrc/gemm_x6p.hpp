// gemm_x6p.hpp - host interface of the pre-split split-f32 GEMM (gemm_x6p.hip).
//
// The split-f32 ("x6") arithmetic of gemm_f32.hpp - every fp32 operand split exactly into
// three bf16 planes, six v_mfma_f32_32x32x16_bf16 per product, fp32 accumulation - with
// the weight operand split ONCE, when the weights are loaded, into a fragment-blocked
// plane image ("W3"):
//
//   W3[nb][kb][p][h][r][j]  bf16,  row n = 32 nb + r, k = 16 kb + 8 h + j, plane p = 0..2
//
// i.e. per 32-row x 16-k block and plane one 1 KB MFMA operand fragment in lane order
// (lane = 32 h + r holds 16 B): one LDS-DMA wave-instruction moves it HBM -> LDS whole and
// one conflict-free ds_read_b128 hands it to the MFMA.  Rows past N are zero (N is padded
// to a multiple of 32).  The activation operand stays fp32 in HBM; it is staged fp32 and
// split while its fragments are read.  Products and their order are those of the
// split-f32 tiles of gemm_f32.hpp: results are bit-identical to them.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace mq {

// bytes of the W3 image of an N x K weight (K % 16 == 0)
inline size_t w3_bytes(int64_t N, int64_t K) { return (size_t)((N + 31) / 32) * (size_t)(K / 16) * 3 * 1024; }
// byte offset of row block `row0` (a multiple of 32) inside a W3 image of depth K: the
// image of rows [row0, N) of W is the tail of W's image
inline size_t w3_row_offset(int64_t row0, int64_t K) { return (size_t)(row0 / 32) * (size_t)(K / 16) * 3 * 1024; }

// Region split of a persistent GEMM's tile walk: the tile grid cut into 8 regions, rx
// column blocks x 8 / rx row blocks, one walked by the workgroups sharing blockIdx.x % 8
// (one XCD under round-robin dispatch: speed only), so an XCD's weight column panels stay
// in its L2 across rounds instead of every round re-reading them.  The pick models an XCD's
// operand reads: its A row panels once, its W column panels once if they fit the 4 MB L2,
// else once per round; 0 (the plain round-robin walk) when every workgroup has at most one
// tile.  r6, K2p at M = 8192 (profiles/r6/ab_x6p_regions/): rx 4 for QKV (152.8 -> 134.9
// us, FETCH 210 -> 181 MB) and FFN-up (time unchanged, FETCH 265 -> 205 MB).
inline int region_pick_rx(int64_t tiles_m, int64_t tiles_n, double a_bytes_per_row_tile,
                          double w_bytes_per_col_tile, int64_t grid) {
  if (tiles_m * tiles_n <= grid || grid < 8) return 0;
  const double l2 = 4.0 * 1024 * 1024;
  const int64_t per_xcd = grid / 8;
  int best = 0;
  double best_b = 0;
  for (int rx = 1; rx <= 8; rx *= 2) {
    const int ry = 8 / rx;
    if (rx > tiles_n || ry > tiles_m) continue;
    const int64_t rm = (tiles_m + ry - 1) / ry, rn = (tiles_n + rx - 1) / rx;
    const int64_t rounds = (rm * rn + per_xcd - 1) / per_xcd;
    const double w = (double)rn * w_bytes_per_col_tile;
    const double b = (double)rm * a_bytes_per_row_tile + (w <= l2 ? w : w * (double)rounds);
    if (best == 0 || b < best_b) {
      best = rx;
      best_b = b;
    }
  }
  return best;
}
// the region [m_lo, m_lo + rm) x [n_lo, n_lo + rn) of tiles walked by XCD group xc (rx > 0)
struct Region {
  int m_lo, rm, n_lo, rn;
};
__host__ __device__ inline Region region_of(int rx, int xc, int tiles_m, int tiles_n) {
  const int ry = 8 / rx, ri = xc / rx, rj = xc - ri * rx;
  Region r;
  r.m_lo = ri * tiles_m / ry;
  r.rm = (ri + 1) * tiles_m / ry - r.m_lo;
  r.n_lo = rj * tiles_n / rx;
  r.rn = (rj + 1) * tiles_n / rx - r.n_lo;
  return r;
}

// split W [N][K] fp32 (row stride K) into its W3 image (w3_bytes(N, K) bytes)
void launch_split_w3(const float* W, int N, int K, void* w3, hipStream_t s);

struct X6pArgs {
  const float* A;  // [M][lda] fp32 activations
  int lda;
  const void* W3;  // W3 image of W [N][K]
  const float* bias;
  const float* resid;
  int ldr;
  float* out;
  int ldo;
  int M, N, K;  // K % 16 == 0
  int rx = -1;  // tile-walk region split (gemm_x6p.hip x6p_pick_rx): -1 = the pick, 0 = none, 1/2/4/8
};

// Tile shapes (workgroups of 8 waves, one per CU): 0 = 128 x 192 (4 compute + 4 loader
// waves; the default: M = 8192 at N = 768 / 1536 / 2304 / 3072 gives whole rounds of 256
// tiles), 1 = 256 x 96 (same waves), 2 = 128 x 192 and 3 = 256 x 192 (8 compute waves),
// 7 = 64 x 192 (4 + 4 waves; out-proj-like shapes, see launch_gemm_x6p); 4-6 are
// measurement variants of tile 0.  -1 = the pick below (+ tile 7 for N, K <= 768 when
// 128 x 192 would run a single round).
int x6p_pick_tile(int M, int N, int num_cus);
// epi: EPI_BIAS / EPI_GELU_ERF / EPI_GELU_TANH / EPI_RESID (gemm_epi.hpp)
void launch_gemm_x6p(const X6pArgs& g, int epi, int tile, int num_cus, hipStream_t s);

}  // namespace mq
