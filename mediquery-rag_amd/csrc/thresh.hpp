// thresh.hpp - K9t, the bf16 threshold scan behind batched bf16 candidate searches
// (MQ_DTYPE_F32_SCREEN batches, MQ_DTYPE_BF16); kernels in thresh.hip.
#pragma once

#include "common.hpp"

namespace mq {

constexpr int kTsRows = 32;          // rows per streamed block (the MFMA tile edge)
constexpr int kTsCap = 4096;         // survivors kept per query
constexpr int64_t kTsMinRows = 65536;  // below this the tiled K9 + K10 path is used

struct ThreshArgs {
  const float* q16;           // bf16 queries [nq][dim] (as packed pairs)
  int nq;
  const unsigned char* rows;  // bf16 shadow [n][dim], allocated to a whole number of blocks
  int64_t n;
  int dim;                    // 256, 512 or 768
  int num_cus;
  int kc;                     // candidates per query (<= MQ_MAX_K)
  float* lmax;                // [nq][2 * num_cus] sample-pass list maxima
  float* tau;                 // [nq]
  int* count;                 // [nq]
  float* cs;                  // [nq][kTsCap] survivor scores
  int* ci;                    // [nq][kTsCap] survivor rows
  float* out_s;               // [nq][kc] candidates, (score desc, id asc)
  int64_t* out_i;
};

// Enqueue the four K9t launches on `s`; timeline stage 0 = the two scans, 1 = tau + select.
void launch_thresh(const ThreshArgs& a, hipStream_t s, Timeline* tl);

}  // namespace mq
