// thresh.hpp - K9t, the bf16 threshold scan behind batched bf16 candidate searches
// (MQ_DTYPE_F32_SCREEN batches, MQ_DTYPE_BF16); kernels in thresh.hip.
#pragma once

#include "common.hpp"

namespace mq {

constexpr int kTsRows = 32;          // rows per streamed block (the MFMA tile edge)
constexpr int kTsCap = 4096;         // survivors kept per query
constexpr int64_t kTsMinRows = 65536;  // below this the tiled K9 + K10 path is used
constexpr int kTsRank = 8;  // screens: tau = 8th largest sample list maximum (~128 survivors)

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
  int tau_rank;               // tau = the tau_rank-th largest sample list maximum (>= tau_rank survivors)
  int* fail_count;            // optional: queries with more than kTsCap or fewer than kc survivors
  int64_t* fail;              //   are appended to fail[] (count in *fail_count, zeroed by the caller)
  // optional row mask (batched filtered search): bit r % 32 of word r / 32 set = row r
  // exists; masked rows are skipped by both passes (>= ceil(n / 32) words)
  const unsigned* mask = nullptr;
};

// Enqueue the four K9t launches on `s`; timeline stage 0 = the two scans, 1 = tau + select.
void launch_thresh(const ThreshArgs& a, hipStream_t s, Timeline* tl);

// K9q: the int8 threshold scan for one query (single-query certified screen).
#ifndef MQ_I8_WG
#define MQ_I8_WG 3
#endif
constexpr int kI8WgPerCu = MQ_I8_WG;   // 256-thread workgroups per CU (= residency at <= 168 VGPRs: the
                                // scan loops are persistent, a non-resident 4th would run late)
constexpr int kI8MaxLists = 1024;  // workgroups per launch = sample lists (tau is found in-kernel)
constexpr int kI8PadRows = 16;  // the shadow is allocated to whole 8- or 16-row units
// Survivors of the appending pass: per query, one segment of kI8Seg slots per workgroup
// (list), filled through an LDS counter with plain stores; the workgroup stores its count
// at the end.  A single global counter made every append a returning atomic to memory
// behind the streaming loads (~13 us for 320 survivors: the appending wave stalls).
constexpr int kI8Seg = 16;
struct ThreshI8Args {
  const float* q;             // fp32 queries [nq][dim]
  int nq;                     // 1
  const unsigned* r8;         // int8 shadow [n][dim] (4 elements per dword)
  const float* scale;         // [n] per-row scales
  int64_t n;
  int dim;                    // 256, 512, 768 or 1024
  int num_cus;
  float* lmax;                // [nq][i8_lists(num_cus)] sample-pass workgroup maxima
  float* tau;                 // [nq]
  int* count;                 // [nq][lists] survivors per segment (may exceed kI8Seg: overflow)
  float* cs;                  // [nq][lists][kI8Seg] survivor scores
  int* ci;                    // [nq][lists][kI8Seg] survivor rows
  int* zero;                  // optional int the sample pass sets to 0 (the caller's fail count)
  // the certificate's tau (index.hip i8_finish_kernel): with the shadow's maxima `stats`
  // and the query's k, tau = min(the kTsRank-th largest sample list maximum, max(the k-th
  // largest - 2E, the 32nd largest)), E the screen's bound - tau + E < e_k then holds by
  // construction unless the floor applies
  const unsigned* stats = nullptr;
  int k = 0;                  // 0: tau = the kTsRank-th largest maximum only
  // optional row mask (filtered search): bit r % 32 of word r / 32 set = row r exists;
  // masked rows are skipped by both passes (>= ceil(n / 32) words)
  const unsigned* mask = nullptr;
};
int i8_lists(int num_cus);
// K9q segments -> a compact list per query (out_count = the survivors, kTsCap + 1 if a
// segment overflowed; entries past kTsCap dropped), for launch_select
void launch_i8_compact(const float* cs, const int* ci, const int* count, int lists, int nq, float* out_cs,
                       int* out_ci, int* out_count, hipStream_t s);
// The sample and appending passes: survivors in cs / ci / count, tau in tau.
void launch_thresh_i8(const ThreshI8Args& a, hipStream_t s, Timeline* tl);
// Survivors -> top-kc candidates per query (K9t's select; slots past the count: (tau, -1)).
void launch_select(const float* cs, const int* ci, const int* count, const float* tau, int nq, int kc,
                   float* out_s, int64_t* out_i, hipStream_t s);
// int8 shadow of rows [0, n): r8 [n][dim] int8, scale [n], err [n] = ||c - scale r8|| per
// row, stats [0] max ||c - scale r8||, [1] max ||scale r8|| (float bits; atomicMax - zero
// them before the first rows).
void launch_i8_shadow(const float* rows, int64_t n, int dim, unsigned* r8, float* scale, float* err,
                      unsigned* stats, hipStream_t s);

}  // namespace mq
