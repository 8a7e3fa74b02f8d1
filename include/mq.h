/*
 * mq.h - C ABI of the MI355X dense-retrieval backend (libmqhip.so).
 *
 * Drop-in boundary for MediQuery-RAG's retrieval pair:
 *   - the encoder replaces OllamaEmbeddings("shaw/dmeta-embedding-zh")
 *       reference src/medical_engine.py:43, src/ingest_medical.py:104
 *       (LangChain Embeddings.embed_query / embed_documents)
 *   - the index replaces the Chroma collection's k-NN
 *       reference src/medical_engine.py:52, src/ingest_medical.py:106-110,
 *       called as vectorstore.similarity_search(query, k=5) at src/agents/nodes.py:93
 * The reference is pure Python; its "FFI" for this path is the LangChain interface.
 * The Python classes in mediquery-rag_amd/mediquery_hip/ bind these entry points with
 * ctypes.
 *
 * Conventions
 *   - Every entry point returns MQ_OK (0) or a negative MQ_E* status; the message of
 *     the last failure on the calling thread is in mq_last_error().
 *   - Pointers flagged "device" are HIP device pointers (e.g. torch data_ptr()); host
 *     pointers are plain malloc/numpy memory.  `stream` is a hipStream_t (NULL = the
 *     default stream).  Host-pointer calls synchronise before returning; device-pointer
 *     calls are asynchronous on `stream`.
 *   - Handles own their device memory; the caller owns every buffer it passes in.
 *   - One handle is used by one thread at a time (each handle has an internal mutex).
 *   - Row identity = insertion order (0..N-1).  Scores are cosine similarities of the
 *     query with the L2-normalised stored row; results are ordered by score desc, then
 *     row id asc.  k > N returns N results and pads the rest with (-inf, -1); an empty
 *     index returns only padding.
 */
#ifndef MQ_H
#define MQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQ_OK 0
#define MQ_EINVAL -1   /* bad argument                       */
#define MQ_ENOMEM -2   /* device or host allocation failed   */
#define MQ_EHIP -3     /* HIP runtime error                  */
#define MQ_EIO -4      /* file I/O error (save/load)         */
#define MQ_ESTATE -5   /* handle in the wrong state          */

#define MQ_DTYPE_F32 0    /* exact fp32 MFMA (v_mfma_f32_32x32x2_f32)                     */
#define MQ_DTYPE_BF16 1   /* bf16 storage (coarse paths)                                    */
#define MQ_DTYPE_F32X6 2  /* fp32 operands split exactly into 3 bf16 pieces, 6 bf16 MFMAs per
                           * product, fp32 accumulate: fp32-class error, 2.67x the MFMA rate;
                           * encoder GEMMs too small to fill the chip (few-row / long single
                           * queries) run exact fp32, which is faster there */
#define MQ_DTYPE_F32_SCREEN 3 /* search only: exact fp32 top-k through certified screens -
                               * bf16 shadow scan for k + 8..16 candidates, fp32 re-rank,
                               * proven error bound; uncertified queries re-run on the
                               * split-f32 screen, then the direct exact scan */

#define MQ_GELU_ERF 0  /* exact erf GELU (HF BERT "gelu")            */
#define MQ_GELU_TANH 1 /* tanh approximation (ggml / llama.cpp gelu)  */
#define MQ_POOL_CLS 0
#define MQ_POOL_MEAN 1

#define MQ_MAX_K 64    /* largest k one search call returns          */

typedef struct mq_index mq_index;
typedef struct mq_encoder mq_encoder;

/* Thread-local message of the most recent failure ("" if none). */
const char* mq_last_error(void);
/* Library build string (arch, version). */
const char* mq_version(void);
/* Build provenance: the first 16 hex digits of the SHA-256 of the csrc/ sources, the
 * Makefile and this header the library was built from (csrc/Makefile STAMPED). */
const char* mq_build_source_hash(void);
/* Number of visible HIP devices (0 without a GPU); never fails. */
int mq_device_count(void);

/* ---------------------------------------------------------------- index ---- */
/* Flat, HBM-resident index of `dim`-wide rows (dim % 32 == 0).  `capacity` rows are
 * reserved up front (it grows on demand by re-allocation).  dtype MQ_DTYPE_F32 is the
 * exact path; MQ_DTYPE_BF16 stores rows in bf16 (coarse path). */
int mq_index_create(int device, int dim, int64_t capacity, int dtype, mq_index** out);
int mq_index_destroy(mq_index* ix);
int mq_index_size(const mq_index* ix, int64_t* n_rows);
int mq_index_dim(const mq_index* ix, int* dim);
/* Append n rows (K8): each row is L2-normalised on the device and stored at the next
 * row ids.  `rows` is [n, dim] f32, host or device. */
int mq_index_add(mq_index* ix, const float* rows, int64_t n, int rows_on_device, void* stream);
/* Drop every row (capacity kept). */
int mq_index_reset(mq_index* ix);
/* Exact top-k (K9 fused score + per-block top-k, K10 merge).
 * queries [nq, dim] f32; out_scores [nq, k] f32; out_ids [nq, k] int64.
 * All three host (io_on_device = 0) or all device (io_on_device = 1). 1 <= k <= MQ_MAX_K.
 * Device calls are asynchronous on `stream` for k <= 16; for k > 16 the call reads a
 * 4-byte overflow flag back (the scan keeps 16 candidates per list and re-scans with
 * 64 when a list may have dropped a top-k member), so it returns after the search. */
int mq_index_search(mq_index* ix, const float* queries, int64_t nq, int k,
                    float* out_scores, int64_t* out_ids, int io_on_device, void* stream);
/* Replace dst's rows with src's rows[0..n) (host int64 row ids in [0, size(src)), any
 * order, repeats allowed), gathered on the device - no host copy of the slab.  dst may be
 * src (in-place compaction after a delete).  Used for Chroma-style `filter` searches
 * and `delete` (reference VectorStore surface).  Synchronous. */
int mq_index_select(mq_index* src, const int64_t* rows, int64_t n, mq_index* dst);
/* Copy stored (normalised) rows [row0, row0 + n) into out [n, dim] f32 (host or device). */
int mq_index_get(mq_index* ix, int64_t row0, int64_t n, float* out, int out_on_device, void* stream);
/* Arithmetic of the fused scan: MQ_DTYPE_F32 (default, exact), MQ_DTYPE_F32X6 (split
 * fp32, large batches; small batches stay on the exact kernel, HBM-bound there), or
 * MQ_DTYPE_BF16: bf16 shadow slab scanned on bf16 MFMA for the top max(k, 50) (capped
 * at MQ_MAX_K) candidates, then an exact fp32 re-rank to the top-k (BASELINE config 5;
 * approximate: recall vs exact is measured, not guaranteed).  dim % 64 == 0.
 * MQ_DTYPE_F32_SCREEN: exact fp32 results via certified screens (above): single queries
 * stream the bf16 shadow (half the HBM bytes), batches scan it on bf16 MFMA; scores are
 * the fp32 re-rank's dot products.  Batches are asynchronous on `stream` (uncertified
 * queries are re-run exactly on the device, mq_index_set_async_screen); single queries
 * and the synchronous batch path read the certificate count back. */
int mq_index_set_precision(mq_index* ix, int dtype);
/* Batches of at most `max_queries` queries (default 4, 0..16; dim % 64 == 0, dim <= 1024)
 * use the streaming fp32 kernel instead of the MFMA tiles, whatever the precision. */
int mq_index_set_stream_threshold(mq_index* ix, int max_queries);
/* Batched bf16 candidate scans (MQ_DTYPE_F32_SCREEN batches, MQ_DTYPE_BF16) of more than
 * 64 queries over >= 65536 rows with dim 256/512/768: 1 (default) = the threshold scan
 * (sample pass -> per-query threshold -> one streaming pass keeping the rows that clear
 * it -> top-kc of the survivors), 0 = the tiled scan with per-lane lists + merge.
 * Same candidates either way up to bf16-score ties at the kc-th place. */
int mq_index_set_threshold_scan(mq_index* ix, int enabled);
/* Single-query MQ_DTYPE_F32_SCREEN searches over >= 65536 rows of dim 256/512/768/1024:
 * 1 (default) = screen on an int8 shadow first (one byte per element + a per-row scale,
 * threshold scan for 64 candidates, fp32 re-rank, certificate with the int8 shadow's
 * measured error bound); uncertified queries re-run on the bf16 stream tier, and after a
 * run of failures (a corpus whose top scores crowd within the int8 bound) the int8 tier
 * sits out the next 256 searches.  0 = start at the bf16 stream tier.  Same results. */
int mq_index_set_int8_screen(mq_index* ix, int enabled);
/* Batched MQ_DTYPE_F32_SCREEN searches: 1 (default) = asynchronous - the certificate
 * failures are never read back; kernels enqueued after the certificate gather the
 * uncertified queries and re-run ALL of them in one exact-f32 MFMA pass over the slab
 * (the direct scan's tile, shape picked on the device from the failure count), merge
 * and write their results in place, returning at once when nothing failed; once a
 * failure has been seen (polled without waiting) the next 16 batches take the
 * synchronous path, and a failure share above 0.2 there sends the next 64 batches
 * straight to the split-f32 screen.
 * The bf16 tier serves k <= 16 only (its 64 candidates leave no margin past that): larger
 * k runs the split-f32 screen (batches > 64) or the direct exact scan.
 * 0 = synchronous: read the failure count, re-run the failures one tier down (split-f32
 * screen, then the direct exact scan).  Same results up to fp32 ties. */
int mq_index_set_async_screen(mq_index* ix, int enabled);
/* Counters of the k > 16 overflow checks so far (either pointer may be NULL): searches
 * re-scanned with 64-entry scan lists, and merges re-run with 64-entry thread lists. */
int mq_index_rescans(const mq_index* ix, int64_t* rescans, int64_t* remerges);
/* Screen counters (MQ_DTYPE_F32_SCREEN; either pointer may be NULL): queries whose
 * certificates failed and that were re-run on the direct exact scan (or on the device
 * by the asynchronous batch path: counting those waits for the last asynchronous
 * search's count copy on its stream), and queries passed down to the next screen
 * (bf16 batch -> split-f32, int8 single -> bf16 stream). */
int mq_index_screen_fallbacks(const mq_index* ix, int64_t* to_direct, int64_t* to_split);
/* Screened searches that bypassed a tier after a run of failed certificates (either
 * pointer may be NULL): batches that skipped the bf16 tier (failure share above 0.2: it
 * sits out 64 searches, then is tried again), and single queries that skipped the int8
 * tier (share above 0.3: it sits out 256). */
int mq_index_screen_skips(const mq_index* ix, int64_t* bf16_skips, int64_t* int8_skips);
/* Device pointer of the row slab ([capacity, dim] of the index dtype). */
int mq_index_data(mq_index* ix, void** device_rows);
/* Device-time accounting with HIP events on the launch stream (off by default).
 * read_timing returns the ms accumulated since the last read: [0] K9 score + top-k,
 * [1] K10 merge; it synchronises on the recorded events and resets the counters. */
int mq_index_set_timing(mq_index* ix, int enabled);
int mq_index_read_timing(mq_index* ix, float* ms, int n);
/* Filtered search (Chroma's `similarity_search(filter=...)`, src/medical_engine.py:52,
 * the LangChain VectorStore surface): a row mask on the device, bit r % 32 of word r / 32
 * set = row r allowed, built from the store's metadata columns by mq_mask_eval /
 * mq_mask_combine (device pointers, async on stream), then one exact search over the
 * allowed rows.  mq_mask_eval: bits (mode)= lut[codes[r]] for rows [0, n), codes[r] = -1
 * (key absent) or >= n_lut - 1 read lut[n_lut - 1]; mq_mask_combine: dst (mode)= src,
 * src NULL = all ones, MQ_MASK_CLEAR zeroes dst. */
#define MQ_MASK_SET 0
#define MQ_MASK_AND 1
#define MQ_MASK_OR 2
#define MQ_MASK_CLEAR 3
int mq_mask_eval(const int32_t* codes, int64_t n, const uint8_t* lut, int n_lut, uint32_t* bits, int mode,
                 void* stream);
/* mq_mask_eval with the table passed by value: lut_words a HOST array of ceil(n_lut / 64)
 * words, bit i % 64 of word i / 64 = lut[i], n_lut <= 256 (a key with few distinct values:
 * no host-to-device copy per condition). */
int mq_mask_eval_bits(const int32_t* codes, int64_t n, const uint64_t* lut_words, int n_lut, uint32_t* bits,
                      int mode, void* stream);
int mq_mask_combine(uint32_t* dst, const uint32_t* src, int64_t n_words, int mode, void* stream);
/* Exact top-k of one query over the allowed rows (same ranking and padding as
 * mq_index_search; bits: a device mask of >= ceil(n / 32) words on the index's GPU).  The
 * int8 certified screen runs with the mask; an uncertified query is answered by the
 * streaming exact scan with the mask (counted by mq_index_masked_gathers).  Synchronous.
 * The mq_mask_* calls launch on the GPU their buffers live on (`stream` must belong to it).
 * Replaces Chroma's `similarity_search(filter=)` / `query(where=)` (src/medical_engine.py:52). */
int mq_index_search_masked(mq_index* ix, const float* query, int k, const uint32_t* bits, float* out_scores,
                           int64_t* out_ids, int io_on_device, void* stream);
/* The same for nq queries at once (queries [nq, dim], outputs [nq, k]; one mask for all) -
 * Chroma's batched `query(query_embeddings=[...], where=)`.  Batches of > 64 queries with
 * k <= 16 run the bf16 threshold scan (K9t) with the mask + fp32 re-rank + certificate;
 * uncertified queries and other batches run the masked streaming exact scan. */
int mq_index_search_masked_batch(mq_index* ix, const float* queries, int64_t nq, int k, const uint32_t* bits,
                                 float* out_scores, int64_t* out_ids, int io_on_device, void* stream);
int mq_index_masked_gathers(const mq_index* ix, int64_t* count);

/* Persistence: a flat binary slab (header + rows); written files are
 * fsync'ed before the call returns. */
int mq_index_save(mq_index* ix, const char* path);
int mq_index_load(mq_index* ix, const char* path);
/* Append-only persistence (the store's segments): save_rows writes rows
 * [row0, row0 + n) as a slab file of n rows; load_append appends a slab file's rows after
 * the index's own, bit-identical (no re-normalisation).  Replace the whole-slab rewrite
 * of Chroma's persist on every add (src/ingest_medical.py:106-110 and
 * src/medical_engine.py:52 share the persist directory). */
int mq_index_save_rows(mq_index* ix, const char* path, int64_t row0, int64_t n);
int mq_index_load_append(mq_index* ix, const char* path);

/* Host-side k-way merge of per-shard candidate lists (the step after the RCCL
 * all-gather).  scores/ids are [n_lists, nq, k_in] (list-major, as an
 * all-gather stacks them); output [nq, k_out] by (score desc, id asc); ids < 0 are
 * padding.  Pure CPU, no device needed. */
int mq_topk_merge_host(const float* scores, const int64_t* ids, int n_lists, int64_t nq,
                       int k_in, int k_out, float* out_scores, int64_t* out_ids);
/* Same merge on the device (inputs/outputs device pointers, async on stream).  Each
 * input list must be sorted (score desc, id asc, padding last), as mq_index_search
 * returns it: the kernel stops reading a list at its first non-qualifying entry. */
int mq_topk_merge_device(const float* scores, const int64_t* ids, int n_lists, int64_t nq,
                         int k_in, int k_out, float* out_scores, int64_t* out_ids, void* stream);

/* -------------------------------------------------------------- encoder ---- */
typedef struct mq_bert_config {
  int vocab_size;     /* 21128 */
  int hidden;         /* 768   */
  int layers;         /* 12    */
  int heads;          /* 12    */
  int ffn;            /* 3072  */
  int max_positions;  /* 1024  */
  int type_vocab;     /* 2     */
  float ln_eps;       /* 1e-12 */
  int gelu;           /* MQ_GELU_* */
  int pooling;        /* MQ_POOL_* */
} mq_bert_config;

int mq_encoder_create(int device, const mq_bert_config* cfg, mq_encoder** out);
int mq_encoder_destroy(mq_encoder* enc);
/* Number of f32 values the weight blob must hold (layout: DESIGN.md / weights.py). */
int64_t mq_encoder_weight_count(const mq_bert_config* cfg);
/* Upload the fp32 weight blob (host pointer, n_floats values). */
int mq_encoder_load_weights(mq_encoder* enc, const float* blob, int64_t n_floats);
/* Arithmetic of the GEMMs: MQ_DTYPE_F32 (exact fp32 MFMA, default) or MQ_DTYPE_F32X6. */
int mq_encoder_set_precision(mq_encoder* enc, int dtype);
/* Device-time accounting per kernel class (HIP events on the launch stream, off by
 * default).  read_timing returns ms since the last read for the stages
 * [0] embed+LN, [1] QKV GEMM, [2] attention, [3] out-proj GEMM, [4] LayerNorm,
 * [5] FFN-up GEMM, [6] FFN-down GEMM, [7] pool+normalise, and resets them. */
#define MQ_ENC_STAGES 8
/* Replay each forward shape as a captured hipGraph (default off; never while timing is
 * on).  Results are bit-identical either way.  On MI355X the host enqueues the ~110
 * launches of a forward faster than the device runs them, so eager launches measured
 * faster for one query (0.628 vs 0.645 ms: the graph path stages ids / mask / out through
 * its own captured buffers); graphs help a host-bound caller. */
int mq_encoder_set_graphs(mq_encoder* enc, int enabled);
/* Tuning options of the forward (explicit, per handle; results stay within the parity
 * tolerances whatever they are set to - each non-default value has a GPU test):
 *   MQ_ENC_OPT_ROWS_MAX          token rows (B x L) up to which the few-row forward runs
 *                                (0..256, default 64; 0 = always the tiled path)
 *   MQ_ENC_OPT_ROWS_SPLITS       few-row FFN-down K splits (0 = automatic, else 1..4 when
 *                                it divides ffn / 256 into an instantiated depth)
 *   MQ_ENC_OPT_SPLITK_MAX        deepest split-K of the tiled path's few-row GEMMs (2..64,
 *                                default 16)
 *   MQ_ENC_OPT_LN_ROWS_PER_WAVE  rows per wave of the batched LayerNorm kernel (1, 2, 4;
 *                                default 4)
 *   MQ_ENC_OPT_FUSE_ATTN_OPROJ   few-row forward: attention + output projection in one
 *                                launch (1, default) or two (0)
 *   MQ_ENC_OPT_FUSED_LN          batched forward, exact f32, hidden <= 768: the residual
 *                                projections (out-proj, FFN-down) on full-row tiles with
 *                                the LayerNorm in their epilogue (1) or GEMM + LayerNorm
 *                                launch (0, default: the full-row tiles measured slower)
 *   MQ_ENC_OPT_SPLITK_TILES      tiled path, M <= 256 rows: a GEMM is split over K only when
 *                                its direct grid has at most this many 32 x 128 tiles
 *                                (0..4096, default 0 = one tile per CU)
 *   MQ_ENC_OPT_LN_ON_LOAD        batched forward, exact f32, M > 256, hidden 768: the
 *                                LayerNorms applied by the consuming GEMM while it stages its
 *                                input, from per-row partials the residual GEMM leaves (1), or
 *                                a LayerNorm launch each (0, default: the staging VALU cost the
 *                                QKV / FFN-up GEMMs 16-18%, more than the 24 launches save)
 *   MQ_ENC_OPT_RESIDENT_LAYERS   few-row forward: layers [0, value) load their weights with
 *                                the default cache policy, later layers non-temporally, so
 *                                back-to-back single queries keep the first layers' weights
 *                                in MALL (0..1024, default 8: BERT-base single query
 *                                0.446 -> 0.427 ms encoder p50; 0 = all non-temporal is the
 *                                slowest, 0.463)
 *   MQ_ENC_OPT_X6_PRESPLIT       split-f32 precision, batched GEMMs: 1 (default) = K2p on the
 *                                weights' W3 plane images (split once, at weight load or
 *                                set_precision), 0 = the split-f32 tiles that split both
 *                                operands while staging them.  Bit-identical results.
 *   MQ_ENC_OPT_ROWS_PLANES       few-row forward: 0 (default) = FFN-down's two K splits and the
 *                                fused attention's two head groups add into ONE output plane
 *                                (two addends per element: bitwise the sum the consumer took), so
 *                                the next QKV / FFN-up reads one plane of rows; 1 = two planes.
 * Setting an option drops the handle's captured graphs. */
#define MQ_ENC_OPT_ROWS_MAX 0
#define MQ_ENC_OPT_ROWS_SPLITS 1
#define MQ_ENC_OPT_SPLITK_MAX 2
#define MQ_ENC_OPT_LN_ROWS_PER_WAVE 3
#define MQ_ENC_OPT_FUSE_ATTN_OPROJ 4
#define MQ_ENC_OPT_FUSED_LN 5
#define MQ_ENC_OPT_SPLITK_TILES 6
#define MQ_ENC_OPT_LN_ON_LOAD 7
#define MQ_ENC_OPT_RESIDENT_LAYERS 8
#define MQ_ENC_OPT_X6_PRESPLIT 9
#define MQ_ENC_OPT_ROWS_PLANES 10
int mq_encoder_set_option(mq_encoder* enc, int option, int value);
int mq_encoder_get_option(const mq_encoder* enc, int option, int* value);
int mq_encoder_set_timing(mq_encoder* enc, int enabled);
int mq_encoder_read_timing(mq_encoder* enc, float* ms, int n);
/* Forward: ids/mask [B, L] int32 -> out [B, hidden] f32, unit-norm (K1..K7).
 * All host (io_on_device = 0) or all device (io_on_device = 1).  L <= max_positions. */
int mq_encoder_embed(mq_encoder* enc, const int32_t* ids, const int32_t* mask, int B, int L,
                     float* out, int io_on_device, void* stream);

/* ------------------------------------------------------------ tokenizer ---- */
/* Host-side BERT tokenisation (the step Ollama runs before the forward, reference
 * src/medical_engine.py:43).  WordPiece over a local vocab.txt, or the deterministic
 * char tokenizer (id = 106 + crc32(char) % (vocab - 106)).  Sequences are
 * [CLS] body [SEP], truncated to max_length, right-padded with 0. */
typedef struct mq_tokenizer mq_tokenizer;
int mq_tokenizer_create_wordpiece(const char* vocab_path, int lower_case, int max_length,
                                  mq_tokenizer** out);
/* The same WordPiece tokenizer over an in-memory vocabulary: tokens[i] is the NUL-terminated
 * UTF-8 token of id i (e.g. the vocab a GGUF model file embeds). */
int mq_tokenizer_create_wordpiece_tokens(const char* const* tokens, int n_tokens, int lower_case,
                                         int max_length, mq_tokenizer** out);
int mq_tokenizer_create_char(int vocab_size, int max_length, mq_tokenizer** out);
int mq_tokenizer_destroy(mq_tokenizer* tok);
/* Encode n NUL-terminated UTF-8 texts.  ids / mask must hold n * max(max_length, pad_to)
 * int32; they are written as [n, L] row-major with L = max(longest sequence, pad_to),
 * returned in *out_len. */
int mq_tokenizer_encode_batch(mq_tokenizer* tok, const char* const* texts, int n, int pad_to,
                              int32_t* ids, int32_t* mask, int* out_len);

/* ------------------------------------------------------- testing hooks ---- */
/* One encoder GEMM on device buffers: out[M,N] = epi(A[M,K] W[N,K]^T + bias (+ resid)),
 * epi 0 bias, 1 bias+GELU(erf), 2 bias+GELU(tanh), 3 bias+residual; tile 0 = 128x128,
 * 1 = 128x96, 2 = 128x64, 3 = 32x128 (exact f32), 4 = split-K (32x128 tiles + ordered
 * slab reduction; synchronous, N % 4 == 0), 5-7 = split-f32 (x6) 128x128 / 128x96 /
 * 128x64, 8 / 9 = exact / split-f32 128x192 on 8-wave workgroups.  K % 32 == 0.  For
 * kernel unit tests. */
int mq_debug_gemm_f32(const float* A, const float* W, const float* bias, const float* resid,
                      float* out, int M, int N, int K, int epi, int tile, void* stream);
/* The W3 plane image of a weight W [N][K] (K % 16 == 0): three bf16 planes of
 * the exact split in 1 KB MFMA fragments.  mq_debug_w3_bytes gives its size (-1 for a bad
 * shape), mq_debug_split_w3 writes it (device buffers, asynchronous on `stream`). */
int64_t mq_debug_w3_bytes(int N, int K);
int mq_debug_split_w3(const float* W, int N, int K, void* w3, void* stream);
/* The encoder GEMM on the pre-split split-f32 kernel (K2p) with W given as its W3 image:
 * tile 0 = 128x192, 1 = 256x96 (4 compute + 4 loader waves), 2 = 128x192, 3 = 256x192
 * (8 compute waves), -1 = the default pick; 4-7 = measurement variants (gemm_x6p.hip);
 * codes >= 100: tile code % 100 with the tile walk cut into one region per XCD,
 * code / 100 - 1 column blocks (0 = the plain round-robin walk; below 100: the pick).
 * Bit-identical to the split-f32 tiles 5-7 / 9 of mq_debug_gemm_f32.  Asynchronous on
 * `stream`.  K % 32 == 0. */
int mq_debug_gemm_x6p(const float* A, const void* W3, const float* bias, const float* resid,
                      float* out, int M, int N, int K, int epi, int tile, void* stream);

/* The int8 screen (K9q) alone for one host query: its kc candidates (screen scores
 * desc, ids; slots past the survivors hold (tau, -1)) and the int8 shadow's statistics
 * stats[0] = max ||c - scale r8||, stats[1] = max ||scale r8||.  For kernel unit tests. */
int mq_debug_int8_screen(mq_index* ix, const float* query, int kc, float* out_scores, int64_t* out_ids,
                         float* stats);

#ifdef __cplusplus
}
#endif
#endif /* MQ_H */
