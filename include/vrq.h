/*
 * vrq.h -- C ABI of libvrq.so, the MI355X (gfx950) hot path of
 * aitrailblazer/VectorRAGQuantization re-built as hand-written HIP kernels.
 *
 * The reference reaches its compute through two un-vendored native
 * dependencies (FAISS C++ for Phase I, NumPy for Phases II/III and the
 * encoders).  Each entry point below replaces one of those call sites; the
 * reference location is cited per function (paths relative to the reference
 * checkout).  The Python host layer (vectorragquantization_amd) binds these
 * symbols with ctypes; the cgo / JNI / ctypes stubs a maintainer would add on
 * the reference side are in INTEGRATION.md.
 *
 * Conventions (all functions):
 *   - every pointer is a DEVICE pointer owned by the caller (allocated e.g. by
 *     torch); the library never allocates, frees or synchronises;
 *   - all work is enqueued on `stream` (a hipStream_t passed as void*, NULL =
 *     the null stream) and is stream-ordered; no host threads, no global
 *     mutable state, so concurrent calls on different streams are safe;
 *   - return VRQ_OK (0) or a negative VRQ_E* code; never abort, never throw;
 *     vrq_strerror() maps a code to text.
 *   - row indices are int64; "rows" are internal (insertion-order) indices of
 *     the caller's shard, reported as row_offset + local row (global row).
 */
#ifndef VRQ_H_
#define VRQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VRQ_ABI_VERSION 1

#define VRQ_OK 0
#define VRQ_EINVAL (-1)       /* bad argument (null pointer, negative size, ...) */
#define VRQ_EHIP (-2)         /* a HIP runtime call or kernel launch failed */
#define VRQ_EUNSUPPORTED (-3) /* shape outside what the kernels implement */
#define VRQ_EWORKSPACE (-4)   /* workspace smaller than *_workspace_size() */

/* flags for vrq_search3 */
#define VRQ_SEARCH_PHASE1_ONLY 1 /* stop after Phase I (FAISS IndexBinaryFlat::search) */
#define VRQ_SEARCH_SHARD 2       /* sharded mode: return all K Phase-I candidates in
                                    (dist,row) order with Phase-II AND Phase-III
                                    scores, no Phase II/III sort (merged later by
                                    vrq_merge_shards) */
#define VRQ_SEARCH_SCAN_VALU 4   /* Phase-I scan: force the wavefront popcount scan */
#define VRQ_SEARCH_SCAN_MFMA 8   /* Phase-I scan: force the matrix-core scan wherever it is
                                    supported (K <= 128, n >= 65536); by default it is used for
                                    nq >= 128.  Both scans give identical results. */
/* vrq_search3_scan only, matrix-core scan only: run a subset of its four stages (none set =
 * all), so a caller can bracket each stage with events; issuing PREFIX, MATRIX, RECHECK,
 * SUFFIX in that order on one stream is exactly the full scan. */
#define VRQ_SCAN_STAGE_PREFIX 16 /* dense matrix-core pass over a spread row sample -> per-query
                                    thresholds (sampled d_(j), guaranteed d_(K)) */
#define VRQ_SCAN_STAGE_MATRIX 32 /* thresholded matrix-core pass over all rows */
#define VRQ_SCAN_STAGE_RECHECK 128 /* per-query proof that the sampled threshold admitted >= K rows
                                      and exact re-run of the rare failed query blocks */
#define VRQ_SCAN_STAGE_SUFFIX 64 /* candidates -> one sorted K-list per query (exact rescan on
                                    list overflow) */

/* encoder modes for vrq_encode.  Inputs must be finite: the reference's NumPy encoders give NaN
 * min/max, NaN means and platform-defined integer casts for a NaN element, so no NaN behaviour is
 * pinned; the d = 1024 kernels fold min/max with v_med3 (a NaN element yields min = -inf, i.e. an
 * all-zero local code) and the generic kernel with fminf/fmaxf (NaN elements ignored). */
#define VRQ_ENC_INT8_GLOBAL 0  /* VectorDBInt8Global._quantize_to_int8 + _to_binary */
#define VRQ_ENC_INT16_GLOBAL 1 /* VectorDBInt16Global._quantize_to_int16 + _to_binary */
#define VRQ_ENC_INT4_GLOBAL 2  /* VectorDBInt4Global._quantize_to_int4 (limit ignored) + _to_binary */
#define VRQ_ENC_INT8_LOCAL 3   /* VectorDBInt8._quantize_to_int8 (+min/max) + _to_binary */
#define VRQ_ENC_INT4_LOCAL 4   /* VectorDBInt4._quantize_to_int4 (+min/max) + _to_binary */
#define VRQ_ENC_BIN_INT16 5    /* VectorDBInt16._to_binary on int16 input */
#define VRQ_ENC_COHERE 6       /* synthetic Cohere provider: int8 (global limit) + ubinary = packbits(x > 0) */
/* vrq_rescore_dequant only: the compare_float32 branch of the VectorDB* searches
 * (VectorDBInt8Global.py:239-240, VectorDBInt8.py:231-232, VectorDBInt4.py:262-263,
 * VectorDBInt16Global.py:240-241, VectorDBInt4Global.py:257-258): q = f32[n, dim] float rows */
#define VRQ_RESCORE_F32 16

int vrq_abi_version(void);
const char* vrq_strerror(int code);

/* ---------------------------------------------------------------------------
 * Phase I -- exhaustive Hamming k-NN over packed codes.
 * Replaces faiss.IndexBinaryFlat::search (hammings_knn_hc) reached from
 *   CohereEnhancedVectorDB.py:267-268 (and VectorDBInt8Global.py:224-225,
 *   VectorDBInt16.py, VectorDBInt4*.py, VectorDBInt16Global.py search()).
 * codes      u8[n, code_bytes]    (code_bytes = d/8; 128 for d = 1024)
 * queries    u8[nq, code_bytes]
 * out_dist   i32[nq, k]  ascending (dist, row) -- FAISS order; missing = INT32_MAX
 * out_rows   i64[nq, k]  row_offset + row; missing = -1
 * Supported: code_bytes in {64, 128, 256}, 1 <= k <= 1024, n < 2^40.
 * ------------------------------------------------------------------------- */
size_t vrq_hamming_topk_workspace_size(int64_t n, int32_t code_bytes, int32_t nq, int32_t k);
int vrq_hamming_topk(const uint8_t* codes, int64_t n, int32_t code_bytes, int64_t row_offset,
                     const uint8_t* queries, int32_t nq, int32_t k, int32_t* out_dist,
                     int64_t* out_rows, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Fused three-phase search -- replaces CohereEnhancedVectorDB.search
 *   (CohereEnhancedVectorDB.py:247-322) for a batch of nq queries:
 *   Phase I   top-K by Hamming (K = binary_k = min(k*binary_oversample, ntotal), :267-275)
 *   Phase II  s2 = q . (2*unpackbits(code)-1) in float64 (:283-293); stable sort desc (:296)
 *   Phase III s3 = float(q . int8 [f32]) / ||int8||_2 [f64], -inf if 0 (:302-318);
 *             over the first K3 = k*int8_oversample (:297); stable sort desc; first k (:321-322)
 * x8     int8[n, dim]   (the RocksDict "int8" value, :221)
 * norms  f64[n]         ||x8 row||_2 (vrq_int8_row_norms), as np.linalg.norm (:308)
 * rescore_row  i64[n] or NULL: row whose code/int8 Phases II/III use for Phase-I row r.
 *        IndexBinaryIDMap2::reconstruct(id) returns the row of the LAST add of an id
 *        (rev_map, :286) and the doc store keeps the last value (:221,303); when an id
 *        occurs on several rows pass rev_map[id_map[r]], else NULL (identity).
 * qf     f32[nq, dim], qb u8[nq, dim/8]
 * outputs [nq, kout] where kout = k (or K with VRQ_SEARCH_SHARD):
 *   out_count i32[nq]; out_rows i64; out_dist i32; out_binary f64; out_cosine f64
 * dim must be 1024 (code_bytes 128) in this ABI version.
 * ------------------------------------------------------------------------- */
size_t vrq_search3_workspace_size(int64_t n, int32_t dim, int32_t nq, int32_t K);
int vrq_search3(const uint8_t* codes, const int8_t* x8, const double* norms, const int64_t* rescore_row,
                int64_t n, int32_t dim, int64_t row_offset, const float* qf, const uint8_t* qb, int32_t nq, int32_t k,
                int32_t K, int32_t K3, int32_t flags, int32_t* out_count, int64_t* out_rows,
                int32_t* out_dist, double* out_binary, double* out_cosine, void* workspace,
                size_t workspace_bytes, void* stream);

/* The two launches vrq_search3 is made of, for callers that time or overlap them:
 * vrq_search3_scan   -- K1, the Phase-I scan: per-chunk exact top-K lists into `workspace`
 * vrq_search3_finish -- K2, exact merge of those lists + Phases II/III + the sorts
 * (same arguments as vrq_search3, the same flags to both; the workspace carries the lists
 * between them). */
int vrq_search3_scan(const uint8_t* codes, int64_t n, int32_t dim, const uint8_t* qb, int32_t nq,
                     int32_t K, int32_t flags, void* workspace, size_t workspace_bytes, void* stream);
int vrq_search3_finish(const uint8_t* codes, const int8_t* x8, const double* norms,
                       const int64_t* rescore_row, int64_t n, int32_t dim, int64_t row_offset,
                       const float* qf, int32_t nq, int32_t k, int32_t K, int32_t K3, int32_t flags,
                       int32_t* out_count, int64_t* out_rows, int32_t* out_dist, double* out_binary,
                       double* out_cosine, const void* workspace, size_t workspace_bytes, void* stream);

/* Which Phase-I scan vrq_search3 / vrq_search3_scan / vrq_hamming_topk would run for this
 * shape and flags: VRQ_SCAN_KIND_VALU (wavefront popcount) or VRQ_SCAN_KIND_MFMA (matrix
 * core; *prefix_rows, if non-NULL, receives the rows scanned outside the thresholded
 * matrix-core pass: 0, or n for the wavefront scan), or a
 * negative VRQ_E* code for an unsupported shape.  Host-only, no device work. */
#define VRQ_SCAN_KIND_VALU 0
#define VRQ_SCAN_KIND_MFMA 1
int vrq_scan_kind(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* prefix_rows);
/* Host-only planning introspection of the matrix-core scan (no reference counterpart; tests and
 * tools): info i64[12] = row-split kernel K1r (1), shared-tile kernel K1m (0) or row-set kernel K1s (2,
 * large batches of short passes), M-blocks (32 queries) per wave (K1s: 4, its 512-query blocks), chunk rows, chunks, per-(query, chunk) list capacity, workspace offsets of
 * the candidate lists (u64 keys (v + 1025) << 40 | row, v = dist - tau), of the list lengths (i32
 * [nq][chunks]) and of tau_s / tau_p / rerun (i32 [nq] each, 256-B aligned), sample rows, sampled
 * order j, offset of the sorted K-lists, workspace bytes.  VRQ_EUNSUPPORTED when the shape takes the
 * wavefront scan. */
int vrq_scan_plan(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* info);
/* Host-only introspection of the matrix-core scan's dense sample pass (tests and tools): info i64[6]
 * = the row-split kernel runs it (1) or K1m's MB = 2 instance (0), sample chunks, rows per sample
 * chunk, rows between consecutive sample chunks, rows between consecutive 64-row sample tiles, and
 * the u16 lane-minimum columns per query at workspace offset 0 (32 per sample chunk: column
 * chunk * 32 + r = min over the chunk's tiles and both 32-row halves of tile row r of
 * dist - popcount(query), + 1024).  VRQ_EUNSUPPORTED when the shape takes the wavefront scan. */
int vrq_scan_sample_plan(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* info);

/* ---------------------------------------------------------------------------
 * Merge of per-shard candidate tuples after the RCCL all-gather (multi-GPU
 * row sharding; the reference is single-process, so this reproduces the
 * single-index semantics of CohereEnhancedVectorDB.py:267-322 exactly):
 *   global top-K by (dist, global row) -> stable sort by s2 desc -> first K3
 *   -> stable sort by s3 desc -> first k.
 * Inputs are the VRQ_SEARCH_SHARD outputs of S shards stacked [S, nq, K]
 * (counts i32[S, nq]); shard s must own a contiguous global row range below
 * shard s+1's.  out_src (nullable) i32[nq, k] receives s*K + p, the position of
 * each result in the stacked inputs (to fetch per-candidate payloads such as
 * external ids).
 * ------------------------------------------------------------------------- */
int vrq_merge_shards(int32_t nshards, int32_t nq, int32_t K, const int32_t* counts,
                     const int64_t* rows, const int32_t* dist, const double* s2,
                     const double* s3, int32_t k, int32_t K3, int32_t* out_count,
                     int64_t* out_rows, int32_t* out_dist, double* out_binary,
                     double* out_cosine, int32_t* out_src, void* stream);

/* ---------------------------------------------------------------------------
 * Stand-alone Phase II / Phase III candidate rescoring (the per-candidate
 * loops of CohereEnhancedVectorDB.py:283-293 and :302-318).
 * cand_rows i64[nq, ncand] local rows (negative = skip, output NaN).
 * ------------------------------------------------------------------------- */
int vrq_rescore_binary(const float* qf, int32_t nq, int32_t dim, const uint8_t* codes, int64_t n,
                       const int64_t* cand_rows, int32_t ncand, double* out, void* stream);
int vrq_rescore_int8_cosine(const float* qf, int32_t nq, int32_t dim, const int8_t* x8,
                            const double* norms, int64_t n, const int64_t* cand_rows,
                            int32_t ncand, double* out, void* stream);

/* ---------------------------------------------------------------------------
 * Encoders -- the VectorDBInt{4,8,16}{,Global} quantize + _to_binary path:
 *   VectorDBInt8Global.py:130-142,154-160   VectorDBInt16Global.py:130-142,154-160
 *   VectorDBInt4Global.py:129-164,190-196   VectorDBInt8.py:114-126,140-146
 *   VectorDBInt4.py:116-154,186-192          VectorDBInt16.py:148-157
 * x       f32[n, dim] (i16[n, dim] for VRQ_ENC_BIN_INT16)
 * codes   u8[n, dim/8]           packbits(x > mean(x)) MSB-first (or x > 0 for COHERE)
 * q       i8[n, dim] | i16[n, dim] | i8[n, (dim+1)/2] (int4 nibbles) | unused
 * minmax  f64[n, 2] (local modes only; may be NULL otherwise)
 * limit   global clip limit (Global modes / COHERE), as passed by the caller
 * dim must be a multiple of 8 and <= 8192.
 * ------------------------------------------------------------------------- */
int vrq_encode(int32_t mode, const void* x, int64_t n, int32_t dim, double limit, uint8_t* codes,
               void* q, double* minmax, void* stream);

/* ---------------------------------------------------------------------------
 * Search side of the VectorDB* classes: dequantisation and the
 * dequantised-dot rescoring of Phase-I candidates.  mode is the VRQ_ENC_* mode that produced the
 * codes (INT8_GLOBAL, INT16_GLOBAL, INT4_GLOBAL, INT8_LOCAL, INT4_LOCAL):
 *   VectorDBInt8Global._dequantize_int8   VectorDBInt8Global.py:144-152
 *   VectorDBInt16Global._dequantize_int16 VectorDBInt16Global.py:144-152
 *   VectorDBInt4Global._dequantize_int4   VectorDBInt4Global.py:166-188
 *   VectorDBInt8._dequantize_int8         VectorDBInt8.py:129-138
 *   VectorDBInt4._dequantize_int4         VectorDBInt4.py:157-184
 * bit-identical to the reference (NumPy 2 scalar rules).  q is the code array (int8 / int16 /
 * packed int4 bytes), minmax f64[n, 2] for the local modes (NULL otherwise), limit for the global
 * ones.  vrq_dequantize writes f32[n, dim]; vrq_rescore_dequant writes, per (query, candidate), the
 * reference score float(np.dot(query_float, dequantised row)) (VectorDBInt8Global.py:232-238 and the
 * same loop in the other classes) as the correctly rounded float32 dot (NaN for negative rows).
 * vrq_rescore_dequant also takes mode VRQ_RESCORE_F32 (q = the f32 float rows, compare_float32).
 * ------------------------------------------------------------------------- */
int vrq_dequantize(int32_t mode, const void* q, const double* minmax, int64_t n, int32_t dim, double limit,
                   float* out, void* stream);
int vrq_rescore_dequant(int32_t mode, const float* qf, int32_t nq, int32_t dim, const void* q,
                        const double* minmax, double limit, int64_t n, const int64_t* cand_rows,
                        int32_t ncand, double* out, void* stream);
/* np.linalg.norm(int8 row) in float64 (CohereEnhancedVectorDB.py:308), computed once at add time */
int vrq_int8_row_norms(const int8_t* x8, int64_t n, int32_t dim, double* out, void* stream);
/* ---------------------------------------------------------------------------
 * Exhaustive batched Phase-II / Phase-III scoring on the matrix cores (BASELINE config 5):
 * the per-candidate scores of CohereEnhancedVectorDB.py:283-293 (VRQ_GEMM_BINARY) or :302-318
 * (VRQ_GEMM_INT8_COSINE) evaluated against EVERY row, top-k fused (no nq x n score matrix):
 *   VRQ_GEMM_BINARY       s = float(q . (2*unpackbits(code)-1)) in float64      (codes)
 *   VRQ_GEMM_INT8_COSINE  s = float32(q . int8) / ||int8||_2, -inf if the norm is 0 (x8, norms)
 * out_rows i64[nq, k] / out_scores f64[nq, k]: the k rows with the largest s ordered (s desc,
 * row asc) -- the reference's stable sorted(..., reverse=True) (:296, :321) over rows in index
 * order -- as row_offset + row, with their exact scores (bit-identical to vrq_search3's);
 * out_count i32[nq] = min(k, n); unused slots -1 / NaN.  Queries must be finite.
 * Exact for every input: int8-quantised queries on v_mfma_i32_32x32x32_i8 give scores within a
 * proven per-query bound, a sampled threshold keeps every row that can reach the top-k, and the
 * survivors are rescored exactly (heavy-tie inputs fall back to an exact scan of every row).
 * flags: 0, or a subset of the VRQ_GEMM_STAGE_* (issued in order SAMPLE, MAIN, FINISH on one
 * workspace = the full call; FINISH consumes the thresholds SAMPLE wrote, so every MAIN + FINISH
 * pair needs its own SAMPLE before it), optionally | VRQ_GEMM_NO_FALLBACK: queries the matrix
 * path could not serve (heavy exact ties) are left with out_count = -1 and unwritten rows instead
 * of taking the exact per-query scan of every row (callers that must bound latency; tests prove
 * with it that the matrix path alone served a batch).
 * Supported: dim = 1024, 1 <= k <= 1024, 1 <= n < 2^32.
 * ------------------------------------------------------------------------- */
#define VRQ_GEMM_BINARY 2
#define VRQ_GEMM_INT8_COSINE 3
#define VRQ_GEMM_STAGE_SAMPLE 16 /* query split + dense sample pass + per-query thresholds */
#define VRQ_GEMM_STAGE_MAIN 32   /* thresholded pass over every row -> candidate lists */
#define VRQ_GEMM_STAGE_FINISH 64 /* exact rescoring + sort of the candidates (+ exact fallback) */
#define VRQ_GEMM_NO_FALLBACK 128 /* skip the exact fallback: unserved queries get out_count = -1 */
size_t vrq_gemm_topk_workspace_size(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k);
/* int8 pieces per query of this build's matrix pass (1: q ~ S*a, 2: q ~ S*(a + b/256)); the
 * algorithmic ops of a pass are 2*nq*n*dim either way (for roofline reporting) */
int vrq_gemm_topk_pieces(void);
/* Host-only planning introspection (no reference counterpart; for tests and tools): the matrix
 * passes' plan of a vrq_gemm_topk / vrq_flat_ip_topk call shape.  info i64[8] = chunk rows, chunks,
 * per-(query, chunk) list capacity, query blocks, sample chunks, rows per sample chunk, workspace
 * bytes, queries per block.  VRQ_EUNSUPPORTED for shapes the path does not serve. */
int vrq_gemm_topk_plan(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k, int64_t* info);
/* Host-only introspection of the workspace layout (tests checking the candidate lists a MAIN stage
 * leaves): info i64[8] = padded queries nq_pad; byte offsets of the per-query thresholds (f32
 * [nq_pad], u units), the list lengths (i32 [nq][chunks]), the lists (u32 rows [nq][chunks][capc]) and
 * the sample maxima (f32 [nq][cols]); sample columns per query, rows between sample chunks, rows per
 * sample chunk.  The int8 query pieces a (q/S = a + rho) sit at offset 0 as i8 [nq_pad][1024]: natural
 * dim order for VRQ_GEMM_INT8_COSINE, and within each 32-dim step the Phase-II k-permutation for
 * VRQ_GEMM_BINARY.  Hit rule of the MAIN pass: binary u = <a, bits> >= ceil(thr); cosine u =
 * f32(<a, x>) * (1 / f32(norm)) >= thr. */
int vrq_gemm_topk_layout(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k, int64_t* info);
int vrq_gemm_topk(int32_t mode, const uint8_t* codes, const int8_t* x8, const double* norms, int64_t n,
                  int32_t dim, int64_t row_offset, const float* qf, int32_t nq, int32_t k, int32_t flags,
                  int32_t* out_count, int64_t* out_rows, double* out_scores, void* workspace,
                  size_t workspace_bytes, void* stream);
/* ---------------------------------------------------------------------------
 * Exact float inner-product top-k: CohereVectorDBFloat's faiss.IndexIDMap(faiss.IndexFlatIP(d))
 * (CohereVectorDBFloat.py:55-64) searched at :156, for a batch of queries, on the matrix cores.
 *   s = q . x in float32 (the exact products summed in float64, rounded once to float32)
 * out_* as vrq_gemm_topk: the k rows with the largest s ordered (s desc, row asc) -- FAISS's
 * IndexFlatIP result order, re-sorted stably by score at :170 -- as row_offset + row, scores f64
 * holding the float32 values.
 * vrq_flat_ip_prepare (once per added batch, rows [0, n) of the given pointers) derives the
 * matrix pass's operands from the float32 rows xf: x8 int8[n, dim] (per-row scaled), inv_scale
 * f64[n] and the running corpus bounds f64[2], which it max-accumulates (zero them before the first
 * batch; after removals the old bounds stay valid upper bounds).  vrq_flat_ip_topk: exact for every
 * input -- int8 queries x int8 rows on v_mfma_i32_32x32x32_i8 within a proven per-query bound, a
 * sampled threshold, exact rescoring of the survivors from xf (exact fallback on heavy ties).
 * Workspace: vrq_gemm_topk_workspace_size(VRQ_GEMM_FLOAT_IP, ...).  Supported: dim = 1024,
 * 1 <= k <= 1024, 1 <= n < 2^32, finite inputs.
 * ------------------------------------------------------------------------- */
#define VRQ_GEMM_FLOAT_IP 4
int vrq_flat_ip_prepare(const float* xf, int64_t n, int32_t dim, int8_t* x8, double* inv_scale, double* bounds,
                        void* stream);
int vrq_flat_ip_topk(const float* xf, const int8_t* x8, const double* inv_scale, const double* bounds, int64_t n,
                     int32_t dim, int64_t row_offset, const float* qf, int32_t nq, int32_t k, int32_t flags,
                     int32_t* out_count, int64_t* out_rows, double* out_scores, void* workspace,
                     size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VRQ_H_ */
