/*
 * mivq.h — C ABI of libmivq.so, the MI355X-native (gfx950) vector-quantization hot path.
 *
 * This is the drop-in boundary that replaces the faiss / numpy calls the reference's
 * quantizer classes make (citations are /root/reference/<path>:<line>).  Every entry
 * point is `extern "C"`, takes plain pointers and sizes, and is stream-ordered:
 *
 *   - Ownership: every buffer is caller-allocated DEVICE memory (e.g. a torch tensor's
 *     data_ptr()).  The library never allocates persistent memory; kernels that need
 *     scratch take an explicit workspace (size from the matching *_workspace_bytes()).
 *   - Errors: 0 on success, a negative MIVQ_ERR_* code otherwise; the message is kept in
 *     a thread-local buffer readable with mivq_last_error().  The Python host raises the
 *     same exception types the reference raises (AssertionError / ValueError /
 *     RuntimeError, see vector-quantization_amd/haag_vq/_native.py).
 *   - Threading: asynchronous on `stream` (a hipStream_t passed as void*; NULL = the
 *     legacy default stream of the current device).  Safe to call concurrently from
 *     several host threads on different streams or devices; no global mutable state
 *     besides the per-thread error string.  No call synchronises the device.
 *   - Codes: PQ codes follow faiss' ProductQuantizer layout (code_size = ceil(M*nbits/8)
 *     bytes per vector, sub-code m in bits [m*nbits, (m+1)*nbits) of the little-endian
 *     bit stream; nbits == 8 is one byte per subspace).  Centroids are laid out
 *     (M, ksub, dsub) f32, exactly `pq.centroids.reshape(M, ksub, dsub)` of
 *     product_quantization.py:72-73.
 */
#ifndef MIVQ_H
#define MIVQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

#define MIVQ_OK 0
#define MIVQ_ERR_INVALID (-1)     /* bad shape / argument            -> ValueError / AssertionError */
#define MIVQ_ERR_UNSUPPORTED (-2) /* configuration not implemented   -> ValueError */
#define MIVQ_ERR_HIP (-3)         /* HIP runtime / launch failure    -> RuntimeError */
#define MIVQ_ERR_WORKSPACE (-4)   /* workspace too small             -> RuntimeError */

#define MIVQ_ABI_VERSION 2 /* 2: mivq_adc_search takes flags */

/* PQ encode flags */
#define MIVQ_PQ_AUTO 0u        /* fp16-MFMA candidate filter + exact fp32 re-check when supported */
#define MIVQ_PQ_FORCE_EXACT 1u /* exact fp32 VALU scan of every centroid (canonical order)     */
#define MIVQ_PQ_LEGACY_MFMA 2u /* diagnostic: subspace-looping MFMA kernel + separate resolve */
#define MIVQ_PQ_LEGACY_EXACT 4u /* diagnostic: lane-per-row exact kernel instead of the tiled one */

/* Metric enum values follow faiss / haag_vq.utils.faiss_utils.MetricType (faiss_utils.py:3-5). */
#define MIVQ_METRIC_INNER_PRODUCT 0
#define MIVQ_METRIC_L2 1

/* ---------------------------------------------------------------- misc */
const char* mivq_last_error(void);
int mivq_abi_version(void);
/* Fills name (>= 64 bytes), compute units, LDS bytes per CU, and total HBM bytes of `device`. */
int mivq_device_info(int device, char* name, int32_t* cus, int64_t* lds_per_cu, int64_t* hbm_bytes);

/* ------------------------------------------------------ product quantizer
 * Replaces faiss.ProductQuantizer.compute_codes / decode behind
 * ProductQuantizer.compress / decompress (product_quantization.py:76-86).
 *
 * Canonical encode (what "bit-exact" is measured against, see oracle/mivq_oracle.c):
 *   cn[m][k]  = fmaf-chain over t ascending of c[m][k][t]^2
 *   dot       = fmaf-chain over t ascending of x[m*dsub+t] * c[m][k][t]   (starts at +0)
 *   score_k   = fl32(cn[m][k] - 2*dot)
 *   code[m]   = smallest k with the minimum score (scores that are NaN never win; an
 *               all-NaN row gives 0).
 */

/* Bytes of the derived codebook data ("prep") for mivq_pq_encode. */
size_t mivq_pq_prep_bytes(int32_t d, int32_t M, int32_t nbits);
/* Builds prep from centroids (device): canonical norms, the fp16 MFMA operand image and
 * the per-subspace rounding-bound constants.  Re-run whenever the centroids change. */
int mivq_pq_prepare(const float* centroids, int32_t d, int32_t M, int32_t nbits, void* prep,
                    void* stream);
size_t mivq_pq_encode_workspace_bytes(int64_t n, int32_t d, int32_t M, int32_t nbits);
/* x: (n, d) f32 row-major; codes: (n, code_size) u8; prep from mivq_pq_prepare (required;
 * the exact path reads its canonical norms and transposed codebook). */
int mivq_pq_encode(const float* x, int64_t n, int32_t d, int32_t M, int32_t nbits,
                   const float* centroids, const void* prep, void* workspace,
                   size_t workspace_bytes, uint8_t* codes, uint32_t flags, void* stream);
/* out: (n, d) f32: out[i, m*dsub:(m+1)*dsub] = centroids[m, code_m(i), :]. */
int mivq_pq_decode(const uint8_t* codes, int64_t n, int32_t d, int32_t M, int32_t nbits,
                   const float* centroids, float* out, void* stream);
/* faiss bit-stream <-> one byte per sub-code (identity copy for nbits == 8). */
int mivq_pq_unpack(const uint8_t* codes, int64_t n, int32_t M, int32_t nbits, uint8_t* out,
                   void* stream);

/* ---------------------------------------------------- k-means (PQ fit)
 * Deterministic centroid update for the per-subspace Lloyd iterations that replace
 * faiss' ProductQuantizer.train (product_quantization.py:67-68): sums[m][k][t] are
 * accumulated over assigned rows in ascending row order, centroids = sums / count for
 * non-empty clusters (empty clusters keep their previous value and report count 0).
 * assign: (n, M) u8 (one byte per subspace, the output of mivq_pq_encode with nbits 8
 * or of mivq_pq_unpack).  counts: (M, ksub) int32. */
int mivq_kmeans_update(const float* x, int64_t n, int32_t d, int32_t M, int32_t ksub,
                       const uint8_t* assign, float* centroids, int32_t* counts, void* stream);

/* ------------------------------------------------------ OPQ rotation
 * Replaces faiss.OPQMatrix.apply / reverse_transform
 * (optimized_product_quantization.py:26,31,34).  A is (d, d) f32 row-major.
 *   transpose == 0 : y = x . A^T   (apply)
 *   transpose == 1 : y = x . A     (reverse_transform of an orthonormal A) */
int mivq_opq_rotate(const float* x, int64_t n, int32_t d, const float* A, int32_t transpose,
                    float* y, void* stream);

/* The same rotation at f16-MFMA speed with fp32 accuracy (the product path of
 * OptimizedProductQuantizer): mivq_opq_prepare splits op(A) once into scaled f16 hi / lo
 * images (prep: mivq_opq_prep_bytes(d) bytes, 16-byte aligned; 0 when d % 8 != 0), and
 * mivq_opq_rotate_prepared computes y = x . op(A) as x_hi b_hi + x_hi b_lo + x_lo b_hi with
 * per-row power-of-two scales of x.  Workspace (16-byte aligned):
 * mivq_opq_rotate_workspace_bytes(n, d) = the row scales (4 n B, rounded up to 256 B). */
size_t mivq_opq_prep_bytes(int32_t d);
int mivq_opq_prepare(const float* A, int32_t d, int32_t transpose, void* prep, void* stream);
size_t mivq_opq_rotate_workspace_bytes(int64_t n, int32_t d);
int mivq_opq_rotate_prepared(const float* x, int64_t n, int32_t d, const void* prep, void* workspace,
                             size_t workspace_bytes, float* y, void* stream);
/* Training: G = X^T Y in fp64 (d, d) row-major for the OPQ orthogonal-Procrustes update
 * (OPQMatrix::train's X^T Yhat, optimized_product_quantization.py:21-28); x, y: (n, d) f32.
 * fp64 MFMA, split over rows, the parts added in a fixed order (deterministic).  Workspace:
 * mivq_opq_gram_workspace_bytes(n, d) bytes, 8-byte aligned. */
size_t mivq_opq_gram_workspace_bytes(int64_t n, int32_t d);
int mivq_opq_gram(const float* x, const float* y, int64_t n, int32_t d, void* workspace,
                  size_t workspace_bytes, double* G, void* stream);

/* ------------------------------------------------------ scalar quantizer
 * Replaces ScalarQuantizer._compress_block / decompress (scalar_quantization.py:52-90)
 * bit-for-bit, in the dtype numpy would compute in (f32 input -> f32 math, f64 -> f64).
 *   lo  = X.min(0), den = (X.max(0) - X.min(0)) + 1e-8 (computed by the caller exactly as
 *   numpy does); codes: u8 for nbits 4 (two dims per byte, even dim in the high nibble,
 *   odd d zero-padded) and 8, u16 for nbits 16.  Decode returns f32 for the f32 variant
 *   and f64 for the f64 variant (what numpy returns). */
int mivq_sq_encode_f32(const float* x, int64_t n, int32_t d, const float* lo, const float* den,
                       int32_t nbits, void* codes, void* stream);
int mivq_sq_encode_f64(const double* x, int64_t n, int32_t d, const double* lo,
                       const double* den, int32_t nbits, void* codes, void* stream);
int mivq_sq_decode_f32(const void* codes, int64_t n, int32_t d, const float* lo,
                       const float* den, int32_t nbits, float* out, void* stream);
int mivq_sq_decode_f64(const void* codes, int64_t n, int32_t d, const double* lo,
                       const double* den, int32_t nbits, double* out, void* stream);

/* ------------------------------------------------------ RaBitQ (1 bit)
 * Replaces faiss.RaBitQuantizer.compute_codes / decode (rabit_quantization.py:20-29).
 * Code row = ceil(d/8) sign bytes (bit j of dim j = (x_j - c_j) > 0, LSB-first) followed by
 * two f32 factors {||x-c||^2, dp_multiplier}; code_size = ceil(d/8) + 8.
 * centroid may be NULL (faiss' default: no centroid). */
int mivq_rabitq_encode(const float* x, int64_t n, int32_t d, const float* centroid,
                       int32_t metric, uint8_t* codes, void* stream);
int mivq_rabitq_decode(const uint8_t* codes, int64_t n, int32_t d, const float* centroid,
                       float* out, void* stream);
/* RaBitQ estimator search: replaces faiss.IndexRaBitQ.search behind RaBitQIndex
 * (methods/search/rabitq_index.py:42-70; qb = IndexRaBitQ.qb query bits, 0..8).  codes: (n,
 * code_size) rows from mivq_rabitq_encode with the same centroid (IndexRaBitQ's center);
 * q: (nq, d) f32.  Per query r = q - c is quantised to qb bits (min/max grid, round half up);
 * the estimate of ||q - x||^2 is  f0 + ||r||^2 - 2 f1 <r', bits>-term  (arithmetic:
 * oracle/mivq_oracle.c oracle_rabitq_est).  dists/ids: (nq, k) ascending keys, ties to the
 * smaller id; L2 keys are the distance estimates, INNER_PRODUCT keys the negated
 * inner-product estimates.  ids = id_offset + row.  Workspace from
 * mivq_rabitq_search_workspace_bytes. */
size_t mivq_rabitq_search_workspace_bytes(int64_t nq, int64_t n, int32_t d, int32_t k);
int mivq_rabitq_search(const uint8_t* codes, int64_t n, int32_t d, const float* centroid,
                       const float* q, int64_t nq, int32_t qb, int32_t metric, int32_t k,
                       int64_t id_offset, void* workspace, size_t workspace_bytes, float* dists,
                       uint32_t* ids, void* stream);

/* ------------------------------------------------------ Extended RaBitQ (B bits)
 * The element-wise / per-row steps of ExtendedRaBitQuantizer.compress / decompress
 * (extended_rabitq.py:125-199), fp64 like the reference, and the two D x D rotations
 * between them (o . P and o_hat . P^T, :140 and :196) as an fp64-MFMA GEMM.
 *   normalize : o = (x - c) / max(||x - c||, 1e-12), nrm = ||x - c||   (x f32 or f64)
 *   quantize  : s = s_raw * sqrt(D); idx = searchsorted(mid-levels, s); t = <s,s_hat>/<s_hat,s_hat>
 *               code row = MSB-first B-bit indices (ceil(D*B/8) bytes) ++ f32 nrm ++ f32 t
 *   dequantize: o_hat = (levels[idx] / sqrt(D)) * t
 *   finish    : x_hat = f32(y * nrm + c)  with y = o_hat . P^T */
int mivq_extrabitq_normalize(const void* x, int32_t x_is_f64, int64_t n, int32_t d,
                             const double* centroid, double* o, double* nrm, void* stream);
int mivq_extrabitq_quantize(const double* s_raw, int64_t n, int32_t d, const double* levels,
                            int32_t nbits, const double* nrm, uint8_t* codes, void* stream);
int mivq_extrabitq_dequantize(const uint8_t* codes, int64_t n, int32_t d, const double* levels,
                              int32_t nbits, double* o_hat, void* stream);
int mivq_extrabitq_finish(const double* y, int64_t n, int32_t d, const uint8_t* codes,
                          int32_t nbits, const double* centroid, float* out, void* stream);
/* s = o . P (transpose 0) or o . P^T (transpose 1); o, s: (n, d) f64 row-major, P: (d, d). */
int mivq_extrabitq_rotate(const double* o, int64_t n, int32_t d, const double* P, int32_t transpose,
                          double* s, void* stream);

/* ------------------------------------------------------ ADC search
 * Flat asymmetric-distance search over PQ codes; the GPU counterpart of
 * FlatQuantizedIndex.search_with_scores (methods/search/flat_quantized_index.py:45-76),
 * which decodes every code and ranks exact distances to the reconstructions.
 *   lut[q][m][k] = sum over t ascending of (q[m*dsub+t] - c[m][k][t])^2 (fmaf chain), or for
 *                  metric == MIVQ_METRIC_INNER_PRODUCT  -(fmaf chain of q * c)
 *   dist(q, i)   = ((lut[q][0][code_0] + lut[q][1][code_1]) + ...) + lut[q][M-1][code_M-1]
 * Results per query are the k smallest (dist, id) pairs in ascending (dist, id) order
 * (ties broken by the smaller global id = id_offset + row); missing slots (n < k) hold
 * dist = +inf, id = 0xFFFFFFFF. */
int mivq_adc_lut(const float* q, int64_t nq, int32_t d, int32_t M, int32_t nbits,
                 const float* centroids, int32_t metric, float* lut, void* stream);
size_t mivq_adc_search_workspace_bytes(int64_t nq, int64_t n, int32_t M, int32_t nbits, int32_t k);
/* codes: (n, M) one byte per sub-code (nbits <= 8; use mivq_pq_unpack for nbits < 8).
 * flags: MIVQ_ADC_AUTO (0) for every product call; the other bits are diagnostics / test
 * hooks and change no result except MIVQ_ADC_NO_RERUN (see below).  The workspace size does
 * not depend on flags. */
#define MIVQ_ADC_AUTO 0u          /* filtered search where the shape allows it, else the fp32 scan */
#define MIVQ_ADC_FORCE_EXACT 1u   /* diagnostic: the fp32 scan for every query (same results)      */
#define MIVQ_ADC_NO_RERUN 2u      /* test hook: queries the filter cannot certify are left NaN      */
#define MIVQ_ADC_SMALL_RERUN_GRID 4u /* test hook: the re-run of uncertified queries on one column of
                                        workgroups, each walking several list-slot blocks          */
int mivq_adc_search(const float* lut, int64_t nq, const uint8_t* codes, int64_t n, int32_t M,
                    int32_t nbits, int32_t k, int64_t id_offset, void* workspace,
                    size_t workspace_bytes, float* dists, uint32_t* ids, uint32_t flags, void* stream);
/* Exact brute-force top-k over an f32 database (the decode-then-search path of
 * FlatQuantizedIndex for SQ / RaBitQ reconstructions, flat_quantized_index.py:57-76):
 *   L2: dist = fmaf chain over t of (q_t - x_t)^2;  IP: dist = -(fmaf chain of q_t * x_t)
 * ranked ascending by (dist, id) exactly like mivq_adc_search (callers negate IP back). */
size_t mivq_flat_search_workspace_bytes(int64_t nq, int64_t n, int32_t d, int32_t k);
int mivq_flat_search(const float* q, int64_t nq, const float* x, int64_t n, int32_t d,
                     int32_t metric, int32_t k, int64_t id_offset, void* workspace,
                     size_t workspace_bytes, float* dists, uint32_t* ids, void* stream);
/* Merges `parts` sorted (nq, k) lists laid out (parts, nq, k) into one sorted (nq, k) list
 * with the same (dist, id) order — the on-device merge after the RCCL all-gather. */
int mivq_topk_merge(const float* dists_in, const uint32_t* ids_in, int32_t parts, int64_t nq,
                    int32_t k, float* dists_out, uint32_t* ids_out, void* stream);

/* ------------------------------------------------------ IVF: coarse quantizer, lists, IVF-PQ
 * GPU counterpart of FaissIvfPqIndex (methods/search/faiss_ivfpq_index.py:46-76: faiss
 * IndexIVFPQ over an IndexFlatL2 / IndexFlatIP coarse quantizer, residual PQ) and of the
 * IVF build in benchmarks/ivf_benchmark.py:170-204.
 *
 * Exact pairwise distances, out (n, m) row-major (the coarse quantizer's exhaustive search
 * and the k-means assignment); the chains of mivq_flat_search:
 *   L2: out[i][j] = fmaf chain over t ascending of (x_i[t] - y_j[t])^2
 *   IP: out[i][j] = -(fmaf chain of x_i[t] * y_j[t]) */
int mivq_pairwise_distances(const float* x, int64_t n, const float* y, int64_t m, int32_t d,
                            int32_t metric, float* out, void* stream);
/* Per row of an (n, m) matrix, the k smallest (value, column) pairs ascending (NaN ranks as
 * +inf, ties to the smaller column); missing slots (m < k) hold (+inf, 0xFFFFFFFF). */
int mivq_topk_rows(const float* dist, int64_t n, int64_t m, int32_t k, float* out_d,
                   uint32_t* out_i, void* stream);
/* Stable bucket sort of assignments (n,) in [0, K), K <= 16384: offsets (K + 1) int64, the
 * rows of bucket l are order[offsets[l] .. offsets[l+1]) in ascending row order. */
size_t mivq_bucket_sort_workspace_bytes(int64_t n, int32_t K);
int mivq_bucket_sort(const uint32_t* assign, int64_t n, int32_t K, int64_t* offsets,
                     uint32_t* order, void* workspace, size_t workspace_bytes, void* stream);
/* k-means update from a bucket sort: centroids[l][t] = (f32 sum over the bucket's rows in
 * ascending row order of x[row][t]) / count for non-empty buckets (empty buckets keep their
 * value); counts (K,) int32. */
int mivq_centroid_update(const float* x, int64_t n, int32_t d, int32_t K, const int64_t* offsets,
                         const uint32_t* order, float* centroids, int32_t* counts, void* stream);
/* r[i][t] = x[i][t] - coarse[assign[i]][t] */
int mivq_ivf_residuals(const float* x, int64_t n, int32_t d, const float* coarse,
                       const uint32_t* assign, float* r, void* stream);
/* dst row i = src row order[i]; row_bytes a multiple of 4 */
int mivq_gather_rows(const void* src, int64_t row_bytes, const uint32_t* order, int64_t n,
                     void* dst, void* stream);
/* IVF-PQ L2 term per vector (faiss' precomputed table folded per code):
 *   tau_i = ((t_0 + t_1) + ...) + t_{M-1},  t_m = cn[m][k] + 2 * (fmaf chain over t of
 *   coarse[assign_i][m*dsub + t] * C[m][k][t]),  k = codes[i][m]
 * cn = the canonical ||C[m][k]||^2 of mivq_pq_prepare (first block of the prep buffer). */
int mivq_ivfpq_terms(const uint8_t* codes, int64_t n, int32_t d, int32_t M, int32_t nbits,
                     const float* pq_centroids, const float* cn, const float* coarse,
                     const uint32_t* assign, float* tau, void* stream);
/* IVF-PQ search over inverted lists in bucket order:
 *   lut (nq, M, ksub): mivq_adc_lut with MIVQ_METRIC_INNER_PRODUCT (= -(q . c) chains)
 *   probe_d, probe_l (nq, nprobe): coarse distances and list ids (mivq_topk_rows); list id
 *     0xFFFFFFFF slots are skipped
 *   offsets (nlist + 1), list_codes (N, M) u8, list_ids (N,), tau (N,) in bucket order
 *   S = ((lut[q][0][c_0] + lut[q][1][c_1]) + ...) + lut[q][M-1][c_{M-1}]
 *   L2: dist = (probe_d + tau) + 2 * S  (= ||q - coarse_l - r_hat||^2 expanded)
 *   IP: dist = probe_d + S              (= -(q . coarse_l + q . r_hat))
 * ranked like mivq_adc_search: ascending (dist, id) with id = the list_ids entry. */
size_t mivq_ivfpq_search_workspace_bytes(int64_t nq, int32_t nprobe, int32_t k);
int mivq_ivfpq_search(const float* lut, int64_t nq, int32_t M, int32_t nbits, const float* probe_d,
                      const uint32_t* probe_l, int32_t nprobe, int32_t nlist, const int64_t* offsets,
                      const uint8_t* list_codes, const uint32_t* list_ids, const float* tau,
                      int32_t metric, int32_t k, void* workspace, size_t workspace_bytes,
                      float* dists, uint32_t* ids, void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* MIVQ_H */
