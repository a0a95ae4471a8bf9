/*
 * selftest.c — memory-safety run of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * `make -C oracle asan` compiles this file, which includes mivq_oracle.c itself, with
 * -fsanitize=address,undefined and runs every exported restatement on small seeded inputs
 * at the shape edges (n = 0 / 1 / ragged, dsub not a multiple of 4, odd d for the 4-bit SQ
 * pack, k > n, nbits < 8, NaN / inf entries).  It checks a few invariants on the way (pack /
 * unpack round trip, decode of the encode's codes, sorted top-k lists) and exits non-zero on
 * any mismatch; the sanitizers abort on any out-of-bounds access or undefined operation.
 * tests/test_oracle.py::test_oracle_asan_selftest builds and runs it.
 */
#include "mivq_oracle.c"

#include <stdio.h>

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static float frand(void) {  /* xorshift64*, uniform in [-1, 1) */
    rng_state ^= rng_state >> 12; rng_state ^= rng_state << 25; rng_state ^= rng_state >> 27;
    return (float)((rng_state * 0x2545F4914F6CDD1Dull) >> 40) / (float)(1u << 23) - 1.0f;
}
static float* fvec(size_t n) {
    float* v = (float*)malloc(sizeof(float) * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) v[i] = frand();
    return v;
}
static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { ++fails; fprintf(stderr, "FAIL: " __VA_ARGS__); fprintf(stderr, "\n"); } } while (0)

static void check_sorted(const float* d, const uint32_t* id, int64_t nq, int k, const char* what) {
    for (int64_t q = 0; q < nq; ++q)
        for (int j = 1; j < k; ++j) {
            const float a = d[q * k + j - 1], b = d[q * k + j];
            CHECK(a < b || (a == b && id[q * k + j - 1] <= id[q * k + j]) || (a != a) || (b != b), "%s order", what);
        }
}

static void pq_case(int64_t n, int d, int M, int nbits) {
    const int ksub = 1 << nbits, dsub = d / M;
    float* x = fvec((size_t)n * d);
    float* C = fvec((size_t)M * ksub * dsub);
    float* cn = (float*)malloc(sizeof(float) * M * ksub);
    uint8_t* u8 = (uint8_t*)malloc((size_t)(n ? n : 1) * M);
    const int cs = (M * nbits + 7) / 8;
    uint8_t* packed = (uint8_t*)malloc((size_t)(n ? n : 1) * cs);
    uint8_t* back = (uint8_t*)malloc((size_t)(n ? n : 1) * M);
    float* rec = (float*)malloc(sizeof(float) * (size_t)(n ? n : 1) * d);
    float* sc = (float*)malloc(sizeof(float) * ksub);
    oracle_pq_norms(C, M, ksub, dsub, cn);
    oracle_pq_encode(x, n, d, M, ksub, C, cn, u8);
    oracle_pq_pack(u8, n, M, nbits, packed);
    oracle_pq_unpack(packed, n, M, nbits, back);
    CHECK(n == 0 || memcmp(u8, back, (size_t)n * M) == 0, "pq pack/unpack n=%lld M=%d nbits=%d", (long long)n, M, nbits);
    oracle_pq_decode(u8, n, d, M, ksub, C, rec);
    for (int64_t i = 0; i < n; ++i)
        for (int m = 0; m < M; ++m) {
            oracle_pq_scores(x + i * d + (int64_t)m * dsub, dsub, ksub, C + (int64_t)m * ksub * dsub, cn + m * ksub, sc);
            for (int k = 0; k < ksub; ++k) CHECK(!(sc[k] < sc[u8[i * M + m]]), "pq argmin");
        }
    /* ADC over the codes, k larger than n */
    const int nq = 3, k = (int)n + 2;
    float* q = fvec((size_t)nq * d);
    float* lut = (float*)malloc(sizeof(float) * nq * M * ksub);
    float* dd = (float*)malloc(sizeof(float) * nq * k);
    uint32_t* ii = (uint32_t*)malloc(sizeof(uint32_t) * nq * k);
    for (int metric = 0; metric <= 1; ++metric) {
        oracle_adc_lut(q, nq, d, M, ksub, C, metric, lut);
        oracle_adc_search(lut, nq, u8, n, M, ksub, k, 5, dd, ii);
        check_sorted(dd, ii, nq, k, "adc");
        CHECK(ii[k - 1] == 0xFFFFFFFFu, "adc sentinel");
        oracle_flat_search(q, nq, rec, n, d, metric, k, 0, dd, ii);
        check_sorted(dd, ii, nq, k, "flat");
    }
    free(x); free(C); free(cn); free(u8); free(packed); free(back); free(rec); free(sc); free(q); free(lut); free(dd); free(ii);
}

static void sq_case(int64_t n, int d, int nbits) {
    float* x = fvec((size_t)n * d);
    double* xd = (double*)malloc(sizeof(double) * (size_t)(n ? n : 1) * d);
    for (int64_t i = 0; i < n * d; ++i) xd[i] = x[i];
    float* lo = fvec(d); float* den = fvec(d);
    double* lod = (double*)malloc(sizeof(double) * d); double* dend = (double*)malloc(sizeof(double) * d);
    for (int j = 0; j < d; ++j) { lo[j] = -1.0f; den[j] = 2.0f + 1e-8f; lod[j] = -1.0; dend[j] = 2.0 + 1e-8; }
    const int cw = nbits == 4 ? (d + 1) / 2 : d;
    void* codes = malloc((size_t)(n ? n : 1) * cw * (nbits == 16 ? 2 : 1));
    float* rec = (float*)malloc(sizeof(float) * (size_t)(n ? n : 1) * d);
    double* recd = (double*)malloc(sizeof(double) * (size_t)(n ? n : 1) * d);
    oracle_sq_encode_f32(x, n, d, lo, den, nbits, codes);
    oracle_sq_decode_f32(codes, n, d, lo, den, nbits, rec);
    const float step = 2.0f / (float)((1 << nbits) - 1);
    for (int64_t i = 0; i < n * d; ++i) CHECK(fabsf(rec[i] - x[i]) <= 0.51f * step + 1e-6f, "sq f32 round trip");
    oracle_sq_encode_f64(xd, n, d, lod, dend, nbits, codes);
    oracle_sq_decode_f64(codes, n, d, lod, dend, nbits, recd);
    free(x); free(xd); free(lo); free(den); free(lod); free(dend); free(codes); free(rec); free(recd);
}

static void rabitq_case(int64_t n, int d) {
    float* x = fvec((size_t)n * d);
    float* c = fvec(d);
    const int cs = (d + 7) / 8 + 8;
    uint8_t* codes = (uint8_t*)malloc((size_t)(n ? n : 1) * cs);
    float* rec = (float*)malloc(sizeof(float) * (size_t)(n ? n : 1) * d);
    const int nq = 2;
    float* q = fvec((size_t)nq * d);
    float* est = (float*)malloc(sizeof(float) * (size_t)nq * (n ? n : 1));
    for (int metric = 0; metric <= 1; ++metric) {
        oracle_rabitq_encode(x, n, d, metric ? c : NULL, metric, codes);
        oracle_rabitq_decode(codes, n, d, metric ? c : NULL, rec);
        oracle_rabitq_est(codes, n, d, q, nq, metric ? c : NULL, 4, metric, est);
    }
    free(x); free(c); free(codes); free(rec); free(q); free(est);
}

static void ivf_case(int64_t n, int d, int M, int K) {
    const int ksub = 256, dsub = d / M;
    float* x = fvec((size_t)n * d);
    float* C = fvec((size_t)M * ksub * dsub);
    float* cn = (float*)malloc(sizeof(float) * M * ksub);
    float* coarse = fvec((size_t)K * d);
    uint32_t* assign = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (int64_t i = 0; i < n; ++i) assign[i] = (uint32_t)(i % K);
    float* cent = (float*)malloc(sizeof(float) * K * d);
    int32_t* counts = (int32_t*)malloc(sizeof(int32_t) * K);
    oracle_centroid_update(x, n, d, K, assign, cent, counts);
    float* pw = (float*)malloc(sizeof(float) * (size_t)(n ? n : 1) * K);
    oracle_pairwise(x, n, coarse, K, d, 1, pw);
    uint8_t* codes = (uint8_t*)malloc((size_t)(n ? n : 1) * M);
    for (int64_t i = 0; i < n * M; ++i) codes[i] = (uint8_t)(i * 37);
    float* tau = (float*)malloc(sizeof(float) * (n ? n : 1));
    oracle_pq_norms(C, M, ksub, dsub, cn);
    oracle_ivfpq_terms(codes, n, d, M, ksub, C, cn, coarse, assign, tau);
    free(x); free(C); free(cn); free(coarse); free(assign); free(cent); free(counts); free(pw); free(codes); free(tau);
}

int main(void) {
    const int64_t ns[] = {0, 1, 7, 65};
    for (int a = 0; a < 4; ++a) {
        pq_case(ns[a], 24, 4, 8);   /* dsub 6 */
        pq_case(ns[a], 30, 5, 4);   /* dsub 6, 4-bit packing */
        pq_case(ns[a], 14, 7, 6);   /* dsub 2, 6-bit packing */
        sq_case(ns[a], 7, 4);       /* odd d: zero-padded nibble */
        sq_case(ns[a], 9, 8);
        sq_case(ns[a], 5, 16);
        rabitq_case(ns[a], 13);     /* d % 8 != 0 */
        rabitq_case(ns[a], 64);
        ivf_case(ns[a], 32, 8, 3);
    }
    /* NaN / inf rows through the encoders */
    float bad[24];
    for (int j = 0; j < 24; ++j) bad[j] = j % 3 == 0 ? NAN : (j % 3 == 1 ? INFINITY : -INFINITY);
    float* C = fvec(4 * 256 * 6);
    float cn[4 * 256];
    uint8_t u8[4];
    oracle_pq_norms(C, 4, 256, 6, cn);
    oracle_pq_encode(bad, 1, 24, 4, 256, C, cn, u8);
    free(C);
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    printf("oracle selftest ok\n");
    return 0;
}
