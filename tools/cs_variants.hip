// Profiling harness: the codebook-stationary PQ encode kernel with parts of its work removed
// (see the V bits at CsCtx in pq_encode_cs.hip).  Built by tools/cs_variants.py; the
// library itself only instantiates V = 0.
#include "../vector-quantization_amd/csrc/pq_encode_cs.hip"

#define VARIANT(v)                                                                                     \
    case v:                                                                                           \
        return (int)mivq::launch_pq_encode_cs_v<6, v>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, items, counts, (hipStream_t)st);

extern "C" __attribute__((visibility("default"))) int cs_variant(int V, const float* x, int64_t n, int d, int M,
                                                                  int dsub, const float* C, const float* cn,
                                                                  const void* img, const float* hinit,
                                                                  const void* bnd, uint8_t* codesT, void* items, void* counts, void* st) {
    switch (V) {
        VARIANT(0) VARIANT(1) VARIANT(2) VARIANT(4) VARIANT(8) VARIANT(17) VARIANT(33) VARIANT(65) VARIANT(145)
        default: return -1;
    }
}
