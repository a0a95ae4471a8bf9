// Profiling harness: the codebook-stationary PQ encode kernel with parts of its work removed
// (see the V bits at CsCtx in pq_encode_cs.hip).  Built by tools/cs_variants.py; the
// library itself only instantiates V = 0.
#include "../vector-quantization_amd/csrc/pq_encode_cs.hip"

#define VARIANT(v)                                                                                     \
    case v:                                                                                           \
        return (int)mivq::launch_ks<6, v>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, (hipStream_t)st);

extern "C" __attribute__((visibility("default"))) int cs_variant(int V, const float* x, int64_t n, int d, int M,
                                                                  int dsub, const float* C, const float* cn,
                                                                  const void* img, const float* hinit,
                                                                  const void* bnd, uint8_t* codesT, void* st) {
    switch (V) {
        VARIANT(0) VARIANT(1) VARIANT(2) VARIANT(3) VARIANT(7) VARIANT(39) VARIANT(35) VARIANT(19)
        default: return -1;
    }
}
