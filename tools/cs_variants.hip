// Profiling harness: the codebook-stationary PQ encode kernel with parts of its work removed
// (see the V bits at CsCtx in pq_encode_cs.hip).  Built by tools/cs_variants.py; the
// library itself only instantiates V = 0.
#include "../vector-quantization_amd/csrc/pq_encode_cs.hip"

#ifndef CS_KS  // K-steps of the subspace shape (dsub = 16 CS_KS for the specialised kernels)
#define CS_KS 6
#endif

#define VARIANT(v)                                                                                     \
    case v:                                                                                           \
        return (int)mivq::launch_pq_encode_cs_v<CS_KS, v>(x, n, d, M, dsub, C, cn, img, hinit, bnd, pd, bnd2, codesT, items, \
                                                      counts, pinfo, (hipStream_t)st);

extern "C" __attribute__((visibility("default"))) int cs_variant(int V, const float* x, int64_t n, int d, int M,
                                                                  int dsub, const float* C, const float* cn,
                                                                  const void* img, const float* hinit,
                                                                  const void* bnd, const void* pd, const void* bnd2,
                                                                  uint8_t* codesT, void* items, void* counts, void* pinfo,
                                                                  void* st) {
    switch (V) {
#ifdef CS_VARIANTS
        CS_VARIANTS
#else
        VARIANT(0) VARIANT(1) VARIANT(2) VARIANT(4) VARIANT(8) VARIANT(17) VARIANT(33) VARIANT(65) VARIANT(145) VARIANT(256) VARIANT(513) VARIANT(1537) VARIANT(2561) VARIANT(4609) VARIANT(7681) VARIANT(16384) VARIANT(32768) VARIANT(65536) VARIANT(131073) VARIANT(131072) VARIANT(262144) VARIANT(1048576) VARIANT(2097152) VARIANT(4194304) VARIANT(8388608) VARIANT(6291456)
#endif
        default: return -1;
    }
}

// Read-bandwidth calibration: every byte of x read once with 16-B loads, U independent loads
// per thread in flight, grid-stride over the buffer; AUX the cache policy (2 = nt).
template <int U, int AUX>
__global__ __launch_bounds__(1024) void read_probe_kernel(const float4* __restrict__ x, int64_t n4, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, 0x7FFFFFFF, 0x00020000);
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < n4; base += stride * U) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * stride;
            if (i < n4) {
                const float4 f = x[i];
                v[u] = __float_as_uint(f.x) ^ __float_as_uint(f.y) ^ __float_as_uint(f.z) ^ __float_as_uint(f.w);
            } else {
                v[u] = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    (void)rs;
    if (acc == 0x12345678u) out[0] = acc;
}

extern "C" __attribute__((visibility("default"))) int read_probe(int P, const float* x, int64_t nfloats, void* out,
                                                                 void* st) {
    const int64_t n4 = nfloats / 4;
    hipStream_t s = (hipStream_t)st;
    switch (P) {
        case 0: read_probe_kernel<4, 0><<<1024, 1024, 0, s>>>((const float4*)x, n4, (uint32_t*)out); break;
        case 1: read_probe_kernel<8, 0><<<512, 1024, 0, s>>>((const float4*)x, n4, (uint32_t*)out); break;
        case 2: read_probe_kernel<12, 0><<<256, 768, 0, s>>>((const float4*)x, n4, (uint32_t*)out); break;
        case 3: read_probe_kernel<2, 0><<<4096, 1024, 0, s>>>((const float4*)x, n4, (uint32_t*)out); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
