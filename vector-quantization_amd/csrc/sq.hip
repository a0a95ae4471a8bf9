// sq.hip — scalar quantizer encode / decode (4 / 8 / 16 bit), bit-exact with numpy.
//
// Restates ScalarQuantizer._compress_block / decompress
// (/root/reference/src/haag_vq/methods/scalar_quantization.py:52-90) in the precision numpy
// computes in: f32 inputs use f32 ops (NEP 50 weak Python scalars), f64 inputs f64 ops; the
// decode's level/(2^b-1) step is always f32 (codes.astype(np.float32)).  No op is fused
// (the library builds with -ffp-contract=off; the steps are written one rounding each).
// astype(uint8/uint16) follows numpy on x86-64: (uintN)(int32)r, every r int32 cannot hold
// (NaN, +-inf, |r| >= 2^31) -> 0.
//
// Layout: one lane handles 8 consecutive dims of a row (HBM-bound, 16-B loads when aligned).
#include "mivq_common.h"

namespace mivq {
namespace {

template <typename T>
__device__ __forceinline__ uint32_t np_cast_uint(T r) {
    if (!(r >= (T)-2147483648.0 && r < (T)2147483648.0)) return 0u;
    return (uint32_t)(int32_t)r;
}

__device__ __forceinline__ float sq_step(float x, float lo, float den, float L) {
    const float a = __fsub_rn(x, lo);
    const float b = __fdiv_rn(a, den);
    return rintf(__fmul_rn(b, L));
}
__device__ __forceinline__ double sq_step(double x, double lo, double den, double L) {
    const double a = __dsub_rn(x, lo);
    const double b = __ddiv_rn(a, den);
    return rint(__dmul_rn(b, L));
}

// Each thread: row i, dims [8g, 8g+8).  Output written as bytes / u16.
template <typename T>
__global__ void sq_encode_kernel(const T* __restrict__ x, int64_t n, int d, const T* __restrict__ lo,
                                 const T* __restrict__ den, int nbits, void* __restrict__ codes) {
    const int groups = (d + 7) / 8;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n * groups) return;
    const int64_t i = gid / groups;
    const int j0 = (int)(gid % groups) * 8;
    const T L = (T)((1 << nbits) - 1);
    uint32_t q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        q[u] = j < d ? np_cast_uint(sq_step(x[i * d + j], lo[j], den[j], L)) : 0u;
    }
    if (nbits == 8) {
        uint8_t* o = static_cast<uint8_t*>(codes) + i * d + j0;
#pragma unroll
        for (int u = 0; u < 8; ++u) if (j0 + u < d) o[u] = (uint8_t)q[u];
    } else if (nbits == 16) {
        uint16_t* o = static_cast<uint16_t*>(codes) + i * d + j0;
#pragma unroll
        for (int u = 0; u < 8; ++u) if (j0 + u < d) o[u] = (uint16_t)q[u];
    } else {  // 4-bit: (q[:,0::2] << 4) | q[:,1::2] in uint8 arithmetic, odd d zero-padded
        const int cw = (d + 1) / 2;
        uint8_t* o = static_cast<uint8_t*>(codes) + i * cw + j0 / 2;
#pragma unroll
        for (int u = 0; u < 8; u += 2)
            if ((j0 + u) / 2 < cw) o[u / 2] = (uint8_t)(((uint8_t)q[u] << 4) | (uint8_t)q[u + 1]);
    }
}

__device__ __forceinline__ float sq_level(const void* codes, int64_t i, int j, int d, int nbits) {
    if (nbits == 16) return (float)static_cast<const uint16_t*>(codes)[i * d + j];
    if (nbits == 8) return (float)static_cast<const uint8_t*>(codes)[i * d + j];
    const uint8_t b = static_cast<const uint8_t*>(codes)[i * ((d + 1) / 2) + (j >> 1)];
    return (float)((j & 1) ? (b & 0x0F) : (b >> 4));
}

template <typename T>
__global__ void sq_decode_kernel(const void* __restrict__ codes, int64_t n, int d, const T* __restrict__ lo,
                                 const T* __restrict__ den, int nbits, T* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * (int64_t)d) return;
    const int64_t i = e / d;
    const int j = (int)(e % d);
    const float L = (float)((1 << nbits) - 1);
    const float s = __fdiv_rn(sq_level(codes, i, j, d, nbits), L);
    if constexpr (sizeof(T) == 4) {
        out[e] = __fadd_rn(__fmul_rn(s, den[j]), lo[j]);
    } else {
        out[e] = __dadd_rn(__dmul_rn((double)s, den[j]), lo[j]);
    }
}

template <typename T>
int sq_encode(const T* x, int64_t n, int32_t d, const T* lo, const T* den, int32_t nbits, void* codes,
              void* stream, const char* name) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "%s: bad sizes n=%lld d=%d", name, (long long)n, d);
    MIVQ_REQUIRE(nbits == 4 || nbits == 8 || nbits == 16, MIVQ_ERR_INVALID,
                 "num_bits must be 4, 8, or 16, got %d", nbits);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && lo && den && codes, MIVQ_ERR_INVALID, "%s: null pointer", name);
    const int64_t work = n * ((d + 7) / 8);
    hipLaunchKernelGGL(sq_encode_kernel<T>, dim3((unsigned)ceil_div(work, 256)), dim3(256), 0, as_stream(stream),
                       x, n, d, lo, den, nbits, codes);
    return check_launch(name);
}

template <typename T>
int sq_decode(const void* codes, int64_t n, int32_t d, const T* lo, const T* den, int32_t nbits, T* out,
              void* stream, const char* name) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "%s: bad sizes", name);
    MIVQ_REQUIRE(nbits == 4 || nbits == 8 || nbits == 16, MIVQ_ERR_INVALID,
                 "num_bits must be 4, 8, or 16, got %d", nbits);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(codes && lo && den && out, MIVQ_ERR_INVALID, "%s: null pointer", name);
    hipLaunchKernelGGL(sq_decode_kernel<T>, dim3((unsigned)ceil_div(n * (int64_t)d, 256)), dim3(256), 0,
                       as_stream(stream), codes, n, d, lo, den, nbits, out);
    return check_launch(name);
}

}  // namespace
}  // namespace mivq

extern "C" int mivq_sq_encode_f32(const float* x, int64_t n, int32_t d, const float* lo, const float* den,
                                  int32_t nbits, void* codes, void* stream) {
    return mivq::sq_encode<float>(x, n, d, lo, den, nbits, codes, stream, "sq_encode_f32");
}
extern "C" int mivq_sq_encode_f64(const double* x, int64_t n, int32_t d, const double* lo, const double* den,
                                  int32_t nbits, void* codes, void* stream) {
    return mivq::sq_encode<double>(x, n, d, lo, den, nbits, codes, stream, "sq_encode_f64");
}
extern "C" int mivq_sq_decode_f32(const void* codes, int64_t n, int32_t d, const float* lo, const float* den,
                                  int32_t nbits, float* out, void* stream) {
    return mivq::sq_decode<float>(codes, n, d, lo, den, nbits, out, stream, "sq_decode_f32");
}
extern "C" int mivq_sq_decode_f64(const void* codes, int64_t n, int32_t d, const double* lo, const double* den,
                                  int32_t nbits, double* out, void* stream) {
    return mivq::sq_decode<double>(codes, n, d, lo, den, nbits, out, stream, "sq_decode_f64");
}
