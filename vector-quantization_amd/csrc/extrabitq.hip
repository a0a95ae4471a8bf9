// extrabitq.hip — multi-bit ("Extended") RaBitQ encode / decode steps on gfx950.
//
// Restates ExtendedRaBitQuantizer.compress / decompress
// (/root/reference/src/haag_vq/methods/extended_rabitq.py:125-199), all in fp64 like numpy:
//   encode: r = x - c; nrm = ||r||; o = r / max(nrm, 1e-12)                 [normalize]
//           s = (o . P) * sqrt(D)   (the D x D product is a plain fp64 GEMM on the host side)
//           idx = searchsorted(mid-levels, s) (left); s_hat = levels[idx]
//           t = <s, s_hat> / <s_hat, s_hat>  (1 when the denominator <= 1e-12)
//           row = B-bit idx packed MSB-first (np.packbits) ++ f32 nrm ++ f32 t   [quantize]
//   decode: o_hat = (levels[idx] / sqrt(D)) * t                              [dequantize]
//           x_hat = f32((o_hat . P^T) * nrm + c)                             [finish]
// One wavefront per row for the reductions (tree order: the factors match numpy to ~1e-15
// relative, the indices are exact except where s lies within rounding of a level midpoint).
#include "mivq_common.h"

namespace mivq {
namespace {

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <typename T>
__global__ __launch_bounds__(256) void erq_normalize_kernel(const T* __restrict__ x, int64_t n, int d,
                                                            const double* __restrict__ c, double* __restrict__ o,
                                                            double* __restrict__ nrm) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    double ss = 0.0;
    for (int j = lane; j < d; j += 64) {
        const double r = __dsub_rn((double)x[row * d + j], c[j]);
        o[row * d + j] = r;
        ss = __fma_rn(r, r, ss);
    }
    ss = wave_sum_d(ss);
    const double nr = sqrt(ss);
    const double inv = fmax(nr, 1e-12);
    for (int j = lane; j < d; j += 64) o[row * d + j] = __ddiv_rn(o[row * d + j], inv);
    if (lane == 0) nrm[row] = nr;
}

// s_raw: (n, d) = o . P.  One wave per row.
__global__ __launch_bounds__(256) void erq_quantize_kernel(const double* __restrict__ s_raw, int64_t n, int d,
                                                           const double* __restrict__ levels, int nbits,
                                                           const double* __restrict__ nrm, uint8_t* __restrict__ codes) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int L = 1 << nbits;
    const int ib = (d * nbits + 7) / 8;
    const int cs = ib + 8;
    uint8_t* code = codes + row * cs;
    const double sq = sqrt((double)d);
    double num = 0.0, den = 0.0;
    // lane owns groups of 8 dims: 8 B-bit indices are exactly nbits whole bytes of the
    // MSB-first stream (np.packbits order), bits past d*nbits stay 0
    const int groups = (d + 7) / 8;
    for (int g = lane; g < groups; g += 64) {
        uint64_t bits = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = g * 8 + u;
            int idx = 0;
            if (j < d) {
                const double s = __dmul_rn(s_raw[row * d + j], sq);
                for (int q = 0; q + 1 < L; ++q) {
                    const double mid = __dmul_rn(0.5, __dadd_rn(levels[q], levels[q + 1]));
                    idx += (mid < s) ? 1 : 0;  // searchsorted(side="left")
                }
                const double sh = levels[idx];
                num = __fma_rn(s, sh, num);
                den = __fma_rn(sh, sh, den);
            }
            bits = (bits << nbits) | (uint64_t)idx;
        }
        for (int b = 0; b < nbits; ++b) {
            const int byte = g * nbits + b;
            if (byte < ib) code[byte] = (uint8_t)(bits >> (8 * (nbits - 1 - b)));
        }
    }
    num = wave_sum_d(num);
    den = wave_sum_d(den);
    if (lane == 0) {
        const double t = den > 1e-12 ? __ddiv_rn(num, den) : 1.0;
        const float nf = (float)nrm[row], tf = (float)t;
        const uint32_t u0 = __float_as_uint(nf), u1 = __float_as_uint(tf);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            code[ib + q] = (uint8_t)(u0 >> (8 * q));
            code[ib + 4 + q] = (uint8_t)(u1 >> (8 * q));
        }
    }
}

__global__ void erq_dequantize_kernel(const uint8_t* __restrict__ codes, int64_t n, int d,
                                      const double* __restrict__ levels, int nbits, double* __restrict__ o_hat) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * (int64_t)d) return;
    const int64_t i = e / d;
    const int j = (int)(e % d);
    const int ib = (d * nbits + 7) / 8;
    const uint8_t* code = codes + i * (ib + 8);
    int idx = 0;
    for (int u = 0; u < nbits; ++u) {
        const int gb = j * nbits + u;
        idx = (idx << 1) | ((code[gb >> 3] >> (7 - (gb & 7))) & 1);
    }
    uint32_t tu = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) tu |= (uint32_t)code[ib + 4 + q] << (8 * q);
    const double t = (double)__uint_as_float(tu);
    o_hat[e] = __dmul_rn(__ddiv_rn(levels[idx], sqrt((double)d)), t);
}

__global__ void erq_finish_kernel(const double* __restrict__ y, int64_t n, int d, const uint8_t* __restrict__ codes,
                                  int nbits, const double* __restrict__ c, float* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * (int64_t)d) return;
    const int64_t i = e / d;
    const int j = (int)(e % d);
    const int ib = (d * nbits + 7) / 8;
    const uint8_t* code = codes + i * (ib + 8);
    uint32_t nu = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) nu |= (uint32_t)code[ib + q] << (8 * q);
    const double nr = (double)__uint_as_float(nu);
    out[e] = (float)__dadd_rn(__dmul_rn(y[e], nr), c[j]);
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" int mivq_extrabitq_normalize(const void* x, int32_t x_is_f64, int64_t n, int32_t d, const double* centroid,
                                        double* o, double* nrm, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "extrabitq_normalize: bad sizes");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && centroid && o && nrm, MIVQ_ERR_INVALID, "extrabitq_normalize: null pointer");
    const dim3 grid((unsigned)ceil_div(n, 4));
    if (x_is_f64)
        hipLaunchKernelGGL(erq_normalize_kernel<double>, grid, dim3(256), 0, as_stream(stream),
                           static_cast<const double*>(x), n, d, centroid, o, nrm);
    else
        hipLaunchKernelGGL(erq_normalize_kernel<float>, grid, dim3(256), 0, as_stream(stream),
                           static_cast<const float*>(x), n, d, centroid, o, nrm);
    return check_launch("extrabitq_normalize");
}

extern "C" int mivq_extrabitq_quantize(const double* s_raw, int64_t n, int32_t d, const double* levels, int32_t nbits,
                                       const double* nrm, uint8_t* codes, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "extrabitq_quantize: bad sizes");
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_INVALID, "num_bits must be in [1, 8]");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(s_raw && levels && nrm && codes, MIVQ_ERR_INVALID, "extrabitq_quantize: null pointer");
    hipLaunchKernelGGL(erq_quantize_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, as_stream(stream), s_raw, n,
                       d, levels, nbits, nrm, codes);
    return check_launch("extrabitq_quantize");
}

extern "C" int mivq_extrabitq_dequantize(const uint8_t* codes, int64_t n, int32_t d, const double* levels,
                                         int32_t nbits, double* o_hat, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0 && nbits >= 1 && nbits <= 8, MIVQ_ERR_INVALID, "extrabitq_dequantize: bad args");
    if (n == 0) return MIVQ_OK;
    hipLaunchKernelGGL(erq_dequantize_kernel, dim3((unsigned)ceil_div(n * (int64_t)d, 256)), dim3(256), 0,
                       as_stream(stream), codes, n, d, levels, nbits, o_hat);
    return check_launch("extrabitq_dequantize");
}

extern "C" int mivq_extrabitq_finish(const double* y, int64_t n, int32_t d, const uint8_t* codes, int32_t nbits,
                                     const double* centroid, float* out, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0 && nbits >= 1 && nbits <= 8, MIVQ_ERR_INVALID, "extrabitq_finish: bad args");
    if (n == 0) return MIVQ_OK;
    hipLaunchKernelGGL(erq_finish_kernel, dim3((unsigned)ceil_div(n * (int64_t)d, 256)), dim3(256), 0,
                       as_stream(stream), y, n, d, codes, nbits, centroid, out);
    return check_launch("extrabitq_finish");
}
