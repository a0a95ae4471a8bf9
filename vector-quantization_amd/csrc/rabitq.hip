// rabitq.hip — 1-bit RaBitQ encode / decode (faiss RaBitQuantizer layout).
//
// Restates faiss.RaBitQuantizer.compute_codes / decode as called by RaBitQuantizer
// (/root/reference/src/haag_vq/methods/rabit_quantization.py:20-29); see
// oracle/mivq_oracle.c for the scalar restatement this kernel is tested against.
//   code row = ceil(d/8) sign bytes (bit j = (x_j - c_j) > 0, LSB-first) ++ f32 {l2, mult}
// The sign bits are bit-exact; the two factors are reduced in a different (parallel) order
// than the sequential restatement, so they — and the decoded values — agree within 1e-6
// relative (the contract is 1e-5).
//
// One wavefront per row: lane L owns byte L, L+64, ... (8 dims each, two 16-B loads), so a
// wave streams 2 KiB of contiguous row data per step; the three sums are wave-reduced.
#include "mivq_common.h"

#include <float.h>

namespace mivq {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <bool VEC>
__global__ __launch_bounds__(256) void rabitq_encode_kernel(const float* __restrict__ x, int64_t n, int d,
                                                            const float* __restrict__ centroid, int metric,
                                                            uint8_t* __restrict__ codes) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int nb = (d + 7) / 8, cs = nb + 8;
    const float* xr = x + row * d;
    uint8_t* code = codes + row * cs;
    float l2 = 0.0f, orl2 = 0.0f, dp = 0.0f;
    for (int byte = lane; byte < nb; byte += 64) {
        const int j0 = byte * 8;
        float v[8];
        if (VEC && j0 + 8 <= d) {
            const float4 a = *reinterpret_cast<const float4*>(xr + j0);
            const float4 b = *reinterpret_cast<const float4*>(xr + j0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = (j0 + u < d) ? xr[j0 + u] : 0.0f;
        }
        uint32_t bits = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (j0 + u >= d) break;
            const float xv = v[u];
            const float rr = centroid ? __fsub_rn(xv, centroid[j0 + u]) : xv;
            l2 = __builtin_fmaf(rr, rr, l2);
            orl2 = __builtin_fmaf(xv, xv, orl2);
            const bool b = rr > 0.0f;
            dp = __fadd_rn(dp, b ? rr : -rr);
            bits |= (uint32_t)b << u;
        }
        code[byte] = (uint8_t)bits;
    }
    l2 = wave_sum(l2);
    orl2 = wave_sum(orl2);
    dp = wave_sum(dp);
    if (lane == 0) {
        const float inv_d_sqrt = d == 0 ? 1.0f : __fdiv_rn(1.0f, sqrtf((float)d));
        const float inv_norm = fabsf(l2) < FLT_EPSILON ? 1.0f : __fdiv_rn(1.0f, sqrtf(l2));
        const float ndp = __fmul_rn(__fmul_rn(dp, inv_norm), inv_d_sqrt);
        const float inv_dp = fabsf(ndp) < FLT_EPSILON ? 1.0f : __fdiv_rn(1.0f, ndp);
        const float f0 = metric == MIVQ_METRIC_INNER_PRODUCT ? __fsub_rn(l2, orl2) : l2;
        const float f1 = __fmul_rn(inv_dp, sqrtf(l2));
        // the trailer is 4-byte aligned only when nb % 4 == 0: write bytes
        const uint32_t u0 = __float_as_uint(f0), u1 = __float_as_uint(f1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            code[nb + q] = (uint8_t)(u0 >> (8 * q));
            code[nb + 4 + q] = (uint8_t)(u1 >> (8 * q));
        }
    }
}

// d % 512 == 0 (every lane owns NI = d / 512 bytes), x and the centroid 16-B aligned: the same
// per-lane arithmetic in the same order as rabitq_encode_kernel (identical codes and factors),
// with the loads of G of a lane's bytes (x and centroid, 16-B loads) issued before any of them is
// used -- the generic loop waited for each byte's loads before issuing the next byte's (one
// 2 KiB step in flight per wave).  1M x 3072: 2.44 -> 2.33 ms (0.65 -> 0.68 of 8 TB/s,
// profiles/r04_s15).
template <int G>
__global__ __launch_bounds__(256) void rabitq_encode_wide_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                 const float* __restrict__ centroid, int metric,
                                                                 uint8_t* __restrict__ codes) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int nb = d / 8, cs = nb + 8, NI = nb / 64;
    const float* xr = x + row * d;
    uint8_t* code = codes + row * cs;
    const bool has_c = centroid != nullptr;
    float l2 = 0.0f, orl2 = 0.0f, dp = 0.0f;
    for (int i0 = 0; i0 < NI; i0 += G) {
        float4 xv[G][2], cv[G][2];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int j0 = (lane + 64 * (i0 + g)) * 8;
            xv[g][0] = *reinterpret_cast<const float4*>(xr + j0);
            xv[g][1] = *reinterpret_cast<const float4*>(xr + j0 + 4);
            if (has_c) {
                cv[g][0] = *reinterpret_cast<const float4*>(centroid + j0);
                cv[g][1] = *reinterpret_cast<const float4*>(centroid + j0 + 4);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float v[8] = {xv[g][0].x, xv[g][0].y, xv[g][0].z, xv[g][0].w,
                                xv[g][1].x, xv[g][1].y, xv[g][1].z, xv[g][1].w};
            const float c[8] = {cv[g][0].x, cv[g][0].y, cv[g][0].z, cv[g][0].w,
                                cv[g][1].x, cv[g][1].y, cv[g][1].z, cv[g][1].w};
            uint32_t bits = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float xu = v[u];
                const float rr = has_c ? __fsub_rn(xu, c[u]) : xu;
                l2 = __builtin_fmaf(rr, rr, l2);
                orl2 = __builtin_fmaf(xu, xu, orl2);
                const bool b = rr > 0.0f;
                dp = __fadd_rn(dp, b ? rr : -rr);
                bits |= (uint32_t)b << u;
            }
            code[lane + 64 * (i0 + g)] = (uint8_t)bits;
        }
    }
    l2 = wave_sum(l2);
    orl2 = wave_sum(orl2);
    dp = wave_sum(dp);
    if (lane == 0) {
        const float inv_d_sqrt = __fdiv_rn(1.0f, sqrtf((float)d));
        const float inv_norm = fabsf(l2) < FLT_EPSILON ? 1.0f : __fdiv_rn(1.0f, sqrtf(l2));
        const float ndp = __fmul_rn(__fmul_rn(dp, inv_norm), inv_d_sqrt);
        const float inv_dp = fabsf(ndp) < FLT_EPSILON ? 1.0f : __fdiv_rn(1.0f, ndp);
        const float f0 = metric == MIVQ_METRIC_INNER_PRODUCT ? __fsub_rn(l2, orl2) : l2;
        const float f1 = __fmul_rn(inv_dp, sqrtf(l2));
        const uint32_t u0 = __float_as_uint(f0), u1 = __float_as_uint(f1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            code[nb + q] = (uint8_t)(u0 >> (8 * q));
            code[nb + 4 + q] = (uint8_t)(u1 >> (8 * q));
        }
    }
}

// One thread per output float: x_j = (bit - 0.5f) * mult * 2 * (1/sqrt(d)) + c_j.
__global__ void rabitq_decode_kernel(const uint8_t* __restrict__ codes, int64_t n, int d,
                                     const float* __restrict__ centroid, float* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * (int64_t)d) return;
    const int64_t i = e / d;
    const int j = (int)(e % d);
    const int nb = (d + 7) / 8, cs = nb + 8;
    const uint8_t* code = codes + i * cs;
    uint32_t mu = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) mu |= (uint32_t)code[nb + 4 + q] << (8 * q);
    const float mult = __uint_as_float(mu);
    const float inv_d_sqrt = __fdiv_rn(1.0f, sqrtf((float)d));
    const float bit = ((code[j >> 3] >> (j & 7)) & 1u) ? 1.0f : 0.0f;
    const float a = __fmul_rn(__fsub_rn(bit, 0.5f), mult);
    const float b = __fmul_rn(a, 2.0f);
    const float c = __fmul_rn(b, inv_d_sqrt);
    out[e] = __fadd_rn(c, centroid ? centroid[j] : 0.0f);
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" int mivq_rabitq_encode(const float* x, int64_t n, int32_t d, const float* centroid, int32_t metric,
                                  uint8_t* codes, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "rabitq_encode: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "RaBitQuantizer supports METRIC_L2 / METRIC_INNER_PRODUCT only, got %d", metric);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && codes, MIVQ_ERR_INVALID, "rabitq_encode: null pointer");
    const bool vec = (d % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0);
#ifndef MIVQ_RQ_WIDE
#define MIVQ_RQ_WIDE 1
#endif
    const int ni = d / 512;
    const bool wide = MIVQ_RQ_WIDE && vec && d % 512 == 0 && reinterpret_cast<uintptr_t>(centroid) % 16 == 0;
    const dim3 grid((unsigned)ceil_div(n, 4));
    if (wide && ni % 6 == 0)
        hipLaunchKernelGGL(rabitq_encode_wide_kernel<6>, grid, dim3(256), 0, as_stream(stream), x, n, d, centroid,
                           metric, codes);
    else if (wide && ni % 4 == 0)
        hipLaunchKernelGGL(rabitq_encode_wide_kernel<4>, grid, dim3(256), 0, as_stream(stream), x, n, d, centroid,
                           metric, codes);
    else if (wide && ni % 3 == 0)
        hipLaunchKernelGGL(rabitq_encode_wide_kernel<3>, grid, dim3(256), 0, as_stream(stream), x, n, d, centroid,
                           metric, codes);
    else if (wide && ni % 2 == 0)
        hipLaunchKernelGGL(rabitq_encode_wide_kernel<2>, grid, dim3(256), 0, as_stream(stream), x, n, d, centroid,
                           metric, codes);
    else if (vec)
        hipLaunchKernelGGL(rabitq_encode_kernel<true>, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0,
                           as_stream(stream), x, n, d, centroid, metric, codes);
    else
        hipLaunchKernelGGL(rabitq_encode_kernel<false>, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0,
                           as_stream(stream), x, n, d, centroid, metric, codes);
    return check_launch("rabitq_encode");
}

extern "C" int mivq_rabitq_decode(const uint8_t* codes, int64_t n, int32_t d, const float* centroid, float* out,
                                  void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "rabitq_decode: bad sizes");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(codes && out, MIVQ_ERR_INVALID, "rabitq_decode: null pointer");
    hipLaunchKernelGGL(rabitq_decode_kernel, dim3((unsigned)ceil_div(n * (int64_t)d, 256)), dim3(256), 0,
                       as_stream(stream), codes, n, d, centroid, out);
    return check_launch("rabitq_decode");
}
