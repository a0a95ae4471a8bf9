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
// Layout: one lane handles 8 consecutive dims of a row (HBM-bound; vector loads and packed
// stores on the aligned f32 fast path).
#include <algorithm>

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

// RN(a / den) from rcp = RN(1 / den) (vector fast path): q0 = RN(a rcp), the exact residual
// e = a - den q0 (one fma), q = RN(q0 + e rcp).  With rcp correctly rounded and q0 within an ulp
// of a / den, q is the correctly rounded quotient (Markstein's theorem) as long as nothing
// over- or underflows: the column's den and the element's a within [2^-62, 2^62] (or a == 0),
// otherwise the IEEE division sequence.  3 VALU instead of ~10.
__device__ __forceinline__ float div_rn_rcp(float a, float den, float rcp, bool col_ok) {
    const float aa = fabsf(a);
    if (col_ok && (aa == 0.0f || (aa >= 0x1p-62f && aa <= 0x1p62f))) {
        const float q0 = __fmul_rn(a, rcp);
        const float e = __builtin_fmaf(-q0, den, a);
        return __builtin_fmaf(e, rcp, q0);
    }
    return __fdiv_rn(a, den);
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

// Fast path (f32, d % 8 == 0, 16-B aligned rows): column-stationary.  Block (gx, gy) covers
// column groups 64 gx + [0, 64) (8 dims each, one per lane) of rows kSqRows gy + [0, kSqRows);
// a lane keeps its 8 lo / den values in registers and walks its rows (wave w takes rows
// w, w + 4, ...), four rows in flight: two 16-B loads of x and one 4 / 8 / 16-B store of
// packed codes per row, no per-element index arithmetic.  Same results as above (the division
// through div_rn_rcp).
constexpr int kSqRows = 64;

__device__ __forceinline__ void sq_pack_store(const uint32_t (&q)[8], int nbits, void* codes, uint64_t i, int d, int j0) {
    if (nbits == 8) {
        uint2 w;
        w.x = (q[0] & 0xFF) | (q[1] & 0xFF) << 8 | (q[2] & 0xFF) << 16 | (q[3] & 0xFF) << 24;
        w.y = (q[4] & 0xFF) | (q[5] & 0xFF) << 8 | (q[6] & 0xFF) << 16 | (q[7] & 0xFF) << 24;
        *reinterpret_cast<uint2*>(static_cast<uint8_t*>(codes) + i * (uint64_t)d + j0) = w;
    } else if (nbits == 16) {
        uint4 w;
        w.x = (q[0] & 0xFFFF) | q[1] << 16; w.y = (q[2] & 0xFFFF) | q[3] << 16;
        w.z = (q[4] & 0xFFFF) | q[5] << 16; w.w = (q[6] & 0xFFFF) | q[7] << 16;
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(codes) + i * (uint64_t)d + j0) = w;
    } else {  // (q[:,0::2] << 4) | q[:,1::2] in uint8 arithmetic
        uint32_t w = 0;
#pragma unroll
        for (int u = 0; u < 8; u += 2) w |= (uint32_t)(uint8_t)(((uint8_t)q[u] << 4) | (uint8_t)q[u + 1]) << (4 * u);
        *reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(codes) + i * (uint64_t)(d >> 1) + (j0 >> 1)) = w;
    }
}

__global__ __launch_bounds__(256) void sq_encode_f32_vec_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                const float* __restrict__ lo,
                                                                const float* __restrict__ den, int nbits,
                                                                void* __restrict__ codes) {
    const int g = blockIdx.x * 64 + (threadIdx.x & 63);
    if (g >= (d >> 3)) return;
    const int j0 = 8 * g;
    const float4 la = *reinterpret_cast<const float4*>(lo + j0), lb = *reinterpret_cast<const float4*>(lo + j0 + 4);
    const float4 da = *reinterpret_cast<const float4*>(den + j0), db = *reinterpret_cast<const float4*>(den + j0 + 4);
    const float lv[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
    const float dv[8] = {da.x, da.y, da.z, da.w, db.x, db.y, db.z, db.w};
    const float L = (float)((1 << nbits) - 1);
    float rv[8];
    bool okv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const float ad = fabsf(dv[u]);
        okv[u] = ad >= 0x1p-62f && ad <= 0x1p62f;
        rv[u] = __fdiv_rn(1.0f, dv[u]);
    }
    for (int64_t rbk = blockIdx.y; rbk * kSqRows < n; rbk += gridDim.y) {
    const int64_t r0 = rbk * kSqRows + (threadIdx.x >> 6);
    const int64_t r1 = min(n, (rbk + 1) * kSqRows);
#ifndef MIVQ_SQ_DEPTH  // rows per wave whose loads are in flight together
#define MIVQ_SQ_DEPTH 4  // 8: 3.75 vs 2.98 ms per 1M x 3072 (profiles/r04_s15)
#endif
    constexpr int SQD = MIVQ_SQ_DEPTH;
    for (int64_t i0 = r0; i0 < r1; i0 += 4 * SQD) {
        float4 xa[SQD], xb[SQD];
#pragma unroll
        for (int k = 0; k < SQD; ++k) {
            const int64_t i = i0 + 4 * k;
            if (i < r1) {
                const float4* xr = reinterpret_cast<const float4*>(x + i * (uint64_t)d + j0);
                xa[k] = xr[0];
                xb[k] = xr[1];
            }
        }
#pragma unroll
        for (int k = 0; k < SQD; ++k) {
            const int64_t i = i0 + 4 * k;
            if (i >= r1) break;
            const float xv[8] = {xa[k].x, xa[k].y, xa[k].z, xa[k].w, xb[k].x, xb[k].y, xb[k].z, xb[k].w};
            uint32_t q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                q[u] = np_cast_uint(rintf(__fmul_rn(div_rn_rcp(__fsub_rn(xv[u], lv[u]), dv[u], rv[u], okv[u]), L)));
            sq_pack_store(q, nbits, codes, (uint64_t)i, d, j0);
        }
    }
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

// Fast decode path (f32 out, d % 8 == 0, aligned): one lane per 8 dims, packed code load, two
// 16-B stores.
__global__ void sq_decode_f32_vec_kernel(const void* __restrict__ codes, int64_t n, int d, const float* __restrict__ lo,
                                         const float* __restrict__ den, int nbits, float* __restrict__ out) {
    const uint32_t groups = (uint32_t)(d >> 3);
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)n * groups) return;
    const uint64_t i = gid / groups;
    const int j0 = (int)(gid - i * groups) * 8;
    uint32_t lv[8];
    if (nbits == 8) {
        const uint2 w = *reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(codes) + i * (uint64_t)d + j0);
#pragma unroll
        for (int u = 0; u < 4; ++u) { lv[u] = (w.x >> (8 * u)) & 0xFF; lv[4 + u] = (w.y >> (8 * u)) & 0xFF; }
    } else if (nbits == 16) {
        const uint4 w = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(codes) + i * (uint64_t)d + j0);
        lv[0] = w.x & 0xFFFF; lv[1] = w.x >> 16; lv[2] = w.y & 0xFFFF; lv[3] = w.y >> 16;
        lv[4] = w.z & 0xFFFF; lv[5] = w.z >> 16; lv[6] = w.w & 0xFFFF; lv[7] = w.w >> 16;
    } else {  // high nibble = even dim
        const uint32_t w = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(codes) + i * (uint64_t)(d >> 1) + (j0 >> 1));
#pragma unroll
        for (int u = 0; u < 4; ++u) { const uint32_t b = (w >> (8 * u)) & 0xFF; lv[2 * u] = b >> 4; lv[2 * u + 1] = b & 0xF; }
    }
    const float L = (float)((1 << nbits) - 1);
    const float4* lr = reinterpret_cast<const float4*>(lo + j0);
    const float4* dr = reinterpret_cast<const float4*>(den + j0);
    const float4 la = lr[0], lb = lr[1], da = dr[0], db = dr[1];
    const float lov[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
    const float dnv[8] = {da.x, da.y, da.z, da.w, db.x, db.y, db.z, db.w};
    float o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = __fadd_rn(__fmul_rn(__fdiv_rn((float)lv[u], L), dnv[u]), lov[u]);
    float4* orow = reinterpret_cast<float4*>(out + i * (uint64_t)d + j0);
    orow[0] = make_float4(o[0], o[1], o[2], o[3]);
    orow[1] = make_float4(o[4], o[5], o[6], o[7]);
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
    if constexpr (sizeof(T) == 4) {
        const bool vec = (d % 8 == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(lo) |
                                           reinterpret_cast<uintptr_t>(den)) % 16 == 0) &&
                         (reinterpret_cast<uintptr_t>(codes) % 16 == 0);
        if (vec) {
            // grid.y is limited to 65535: blocks stride over the row blocks beyond that
            const int64_t rb = std::min<int64_t>(ceil_div(n, (int64_t)kSqRows), 65535);
            hipLaunchKernelGGL(sq_encode_f32_vec_kernel, dim3((unsigned)ceil_div(d / 8, 64), (unsigned)rb), dim3(256), 0,
                               as_stream(stream), x, n, d, lo, den, nbits, codes);
            return check_launch(name);
        }
    }
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
    if constexpr (sizeof(T) == 4) {
        const bool vec = (d % 8 == 0) && ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(lo) |
                                           reinterpret_cast<uintptr_t>(den) | reinterpret_cast<uintptr_t>(out)) % 16 == 0);
        if (vec) {
            hipLaunchKernelGGL(sq_decode_f32_vec_kernel, dim3((unsigned)ceil_div(n * (int64_t)(d / 8), 256)), dim3(256),
                               0, as_stream(stream), codes, n, d, lo, den, nbits, out);
            return check_launch(name);
        }
    }
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
