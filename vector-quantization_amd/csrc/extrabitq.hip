// extrabitq.hip — multi-bit ("Extended") RaBitQ encode / decode steps on gfx950.
//
// Restates ExtendedRaBitQuantizer.compress / decompress
// (/root/reference/src/haag_vq/methods/extended_rabitq.py:125-199), all in fp64 like numpy:
//   encode: r = x - c; nrm = ||r||; o = r / max(nrm, 1e-12)                 [normalize]
//           s = (o . P) * sqrt(D)   (the D x D product: erq_rotate_kernel, fp64 MFMA)
//           idx = searchsorted(mid-levels, s) (left); s_hat = levels[idx]
//           t = <s, s_hat> / <s_hat, s_hat>  (1 when the denominator <= 1e-12)
//           row = B-bit idx packed MSB-first (np.packbits) ++ f32 nrm ++ f32 t   [quantize]
//   decode: o_hat = (levels[idx] / sqrt(D)) * t                              [dequantize]
//           x_hat = f32((o_hat . P^T) * nrm + c)                             [finish]
// The two D x D rotations (o . P, o_hat . P^T; extended_rabitq.py:140,196) run on
// erq_rotate_kernel: v_mfma_f64_16x16x4_f64, 128 x 128 output tiles, K slices of 16 staged
// through LDS (double-buffered), fp64 accumulation (mivq_extrabitq_rotate).
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


// ---------------------------------------------------------------- fp64 rotation GEMM
// s = o . op(P) for the (n, d) row block o and the (d, d) matrix P: op(P) = P (transpose 0,
// encode: extended_rabitq.py:140) or P^T (transpose 1, decode: :196).  Workgroup: 256 threads,
// a 128 x 128 tile of s (4 waves of 64 x 64 = 4 x 4 blocks of v_mfma_f64_16x16x4_f64, 16
// accumulators of 4 doubles per lane), K in slices of 16 through two LDS stages.  Operand maps
// (cdna_hip_programming.md, f64 MFMA): A: lane l holds A[l & 15][l >> 4], B: B[l >> 4][l & 15],
// D: col = l & 15, row = (l >> 4) + 4 reg.  Every product is exact fp64 FMA accumulation
// (sum order: the MFMA's over k, slices ascending); rows past n / columns past d are masked.
constexpr int kRotT = 128, kRotK = 16;
constexpr int kRotAP = kRotK + 1;   // A stage row pitch (doubles): [row][k]
constexpr int kRotBP = kRotT + 1;   // B stage row pitch (doubles): [k][col]
typedef double f64x4 __attribute__((ext_vector_type(4)));

// Tile of workgroup b.  MIVQ_ERQ_XCD (default): the workgroups of one XCD (b % 8, dealt
// round-robin) take a contiguous range of tiles, so the column tiles of one 128-row block run
// side by side on one XCD and share its L2 copy of the o strip (3 MB at D = 3072); the round-3
// order (b itself) spread them over all eight XCDs, each fetching the strip again.
#ifndef MIVQ_ERQ_XCD
#define MIVQ_ERQ_XCD 1
#endif
#ifndef MIVQ_ERQ_SFIRST  // stage-first loop order in erq_rotate_fast_kernel (61.8 -> 58.6 ms, r04_s25)
#define MIVQ_ERQ_SFIRST 1
#endif
__device__ __forceinline__ int64_t erq_tile(int64_t b, int64_t G) {
    if (!MIVQ_ERQ_XCD) return b;
    const int64_t x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    return x * q + (x < r ? x : r) + j;
}

__global__ __launch_bounds__(256) void erq_rotate_kernel(const double* __restrict__ o, int64_t n, int d,
                                                         const double* __restrict__ P, int transpose,
                                                         double* __restrict__ s, int64_t ctiles) {
    __shared__ double As[2][kRotT * kRotAP];
    __shared__ double Bs[2][kRotK * kRotBP];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int64_t t = erq_tile(blockIdx.x, gridDim.x);
    const int64_t r0 = (t / ctiles) * kRotT;
    const int c0 = (int)(t % ctiles) * kRotT;
    const int wr = w >> 1, wc = w & 1;  // wave tile: rows wr*64.., cols wc*64..
    f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f64x4){0.0, 0.0, 0.0, 0.0};

    // staging: A slice = 128 rows x 16 k (each thread 8 doubles: row tid / 2, k 8 (tid & 1) ..);
    // B slice = 16 k x 128 cols (each thread 8 doubles)
    double ra[8], rb[8];
    auto gload = [&](int k0) __attribute__((always_inline)) {
        {
            const int rr = tid >> 1, kk = 8 * (tid & 1);
            const int64_t gr = r0 + rr;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                ra[u] = (gr < n && k0 + kk + u < d) ? o[gr * d + k0 + kk + u] : 0.0;
        }
        if (transpose == 0) {  // B[k][j] = P[k][j]: rows of P, 8 consecutive columns per thread
            const int kk = tid >> 4, jj = 8 * (tid & 15);
#pragma unroll
            for (int u = 0; u < 8; ++u)
                rb[u] = (k0 + kk < d && c0 + jj + u < d) ? P[(int64_t)(k0 + kk) * d + c0 + jj + u] : 0.0;
        } else {  // B[k][j] = P[j][k]: column j of op(P) is row j of P, 8 consecutive k per thread
            const int jj = tid >> 1, kk = 8 * (tid & 1);
#pragma unroll
            for (int u = 0; u < 8; ++u)
                rb[u] = (c0 + jj < d && k0 + kk + u < d) ? P[(int64_t)(c0 + jj) * d + k0 + kk + u] : 0.0;
        }
    };
    auto sstore = [&](int st) __attribute__((always_inline)) {
        {
            const int rr = tid >> 1, kk = 8 * (tid & 1);
#pragma unroll
            for (int u = 0; u < 8; ++u) As[st][rr * kRotAP + kk + u] = ra[u];
        }
        if (transpose == 0) {
            const int kk = tid >> 4, jj = 8 * (tid & 15);
#pragma unroll
            for (int u = 0; u < 8; ++u) Bs[st][kk * kRotBP + jj + u] = rb[u];
        } else {
            const int jj = tid >> 1, kk = 8 * (tid & 1);
#pragma unroll
            for (int u = 0; u < 8; ++u) Bs[st][(kk + u) * kRotBP + jj] = rb[u];
        }
    };
    const int nk = (d + kRotK - 1) / kRotK;
    gload(0);
    sstore(0);
    __syncthreads();
    const int fi = l & 15, fk = l >> 4;
    for (int ks = 0; ks < nk; ++ks) {
        const int st = ks & 1;
        if (ks + 1 < nk) gload((ks + 1) * kRotK);
#pragma unroll
        for (int k4 = 0; k4 < kRotK; k4 += 4) {
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) af[a] = As[st][(wr * 64 + a * 16 + fi) * kRotAP + k4 + fk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[st][(k4 + fk) * kRotBP + wc * 64 + b * 16 + fi];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        if (ks + 1 < nk) sstore(st ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t row = r0 + wr * 64 + a * 16 + fk + 4 * g;
                const int col = c0 + wc * 64 + b * 16 + fi;
                if (row < n && col < d) s[row * d + col] = acc[a][b][g];
            }
}

// d % 32 == 0 (every BASELINE width): the same tile, slices and MFMA order as erq_rotate_kernel
// (identical results), with the global side rebuilt: each thread's 8-double chunks are in or out
// of range as a whole, so they load as 16-B buffer loads (range-checked: rows past n read zeros,
// no branches), and the loads run TWO slices ahead through two register stages (slice ks + 2
// loads while slice ks computes; slice ks + 1, loaded a slice earlier, goes to LDS after it).
// The generic kernel's per-element guarded 8-B loads compiled to a branch per load and a
// vmcnt(0) in the middle of its loads.
typedef unsigned int erq_u32x4 __attribute__((ext_vector_type(4)));
template <int TR>
__global__ __launch_bounds__(256, 2) void erq_rotate_fast_kernel(const double* __restrict__ o, int64_t n, int d,
                                                              const double* __restrict__ P,
                                                              double* __restrict__ s, int64_t ctiles) {
    __shared__ double As[2][kRotT * kRotAP];
    __shared__ double Bs[2][kRotK * kRotBP];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int64_t t = erq_tile(blockIdx.x, gridDim.x);
    const int64_t r0 = (t / ctiles) * kRotT;
    const int c0 = (int)(t % ctiles) * kRotT;
    const int wr = w >> 1, wc = w & 1;
    f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f64x4){0.0, 0.0, 0.0, 0.0};
    constexpr int kOob = (int)0x80000000u;
    const int rows = (int)(n - r0 < kRotT ? n - r0 : kRotT);
    // o rows r0 .. r0 + rows of this tile (< 4 GiB: 128 rows); P whole (d^2 * 8 < 2^31 checked)
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc((void*)(o + r0 * d), 0, rows * d * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void*)P, 0, d * d * 8, 0x00020000);
    const int ar = tid >> 1, ak = 8 * (tid & 1);                        // A: row, k offset
    const int bk = TR ? 8 * (tid & 1) : tid >> 4, bj = TR ? tid >> 1 : 8 * (tid & 15);  // B
    auto gload = [&](int k0, double (&ra)[8], double (&rb)[8]) __attribute__((always_inline)) {
        const int va = k0 + ak < d ? (ar * d + k0 + ak) * 8 : kOob;
        const int vb = TR ? ((c0 + bj < d && k0 + bk < d) ? ((c0 + bj) * d + k0 + bk) * 8 : kOob)
                          : ((k0 + bk < d && c0 + bj < d) ? ((k0 + bk) * d + c0 + bj) * 8 : kOob);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const erq_u32x4 ua = __builtin_amdgcn_raw_buffer_load_b128(ors, va == kOob ? kOob : va + 16 * q, 0, 0);
            const erq_u32x4 ub = __builtin_amdgcn_raw_buffer_load_b128(prs, vb == kOob ? kOob : vb + 16 * q, 0, 0);
            ra[2 * q] = __hiloint2double((int)ua[1], (int)ua[0]);
            ra[2 * q + 1] = __hiloint2double((int)ua[3], (int)ua[2]);
            rb[2 * q] = __hiloint2double((int)ub[1], (int)ub[0]);
            rb[2 * q + 1] = __hiloint2double((int)ub[3], (int)ub[2]);
        }
    };
    auto sstore = [&](int st, const double (&ra)[8], const double (&rb)[8]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 8; ++u) As[st][ar * kRotAP + ak + u] = ra[u];
        if (TR) {
#pragma unroll
            for (int u = 0; u < 8; ++u) Bs[st][(bk + u) * kRotBP + bj] = rb[u];
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) Bs[st][bk * kRotBP + bj + u] = rb[u];
        }
    };
    const int fi = l & 15, fk = l >> 4;
    auto slice = [&](int st) __attribute__((always_inline)) {
#pragma unroll
        for (int k4 = 0; k4 < kRotK; k4 += 4) {
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) af[a] = As[st][(wr * 64 + a * 16 + fi) * kRotAP + k4 + fk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[st][(k4 + fk) * kRotBP + wc * 64 + b * 16 + fi];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
    };
    const int nk = (d + kRotK - 1) / kRotK;
    double ra0[8], rb0[8], ra1[8], rb1[8];
    gload(0, ra0, rb0);
    gload(kRotK, ra1, rb1);
    sstore(0, ra0, rb0);
    if (MIVQ_ERQ_SFIRST) {
        // stage first: each half-trip stores the next slice (loaded a half-trip and more ago)
        // BEFORE its MFMAs, then issues the loads of the slice three ahead into the freed stage
        gload(2 * kRotK, ra0, rb0);
        __syncthreads();
        for (int ks = 0; ks < nk; ks += 2) {
            sstore(1, ra1, rb1);                 // slice ks + 1
            gload((ks + 3) * kRotK, ra1, rb1);
            slice(0);                            // slice ks
            __syncthreads();
            sstore(0, ra0, rb0);                 // slice ks + 2 (past nk: zeros, never read)
            gload((ks + 4) * kRotK, ra0, rb0);
            slice(1);                            // slice ks + 1
            __syncthreads();
        }
    } else {
    __syncthreads();
    // two slices per trip (nk is even: d % 32 == 0) so the register stages stay static and no
    // branch splits the loop: slice ks computes from LDS stage 0 while slice ks + 2 loads into
    // the stage slice ks came from; loads past d read zeros, and the last trip's stores of them
    // into stage 0 are never read
    for (int ks = 0; ks < nk; ks += 2) {
        gload((ks + 2) * kRotK, ra0, rb0);
        slice(0);
        sstore(1, ra1, rb1);
        __syncthreads();
        gload((ks + 3) * kRotK, ra1, rb1);
        slice(1);
        sstore(0, ra0, rb0);
        __syncthreads();
    }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t row = r0 + wr * 64 + a * 16 + fk + 4 * g;
                const int col = c0 + wc * 64 + b * 16 + fi;
                if (row < n && col < d) s[row * d + col] = acc[a][b][g];
            }
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

extern "C" int mivq_extrabitq_rotate(const double* o, int64_t n, int32_t d, const double* P, int32_t transpose,
                                     double* s, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "extrabitq_rotate: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(transpose == 0 || transpose == 1, MIVQ_ERR_INVALID, "extrabitq_rotate: transpose must be 0 or 1");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(o && P && s && o != s, MIVQ_ERR_INVALID, "extrabitq_rotate: null or aliased pointer");
    const int64_t ct = ceil_div(d, kRotT), tiles = ceil_div(n, kRotT) * ct;
    MIVQ_REQUIRE(tiles < ((int64_t)1 << 31), MIVQ_ERR_UNSUPPORTED, "extrabitq_rotate: n=%lld too large", (long long)n);
#ifndef MIVQ_ERQ_FAST
#define MIVQ_ERQ_FAST 1
#endif
    // the fast kernel's buffer offsets are 32-bit: d^2 * 8 bytes of P and 128 rows of o
    if (MIVQ_ERQ_FAST && d % 32 == 0 && (int64_t)d * d * 8 < ((int64_t)1 << 31)) {
        if (transpose)
            hipLaunchKernelGGL(erq_rotate_fast_kernel<1>, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), o, n, d,
                               P, s, ct);
        else
            hipLaunchKernelGGL(erq_rotate_fast_kernel<0>, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), o, n, d,
                               P, s, ct);
    } else {
        hipLaunchKernelGGL(erq_rotate_kernel, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), o, n, d, P,
                           transpose, s, ct);
    }
    return check_launch("extrabitq_rotate");
}
