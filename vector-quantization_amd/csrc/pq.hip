// pq.hip — product-quantizer encode / decode / prepare / k-means update for gfx950.
//
// Replaces faiss.ProductQuantizer.compute_codes / decode / train behind
// ProductQuantizer.compress / decompress / fit (/root/reference/src/haag_vq/methods/
// product_quantization.py:58-86).  The canonical arithmetic (what "bit-exact" means) is
// spelled out in include/mivq.h and oracle/mivq_oracle.c:
//     score_k = fl(cn_k - 2 * dot_k),  dot_k / cn_k = sequential fmaf chains over t,
//     code    = smallest k with the minimum score.
//
// Two encode engines:
//   * pq_encode_exact  — any shape: one lane per row, centroids broadcast through the
//     scalar cache, KG independent canonical chains per lane.  Bit-exact by construction.
//   * pq_encode_mfma   — ksub == 256, dsub % 4 == 0, dsub <= 128: an fp16 MFMA
//     (v_mfma_f32_32x32x16_f16) computes approximate scores for 32 rows x 32 centroids per
//     instruction; every (row, subspace) keeps its top-3 approximate scores, and the
//     candidates inside a rigorous error window (derived below) are re-scored with the
//     canonical fp32 chain.  1 candidate: done; 2: exact re-check in the same kernel; >= 3
//     (or fp16 overflow): flagged and settled by pq_resolve with the exact scan.  Codes
//     are therefore identical to the canonical (oracle) codes, not "mostly".
#include "mivq_common.h"
#include "pq_internal.h"

#include <math.h>

namespace mivq {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------ prepare
// One thread per (m, k): canonical norm (sequential fmaf chain), transposed copy.
__global__ void pq_prep_norms_kernel(const float* __restrict__ C, int M, int ksub, int dsub,
                                     float* __restrict__ cn, float* __restrict__ ct) {
    const int64_t mk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (mk >= (int64_t)M * ksub) return;
    const int m = (int)(mk / ksub), k = (int)(mk % ksub);
    const float* c = C + mk * dsub;
    float acc = 0.0f;
    for (int t = 0; t < dsub; ++t) {
        const float v = c[t];
        acc = __builtin_fmaf(v, v, acc);
        ct[((int64_t)m * dsub + t) * ksub + k] = v;
    }
    cn[mk] = acc;
}

// Unit roundoffs used by the filter error bound.
constexpr float kU32 = 5.9604645e-8f;    // 2^-24
constexpr float kUh = 4.8828125e-4f;     // 2^-11: f32 -> f16 round-to-nearest-even
// |error| of an f16 subnormal result: <= 2^-25 (round to nearest; the kernels are built with
// f16 denormals preserved, .amdhsa_float_denorm_mode_16_64 = 3), taken as 2^-24.
constexpr float kEta = 5.9604645e-8f;    // 2^-24
constexpr float kPack = 3.0517578e-5f;   // 2^-15: 8 low mantissa bits replaced by the index
constexpr int kScaleC = 14;              // max |c~| <= 2^14
constexpr int kScaleX = 12;              // |x~| < 65504 while |x| < 2^4 * 2^ceil(log2 max|c|)

// Scale exponent of subspace m: e = ceil(log2 max|c|) (clamped), tau = 2^(kScaleC - e),
// sigma = 2^(kScaleX - e) (or 1, see pq_prep_mfma_kernel).  Block-wide (256 threads); `red` is
// 256 floats of LDS.
__device__ int subspace_scale_exp(const float* Cm, int dsub, float* red) {
    const int tid = threadIdx.x;
    float mabs = 0.0f;
    for (int t = 0; t < dsub; ++t) mabs = fmaxf(mabs, fabsf(Cm[(int64_t)tid * dsub + t]));
    red[tid] = mabs;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
        __syncthreads();
    }
    const float cmax_abs = red[0];
    __syncthreads();
    int e = 0;
    if (cmax_abs > 0.0f && isfinite(cmax_abs)) e = (int)ceilf(log2f(cmax_abs));
    return max(-100, min(100, e));
}

// Pairwise spreads of the prepared image of subspace m (the window derivation above
// pq_encode_mfma_kernel):  Dmax = max_ij ||c~_i - c~_j||,  DDmax = max_ij ||dc_i - dc_j||,
// c~ = f16(tau c), dc = c~ - tau c (exact in fp32).  Grid (M, 16): block (m, g) takes rows
// i in [16g, 16g + 16) against all 256 j (the image staged in LDS by 32-dimension chunks),
// one fp32 chain per pair (relative rounding of a
// squared sum <= (dsub + 3) 2^-24, covered by the (1 + 1e-5) applied to the norms); the
// maxima of the squared sums go to spread[m] with atomicMax on their bits (non-negative).
constexpr int kSpreadTC = 32;  // dimensions per LDS chunk of the spread kernel

__global__ __launch_bounds__(256) void pq_prep_spread_kernel(const float* __restrict__ C, int dsub,
                                                             uint32_t* __restrict__ spread, float2* __restrict__ pd) {
    // the image of all 256 centroids for kSpreadTC dimensions at a time: (c~, c~ - tau c) per
    // element, rows padded to an odd number of float2 (the 16 j rows a lane group reads sit on
    // distinct banks)
    __shared__ float2 img[256][kSpreadTC + 1];
    __shared__ float red[256];
    const int m = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
    const float* Cm = C + (int64_t)m * 256 * dsub;
    const float tau = ldexpf(1.0f, kScaleC - subspace_scale_exp(Cm, dsub, red));
    const int il = 16 * g + (tid >> 4), jl = tid & 15;
    float s1[16], s2[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) s1[jj] = s2[jj] = 0.0f;
    for (int t0 = 0; t0 < dsub; t0 += kSpreadTC) {
        const int tc = min(kSpreadTC, dsub - t0);
        __syncthreads();
        for (int e = tid; e < 256 * kSpreadTC; e += 256) {
            const int k = e / kSpreadTC, t = e - k * kSpreadTC;
            if (t < tc) {
                const float ti = tau * Cm[(int64_t)k * dsub + t0 + t];
                const float hi = (float)(_Float16)ti;
                img[k][t] = make_float2(hi, hi - ti);
            }
        }
        __syncthreads();
        for (int t = 0; t < tc; ++t) {
            const float2 a = img[il][t];
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const float2 b = img[16 * jj + jl][t];
                const float dh = a.x - b.x, dc = a.y - b.y;
                s1[jj] = __builtin_fmaf(dh, dh, s1[jj]);
                s2[jj] = __builtin_fmaf(dc, dc, s2[jj]);
            }
        }
    }
    // NaN pairs (a NaN centroid never wins, and its filter score is never a candidate) are
    // skipped by fmaxf; inf gives inf -> the window is infinite
    float d1 = 0.0f, d2 = 0.0f;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        d1 = fmaxf(d1, s1[jj]);
        d2 = fmaxf(d2, s2[jj]);
        if (pd)  // the pair's own spreads (NaN stays NaN: the pair window then never settles it)
            pd[((int64_t)m * 256 + il) * 256 + 16 * jj + jl] =
                make_float2(sqrtf(s1[jj]) * (1.0f + 1e-5f), sqrtf(s2[jj]) * (1.0f + 1e-5f));
    }
    atomicMax(&spread[2 * m + 0], __float_as_uint(d1));
    atomicMax(&spread[2 * m + 1], __float_as_uint(d2));
}

// One block (256 threads) per subspace m: scales, the f16 operand image, the scaled
// accumulator init and the bound constants.  See the derivation at pq_encode_mfma.
__global__ void pq_prep_mfma_kernel(const float* __restrict__ C, const float* __restrict__ cn,
                                    int M, int dsub, int KS, half8* __restrict__ img,
                                    float* __restrict__ hinit, float4* __restrict__ bnd,
                                    const uint32_t* __restrict__ spread, float4* __restrict__ bnd2) {
    const int m = blockIdx.x;
    const int tid = threadIdx.x;  // 256 threads
    __shared__ float red_nrm[256];
    const float* Cm = C + (int64_t)m * 256 * dsub;
    const int e = subspace_scale_exp(Cm, dsub, red_nrm);
    // max ||c||^2 over the subspace
    red_nrm[tid] = cn[(int64_t)m * 256 + tid];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red_nrm[tid] = fmaxf(red_nrm[tid], red_nrm[tid + s]);
        __syncthreads();
    }
    const float cn_max = red_nrm[0];
    const float tau = ldexpf(1.0f, kScaleC - e);  // c~ = f16(tau * c)
    // x~ = f16(sigma * x).  sigma = 1 (no scaling multiply in the encode kernels) whenever the
    // codebook's magnitude is ordinary; otherwise the power of two that puts sigma x in the f16
    // range next to c~.  f16 subnormals of x~ cost at most 2^-25 each (kEta).
    const float sigma = (e >= -8 && e <= 8) ? 1.0f : ldexpf(1.0f, kScaleX - e);
    const float st = sigma * tau;
    // operand image: fragment (cb, ks), lane l holds c~[cb*32 + (l&31)][t(ks, l>>5, j)]
    //   t(ks, h, j) = h*8*KS + 8*ks + j   (zero when t >= dsub)
    const int frag_elems = 8 * KS * 64;  // fragments * lanes
    for (int f = tid; f < frag_elems; f += 256) {
        const int l = f & 63;
        const int fk = f >> 6;           // cb * KS + ks
        const int cb = fk / KS, ks = fk % KS;
        const int k = cb * 32 + (l & 31), h = l >> 5;
        half8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = h * 8 * KS + 8 * ks + j;
            v[j] = (_Float16)(t < dsub ? tau * Cm[(int64_t)k * dsub + t] : 0.0f);
        }
        img[(int64_t)m * frag_elems + f] = v;
    }
    // accumulator init: -(cn/2) * sigma * tau  (exact: powers of two)
    hinit[(int64_t)m * 256 + tid] = -0.5f * cn[(int64_t)m * 256 + tid] * st;
    if (tid == 0) {
        // Window W(Xs) = a * Xs + b in accumulator units; Xs = sigma * ||x_m||, Cs = tau * Cmax,
        // Hs = sigma * tau * Cmax^2 >= 2 |accumulator init| (the terms that scale with ||c||^2:
        // rounding of cn and of the accumulation of the init, the canonical cn chain, the packed
        // index bits).
        const float Cs = tau * sqrtf(cn_max) * (1.0f + 1e-6f);
        const float Hs = st * cn_max * (1.0f + 1e-6f);
        const float Dm = sqrtf(__uint_as_float(spread[2 * m + 0])) * (1.0f + 1e-5f);
        const float DDm = sqrtf(__uint_as_float(spread[2 * m + 1])) * (1.0f + 1e-5f);
        const float gd = (float)dsub * kU32 / (1.0f - (float)dsub * kU32);
        const float gn = (float)(dsub + 2) * kU32 / (1.0f - (float)(dsub + 2) * kU32);
        const float sq = sqrtf((float)dsub);
        const float a_rest = Cs * (2.004f * gn + 2.004f * kPack + 2.0f * (gd + kU32));
        const float b_rest = Hs * (gn + 2.0f * gd + kPack + kU32);
        const float eta1 = 1.001f * kEta * sq;
        const float a = kUh * Dm + DDm + a_rest;
        const float b = eta1 * Dm + b_rest;
        const bool ok = isfinite(Cs) && isfinite(Hs) && isfinite(a) && isfinite(b) && isfinite(Dm) && isfinite(DDm);
        bnd[m] = make_float4(sigma, ok ? a * 1.0625f : INFINITY, ok ? b * 1.0625f + 1e-30f : INFINITY, tau);
        // the pair window W12 = 1.0625 ((u_h Xs + eta') D_12 + Xs DD_12 + a_rest Xs + b_rest)
        bnd2[m] = make_float4(ok ? a_rest : INFINITY, ok ? b_rest : INFINITY, eta1, 0.0f);
    }
}

// ------------------------------------------------------------------------ exact encode
// grid (ceil(n/64), M), block 64 (one wave): lane = row.  The row's subvector is staged in
// LDS (coalesced load, padded stride); centroid values are wave-uniform, so they come
// through scalar loads from the transposed codebook ct[m][t][k..k+KG).
template <int KG>
__global__ __launch_bounds__(64) void pq_encode_exact_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int ksub, int dsub,
    const float* __restrict__ ct, const float* __restrict__ cn, uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [64][dsub + 1]
    const int lane = threadIdx.x;
    const int m = blockIdx.y;
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    const int stride = dsub + 1;
    for (int e = lane; e < 64 * dsub; e += 64) {
        const int rr = e / dsub, t = e % dsub;
        const int64_t row = r0 + rr;
        xs[rr * stride + t] = row < n ? x[row * d + (int64_t)m * dsub + t] : 0.0f;
    }
    __syncthreads();
    const float* xr = xs + lane * stride;
    const float* ctm = ct + (int64_t)m * dsub * ksub;
    const float* cnm = cn + (int64_t)m * ksub;
    float best = INFINITY;
    int bi = 0;
    for (int k0 = 0; k0 < ksub; k0 += KG) {
        float acc[KG];
#pragma unroll
        for (int j = 0; j < KG; ++j) acc[j] = 0.0f;
#pragma unroll 4
        for (int t = 0; t < dsub; ++t) {
            const float xv = xr[t];
            const float* crow = ctm + (int64_t)t * ksub + k0;
#pragma unroll
            for (int j = 0; j < KG; ++j) acc[j] = __builtin_fmaf(xv, crow[j], acc[j]);
        }
#pragma unroll
        for (int j = 0; j < KG; ++j) {
            const float s = __builtin_fmaf(-2.0f, acc[j], cnm[k0 + j]);
            if (s < best) { best = s; bi = k0 + j; }
        }
    }
    const int64_t row = r0 + lane;
    if (row < n) out[row * M + m] = (uint8_t)bi;
}

// ------------------------------------------------------------------ tiled exact encode
// The exact path for subspaces the MFMA filter does not take (dsub > 192, or a forced exact
// assignment), ksub = 256, dsub % 4 == 0.  A VALU register-blocked GEMM: grid
// (ceil(n/128), M), block 256; thread (rg = tid >> 4, cg = tid & 15) owns rows rg*8 .. +8
// and centroids {64 q + 4 cg + i : q, i < 4}, 128 fp32 accumulators (scalar v_fma_f32: round 3
// ran them as v_pk_fma_f32 pairs, but packed fp32 math must not read LDS-loaded registers,
// DESIGN.md §8).  Each accumulator is still ONE fma chain over t = 0, 1, ..., dsub-1 from
// 0.0f, then s = fma(-2, acc, cn[k]) -- the canonical score, so codes are bit-exact.  dsub is
// walked in chunks of kXT dims: x chunk transposed to xs[t][row] (rows as b128 broadcasts),
// codebook chunk cs[t][k] from the transposed codebook ct (conflict-free b128 reads).
// Argmin: lexicographic (score, k) within the thread, then across the 16 cg lanes by xor
// shuffles -- the same winner as a strict-< scan in ascending k (NaN never wins, ties go to
// the lower index, all non-finite-or-+inf rows give 0).
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kXT = 32;          // dims per chunk
constexpr int kXRows = 128;      // rows per block
constexpr int kXsStride = kXRows + 4;
__global__ __launch_bounds__(256, 2) void pq_encode_exact_tiled_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub, const float* __restrict__ ct,
    const float* __restrict__ cn, uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float xs[kXT * kXsStride];
    __shared__ __attribute__((aligned(16))) float cs[kXT * 256];
    const int tid = threadIdx.x;
    const int rg = tid >> 4, cg = tid & 15;
    const int m = blockIdx.y;
    const int64_t r0 = (int64_t)blockIdx.x * kXRows;
    const float* ctm = ct + (int64_t)m * dsub * 256;
    float acc[8][16];  // scalar chains: no packed fp32 on LDS-loaded registers
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[r][j] = 0.0f;
    for (int t0 = 0; t0 < dsub; t0 += kXT) {
        const int tl = min(kXT, dsub - t0);  // multiple of 4
        __syncthreads();
        // x chunk: 128 rows x tl dims, float4 per thread-step (8 lanes per row segment)
        for (int e = tid; e < kXRows * (kXT / 4); e += 256) {
            const int rr = e >> 3, tq = e & 7;
            const int64_t row = r0 + rr;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (row < n && tq * 4 < tl)
                v = *reinterpret_cast<const float4*>(x + row * d + (int64_t)m * dsub + t0 + tq * 4);
            xs[(tq * 4 + 0) * kXsStride + rr] = v.x;
            xs[(tq * 4 + 1) * kXsStride + rr] = v.y;
            xs[(tq * 4 + 2) * kXsStride + rr] = v.z;
            xs[(tq * 4 + 3) * kXsStride + rr] = v.w;
        }
        for (int e = tid; e < tl * 64; e += 256) {
            const int tt = e >> 6, kq = e & 63;
            *reinterpret_cast<float4*>(cs + tt * 256 + kq * 4) =
                *reinterpret_cast<const float4*>(ctm + (int64_t)(t0 + tt) * 256 + kq * 4);
        }
        __syncthreads();
#pragma unroll 2
        for (int t = 0; t < tl; ++t) {
            const float4 xa = *reinterpret_cast<const float4*>(xs + t * kXsStride + rg * 8);
            const float4 xb = *reinterpret_cast<const float4*>(xs + t * kXsStride + rg * 8 + 4);
            const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
            float c1[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 c = *reinterpret_cast<const float4*>(cs + t * 256 + q * 64 + cg * 4);
                c1[4 * q] = c.x; c1[4 * q + 1] = c.y; c1[4 * q + 2] = c.z; c1[4 * q + 3] = c.w;
            }
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int j = 0; j < 16; ++j) acc[r][j] = __builtin_fmaf(xv[r], c1[j], acc[r][j]);
        }
    }
    const float* cnm = cn + (int64_t)m * 256;
    float cnv[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 c = *reinterpret_cast<const float4*>(cnm + q * 64 + cg * 4);
        cnv[4 * q] = c.x; cnv[4 * q + 1] = c.y; cnv[4 * q + 2] = c.z; cnv[4 * q + 3] = c.w;
    }
    int mine = 0;  // the code of row rg*8 + cg (cg < 8)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        float best = INFINITY;
        int bi = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float s = __builtin_fmaf(-2.0f, acc[r][j], cnv[j]);
            const int k = (j >> 2) * 64 + cg * 4 + (j & 3);
            if (s < best) { best = s; bi = k; }  // k ascends within the thread
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const float ob = __shfl_xor(best, off, 16);
            const int oi = __shfl_xor(bi, off, 16);
            if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (cg == r) mine = bi;
    }
    const int64_t row = r0 + rg * 8 + cg;
    if (cg < 8 && row < n) out[row * M + m] = (uint8_t)mine;
}

// ------------------------------------------------------------------------- MFMA encode
// Error window (all in accumulator units, i.e. scaled by sigma*tau; a_k = <x,c_k> - |c_k|^2/2
// is maximised, Xs >= sigma*||x_m||, Cs = tau*max_k ||c_k||, x~ = f16(sigma x), c~_k = f16(tau c_k),
// dx = x~ - sigma x, dc_k = c~_k - tau c_k).  For the canonical winner k* and any k, the
// f16 rounding enters the DIFFERENCE of the two filter scores only as
//     <dx, c~_k - c~_k*> + <sigma x, dc_k - dc_k*>  <=  ||dx|| Dmax + Xs DDmax,
//     ||dx|| <= u_h Xs + eta sqrt(dsub)   (f16 rounding, denormals/flush),
// with Dmax = max_ij ||c~_i - c~_j|| and DDmax = max_ij ||dc_i - dc_j|| measured on the
// prepared image (pq_prep_mfma_kernel).  Per score, on top of that:
//   E' = g_{dsub+2} (Hs/2 + 1.002 Xs Cs) + g_dsub Hs/2 + 2^-15 (Hs/2 + 1.002 Xs Cs)
//     (fp32 accumulation in any order, rounding of cn, the 8 index bits packed into the mantissa)
//   canonical  |st*A_k - st*a_k| <= G/2 with G = (g_dsub + u) (Hs + 2 Xs Cs)
//   (Hs = sigma tau Cmax^2 bounds twice the accumulator init |cn| sigma tau / 2)
//   => p_{k*} >= p_max - (||dx|| Dmax + Xs DDmax + 2E' + G).
// W = a*Xs + b (pq_prep_mfma_kernel) includes a 1.0625 safety factor.
constexpr int kWaves = 8;  // 512 threads: 2 waves per SIMD, 256 rows per workgroup

__device__ __forceinline__ void top3_insert(float& t1, float& t2, float& t3, float v) {
    const float n1 = fmaxf(t1, v);
    const float n2 = __builtin_amdgcn_fmed3f(t1, t2, v);
    const float n3 = __builtin_amdgcn_fmed3f(t2, t3, v);
    t1 = n1; t2 = n2; t3 = n3;
}

__device__ __forceinline__ float pack_idx(float v, uint32_t k) {
    return __uint_as_float((__float_as_uint(v) & 0xFFFFFF00u) | k);
}

template <int KS>
struct MfmaSmem {
    static constexpr int kFrag = 8 * KS * 64;  // half8 per subspace image
};

template <int KS>
__global__ __launch_bounds__(512, 2) void pq_encode_mfma_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub,
    const float* __restrict__ C, const float* __restrict__ cn, const half8* __restrict__ img,
    const float* __restrict__ hinit, const float4* __restrict__ bnd, uint8_t* __restrict__ codes,
    uint32_t* __restrict__ flags) {
    constexpr int FR = MfmaSmem<KS>::kFrag;
    constexpr int HALF = 8 * KS;  // floats per lane-half of a subvector
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    half8* cbuf = reinterpret_cast<half8*>(smem);                       // [2][FR]
    float* hbuf = reinterpret_cast<float*>(smem + 2 * FR * 16);          // [2][256]
    uint8_t* cstage = smem + 2 * FR * 16 + 2 * 256 * 4;                  // [256][M]

    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63;
    const int r = l & 31, h = l >> 5;
    const int64_t r0 = (int64_t)blockIdx.x * (kWaves * 32);
    const int64_t row = r0 + w * 32 + r;
    const bool row_ok = row < n;
    const float* xrow = x + (row_ok ? row : 0) * (int64_t)d;

    // number of valid float4 chunks of this lane's half-subvector
    const int h_begin = h * HALF;
    const int nchunk = max(0, min(HALF, dsub - h_begin)) >> 2;

    float4 xc[HALF / 4];  // raw f32 of the current subspace
    float4 xn_[HALF / 4]; // prefetched next subspace
    auto load_x = [&](int m, float4* dst) {
#pragma unroll
        for (int i = 0; i < HALF / 4; ++i) {
            if (row_ok && i < nchunk)
                dst[i] = *reinterpret_cast<const float4*>(xrow + (int64_t)m * dsub + h_begin + 4 * i);
            else
                dst[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    // codebook image staging: FR half8 per subspace, 512 threads
    constexpr int CPT = (FR + 511) / 512;
    half8 cn_reg[CPT];
    float4 hn_reg;
    auto load_cb = [&](int m) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int f = tid + i * 512;
            if (f < FR) cn_reg[i] = img[(int64_t)m * FR + f];
        }
        if (tid < 64) hn_reg = reinterpret_cast<const float4*>(hinit + (int64_t)m * 256)[tid];
    };
    auto store_cb = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int f = tid + i * 512;
            if (f < FR) cbuf[buf * FR + f] = cn_reg[i];
        }
        if (tid < 64) reinterpret_cast<float4*>(hbuf + buf * 256)[tid] = hn_reg;
    };

    load_cb(0);
    load_x(0, xc);
    store_cb(0);
    __syncthreads();

    for (int m = 0; m < M; ++m) {
        const int buf = m & 1;
        const bool has_next = (m + 1) < M;
        if (has_next) {
            load_cb(m + 1);
            load_x(m + 1, xn_);
        }
        const float4 bm = bnd[m];
        const float sigma = bm.x;
        // B fragments (f16) + fp32 squared norm of this half
        half8 bf[KS];
        float xx = 0.0f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const float4 a = xc[2 * ks], b = xc[2 * ks + 1];
            xx = __builtin_fmaf(a.x, a.x, xx); xx = __builtin_fmaf(a.y, a.y, xx);
            xx = __builtin_fmaf(a.z, a.z, xx); xx = __builtin_fmaf(a.w, a.w, xx);
            xx = __builtin_fmaf(b.x, b.x, xx); xx = __builtin_fmaf(b.y, b.y, xx);
            xx = __builtin_fmaf(b.z, b.z, xx); xx = __builtin_fmaf(b.w, b.w, xx);
            half8 v;
            v[0] = (_Float16)(sigma * a.x); v[1] = (_Float16)(sigma * a.y);
            v[2] = (_Float16)(sigma * a.z); v[3] = (_Float16)(sigma * a.w);
            v[4] = (_Float16)(sigma * b.x); v[5] = (_Float16)(sigma * b.y);
            v[6] = (_Float16)(sigma * b.z); v[7] = (_Float16)(sigma * b.w);
            bf[ks] = v;
        }
        xx += __shfl_xor(xx, 32);
        float t1 = -INFINITY, t2 = -INFINITY, t3 = -INFINITY;
        const half8* cb_img = cbuf + buf * FR;
        const float* hb = hbuf + buf * 256;
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
            floatx16 acc;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 hv = *reinterpret_cast<const float4*>(hb + cb * 32 + 8 * q + 4 * h);
                acc[4 * q + 0] = hv.x; acc[4 * q + 1] = hv.y;
                acc[4 * q + 2] = hv.z; acc[4 * q + 3] = hv.w;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const half8 a = cb_img[(cb * KS + ks) * 64 + l];
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bf[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i)
                top3_insert(t1, t2, t3, pack_idx(acc[i], (uint32_t)(cb * 32 + (i & 3) + 8 * (i >> 2))));
        }
        // restore the lane half in bit 2 of the index, then merge with the partner lane
        const uint32_t hbit = (uint32_t)h << 2;
        t1 = __uint_as_float(__float_as_uint(t1) | hbit);
        t2 = __uint_as_float(__float_as_uint(t2) | hbit);
        t3 = __uint_as_float(__float_as_uint(t3) | hbit);
        {
            const float p1 = __shfl_xor(t1, 32), p2 = __shfl_xor(t2, 32), p3 = __shfl_xor(t3, 32);
            top3_insert(t1, t2, t3, p1);
            top3_insert(t1, t2, t3, p2);
            top3_insert(t1, t2, t3, p3);
        }
        const float xn = sqrtf(xx) * (1.0f + 1e-5f);
        const float Xs = sigma * xn;
        const float W = bm.y * Xs + bm.z;
        const float thr = t1 - W;
        // fp16 overflow guard: |x~_t| <= sigma*||x|| < 65504 keeps every operand finite
        const bool bad = !(Xs < 65000.0f) || !isfinite(t1) || !isfinite(W);
        const int ncand = bad ? 3 : 1 + (t2 >= thr) + (t3 >= thr);
        const int k1 = (int)(__float_as_uint(t1) & 0xFFu);
        const int k2 = (int)(__float_as_uint(t2) & 0xFFu);
        int code = k1;
        // exact re-check of two candidates: canonical chain split across the lane pair
        // (lane h=0 owns t in [0, HALF), lane h=1 owns [HALF, 2*HALF)), pipelined so the two
        // chains share three passes over HALF steps.
        if (__any(ncand == 2)) {
            const bool need = (ncand == 2);
            const float* Cm = C + (int64_t)m * 256 * dsub;
            float carry = 0.0f;  // chain value handed from h=0 to h=1
            float dot1 = 0.0f, dot2 = 0.0f;
#pragma unroll
            for (int phase = 0; phase < 3; ++phase) {
                // phase 0: h0 runs k1 first half; phase 1: h0 runs k2 first half, h1 runs k1
                // second half; phase 2: h1 runs k2 second half.
                const bool active = need && ((h == 0 && phase < 2) || (h == 1 && phase > 0));
                const int kk = (h == 0) ? (phase == 0 ? k1 : k2) : (phase == 1 ? k1 : k2);
                float acc = (h == 0) ? 0.0f : carry;
                if (active) {
                    const float* crow = Cm + (int64_t)kk * dsub + h_begin;
#pragma unroll
                    for (int i = 0; i < HALF / 4; ++i) {
                        if (i < nchunk) {
                            const float4 cv = *reinterpret_cast<const float4*>(crow + 4 * i);
                            const float4 xv = xc[i];
                            acc = __builtin_fmaf(xv.x, cv.x, acc);
                            acc = __builtin_fmaf(xv.y, cv.y, acc);
                            acc = __builtin_fmaf(xv.z, cv.z, acc);
                            acc = __builtin_fmaf(xv.w, cv.w, acc);
                        }
                    }
                }
                const float other = __shfl_xor(acc, 32);
                if (h == 1) {
                    carry = other;  // the h=0 partial of this phase feeds the next phase
                    if (phase == 1) dot1 = acc;
                    if (phase == 2) dot2 = acc;
                }
            }
            if (need && h == 1) {
                const float* cnm = cn + (int64_t)m * 256;
                const float s1 = __builtin_fmaf(-2.0f, dot1, cnm[k1]);
                const float s2 = __builtin_fmaf(-2.0f, dot2, cnm[k2]);
                code = (s2 < s1 || (s2 == s1 && k2 < k1)) ? k2 : k1;
            }
            code = __shfl(code, (l & 31) + 32);  // h=1 lane holds the answer
        }
        const unsigned long long fb = __ballot(ncand >= 3);
        if (h == 0) cstage[(w * 32 + r) * M + m] = (uint8_t)code;
        if (l == 0) {
            const int64_t vb = r0 / 32 + w;
            if (vb * 32 < n) flags[vb * M + m] = (uint32_t)(fb & 0xFFFFFFFFull);
        }
        if (has_next) {
            store_cb(buf ^ 1);
#pragma unroll
            for (int i = 0; i < HALF / 4; ++i) xc[i] = xn_[i];
        }
        __syncthreads();
    }
    // coalesced copy of the staged code rows
    const int64_t rows = min((int64_t)(kWaves * 32), n - r0);
    const int64_t bytes = rows * M;
    uint8_t* dst = codes + r0 * M;
    for (int64_t e = tid; e < bytes; e += 512) dst[e] = cstage[e];
}

// Settles the (row, subspace) pairs the filter flagged: one block (256 threads = one lane per
// centroid) runs the canonical chain for every centroid and takes the first minimum.
__global__ __launch_bounds__(256) void pq_resolve_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub, const float* __restrict__ ct,
    const float* __restrict__ cn, const uint32_t* __restrict__ flags, int64_t nwords,
    uint8_t* __restrict__ codes) {
    extern __shared__ __attribute__((aligned(16))) float xsub[];  // [dsub]
    __shared__ float rkey[256];
    __shared__ int ridx[256];
    const int tid = threadIdx.x;
    for (int64_t wd = blockIdx.x; wd < nwords; wd += gridDim.x) {
        uint32_t bits = flags[wd];
        if (bits == 0) continue;
        const int64_t vb = wd / M;
        const int m = (int)(wd % M);
        while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1;
            const int64_t row = vb * 32 + b;
            if (row >= n) continue;
            __syncthreads();
            for (int t = tid; t < dsub; t += 256) xsub[t] = x[row * d + (int64_t)m * dsub + t];
            __syncthreads();
            const float* ctm = ct + (int64_t)m * dsub * 256;
            float dot = 0.0f;
            for (int t = 0; t < dsub; ++t) dot = __builtin_fmaf(xsub[t], ctm[(int64_t)t * 256 + tid], dot);
            const float s = __builtin_fmaf(-2.0f, dot, cn[(int64_t)m * 256 + tid]);
            rkey[tid] = (s < INFINITY) ? s : INFINITY;  // NaN / +inf never win
            ridx[tid] = tid;
            __syncthreads();
            for (int st = 128; st > 0; st >>= 1) {
                if (tid < st) {
                    const float a = rkey[tid], c2 = rkey[tid + st];
                    const int ia = ridx[tid], ic = ridx[tid + st];
                    if (c2 < a || (c2 == a && ic < ia)) { rkey[tid] = c2; ridx[tid] = ic; }
                }
                __syncthreads();
            }
            if (tid == 0) codes[row * M + m] = (uint8_t)(rkey[0] < INFINITY ? ridx[0] : 0);
        }
    }
}

// ------------------------------------------------------------------------ pack / unpack
__global__ void pq_pack_kernel(const uint8_t* __restrict__ u8, int64_t n, int M, int nbits,
                               uint8_t* __restrict__ out) {
    const int cs = (M * nbits + 7) / 8;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // output byte
    if (e >= n * cs) return;
    const int64_t i = e / cs;
    const int byte = (int)(e % cs);
    uint32_t v = 0;
    for (int bit = 0; bit < 8; ++bit) {
        const int gb = byte * 8 + bit;
        const int m = gb / nbits, b = gb % nbits;
        if (m < M) v |= (uint32_t)((u8[i * M + m] >> b) & 1u) << bit;
    }
    out[e] = (uint8_t)v;
}

__global__ void pq_unpack_kernel(const uint8_t* __restrict__ packed, int64_t n, int M, int nbits,
                                 uint8_t* __restrict__ out) {
    const int cs = (M * nbits + 7) / 8;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * M) return;
    const int64_t i = e / M;
    const int m = (int)(e % M);
    const uint8_t* p = packed + i * cs;
    uint32_t v = 0;
    for (int b = 0; b < nbits; ++b) {
        const int gb = m * nbits + b;
        v |= (uint32_t)((p[gb >> 3] >> (gb & 7)) & 1u) << b;
    }
    out[e] = (uint8_t)v;
}

// ------------------------------------------------------------------------------ decode
// One thread per 4 output floats (dsub % 4 == 0) or per float.
template <int VEC>
__global__ void pq_decode_kernel(const uint8_t* __restrict__ codes, int64_t n, int d, int M,
                                 int nbits, int dsub, const float* __restrict__ C,
                                 float* __restrict__ out) {
    const int ksub = 1 << nbits;
    const int cs = (M * nbits + 7) / 8;
    const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * VEC;
    if (e >= n * (int64_t)d) return;
    const int64_t i = e / d;
    const int j = (int)(e % d);
    const int m = j / dsub, t = j % dsub;
    uint32_t code;
    if (nbits == 8) {
        code = codes[i * cs + m];
    } else {
        code = 0;
        const uint8_t* p = codes + i * cs;
        for (int b = 0; b < nbits; ++b) {
            const int gb = m * nbits + b;
            code |= (uint32_t)((p[gb >> 3] >> (gb & 7)) & 1u) << b;
        }
    }
    const float* src = C + ((int64_t)m * ksub + code) * dsub + t;
    if (VEC == 4) *reinterpret_cast<float4*>(out + e) = *reinterpret_cast<const float4*>(src);
    else out[e] = *src;
}

// ------------------------------------------------------------------- k-means update
// grid (ksub, M), block 256: block (k, m) gathers, in ascending row order, the rows assigned
// to centroid k of subspace m and sums their subvectors sequentially (deterministic).
constexpr int kKmDims = 8;  // dims per thread of kmeans_update_kernel: dsub <= 2048

__global__ __launch_bounds__(256) void kmeans_update_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int ksub, int dsub,
    const uint8_t* __restrict__ assign, float* __restrict__ centroids, int32_t* __restrict__ counts) {
    __shared__ int64_t rows[256];
    __shared__ int nsel;
    const int k = blockIdx.x, m = blockIdx.y, tid = threadIdx.x;
    float sum[kKmDims];  // thread tid owns dimensions tid + 256 u (dsub <= 256 kKmDims)
#pragma unroll
    for (int u = 0; u < kKmDims; ++u) sum[u] = 0.0f;
    int64_t count = 0;
    for (int64_t base = 0; base < n; base += 256) {
        const int64_t rr = base + tid;
        const bool hit = rr < n && assign[rr * M + m] == (uint8_t)k;
        // ordered compaction of this chunk's hits
        const unsigned long long b = __ballot(hit);
        __shared__ int wave_off[4];
        const int wv = tid >> 6, ln = tid & 63;
        if (ln == 0) wave_off[wv] = __popcll(b);
        __syncthreads();
        if (tid == 0) {
            int s = 0;
            for (int q = 0; q < 4; ++q) { const int c = wave_off[q]; wave_off[q] = s; s += c; }
            nsel = s;
        }
        __syncthreads();
        if (hit) rows[wave_off[wv] + __popcll(b & ((1ull << ln) - 1ull))] = rr;
        __syncthreads();
        const int ns = nsel;
#pragma unroll
        for (int u = 0; u < kKmDims; ++u)
            if (tid + 256 * u < dsub)
                for (int q = 0; q < ns; ++q) sum[u] += x[rows[q] * d + (int64_t)m * dsub + tid + 256 * u];
        count += ns;
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < kKmDims; ++u)
        if (tid + 256 * u < dsub && count > 0)
            centroids[((int64_t)m * ksub + k) * dsub + tid + 256 * u] = sum[u] / (float)count;
    if (tid == 0) counts[(int64_t)m * ksub + k] = (int32_t)count;
}

int mfma_smem_bytes(int KS, int M) { return 2 * 8 * KS * 64 * 16 + 2 * 256 * 4 + kWaves * 32 * M; }

template <int KS>
hipError_t launch_mfma(const float* x, int64_t n, int d, int M, int dsub, const float* C,
                       const float* cn, const half8* img, const float* hinit, const float4* bnd,
                       uint8_t* codes, uint32_t* flags, hipStream_t st) {
    const int smem = mfma_smem_bytes(KS, M);
    auto kern = pq_encode_mfma_kernel<KS>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    if (e != hipSuccess) return e;
    const int64_t grid = ceil_div(n, kWaves * 32);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), smem, st, x, n, d, M, dsub, C, cn,
                       img, hinit, bnd, codes, flags);
    return hipGetLastError();
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" size_t mivq_pq_prep_bytes(int32_t d, int32_t M, int32_t nbits) {
    if (M <= 0 || d <= 0 || d % M != 0 || nbits < 1 || nbits > 8) return 0;
    return pq_prep_layout(d, M, nbits).total;
}

extern "C" int mivq_pq_prepare(const float* centroids, int32_t d, int32_t M, int32_t nbits,
                               void* prep, void* stream) {
    MIVQ_REQUIRE(M > 0 && d > 0, MIVQ_ERR_INVALID, "pq_prepare: d=%d M=%d must be positive", d, M);
    MIVQ_REQUIRE(d % M == 0, MIVQ_ERR_INVALID, "D must be divisible by M (number of subquantizers): d=%d M=%d", d, M);
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "pq_prepare: nbits=%d not in [1, 8]", nbits);
    MIVQ_REQUIRE(centroids && prep, MIVQ_ERR_INVALID, "pq_prepare: null pointer");
    const PqPrepLayout L = pq_prep_layout(d, M, nbits);
    unsigned char* p = static_cast<unsigned char*>(prep);
    hipStream_t st = as_stream(stream);
    const int64_t mk = (int64_t)M * L.ksub;
    // pads between the regions are zeroed so that equal codebooks give byte-equal prep buffers
    // (pd, the large table, is written in full by pq_prep_spread_kernel)
    hipError_t me = hipMemsetAsync(p, 0, L.pd, st);
    if (me == hipSuccess) me = hipMemsetAsync(p + L.bnd2, 0, L.total - L.bnd2, st);
    if (me != hipSuccess) return set_error(MIVQ_ERR_HIP, "pq_prepare(memset): %s", hipGetErrorString(me));
    hipLaunchKernelGGL(pq_prep_norms_kernel, dim3((unsigned)ceil_div(mk, 256)), dim3(256), 0, st,
                       centroids, M, L.ksub, L.dsub, reinterpret_cast<float*>(p + L.cn),
                       reinterpret_cast<float*>(p + L.ct));
    int rc = check_launch("pq_prep_norms");
    if (rc) return rc;
    if (L.mfma) {
        uint32_t* spread = reinterpret_cast<uint32_t*>(p + L.spread);
        float2* pd = M <= kPdMaxM ? reinterpret_cast<float2*>(p + L.pd) : nullptr;
        hipLaunchKernelGGL(pq_prep_spread_kernel, dim3(M, 16), dim3(256), 0, st, centroids, L.dsub, spread, pd);
        rc = check_launch("pq_prep_spread");
        if (rc) return rc;
        hipLaunchKernelGGL(pq_prep_mfma_kernel, dim3(M), dim3(256), 0, st, centroids,
                           reinterpret_cast<const float*>(p + L.cn), M, L.dsub, L.ks,
                           reinterpret_cast<half8*>(p + L.img), reinterpret_cast<float*>(p + L.hinit),
                           reinterpret_cast<float4*>(p + L.bnd), spread, reinterpret_cast<float4*>(p + L.bnd2));
        rc = check_launch("pq_prep_mfma");
    }
    return rc;
}

extern "C" size_t mivq_pq_encode_workspace_bytes(int64_t n, int32_t d, int32_t M, int32_t nbits) {
    if (n < 0 || M <= 0) return 0;
    size_t b = 0;
    if (nbits != 8) b += align_up((size_t)n * M, 256);                 // unpacked codes
    b += align_up((size_t)n * M, 256);  // transposed codes (cs path)
    // cs path: n*M uint2 resolve items; legacy MFMA path: its filter flags (never both)
    b += align_up(std::max((size_t)n * M * 8, (size_t)ceil_div(n, 32) * M * sizeof(uint32_t)), 256);
    b += align_up(cs_counts_bytes(n, M), 256);  // cs path: list counts per workgroup
    return b;
}

extern "C" int mivq_pq_encode(const float* x, int64_t n, int32_t d, int32_t M, int32_t nbits,
                              const float* centroids, const void* prep, void* workspace,
                              size_t workspace_bytes, uint8_t* codes, uint32_t flags_in,
                              void* stream) {
    MIVQ_REQUIRE(M > 0 && d > 0 && n >= 0, MIVQ_ERR_INVALID, "pq_encode: bad sizes n=%lld d=%d M=%d", (long long)n, d, M);
    MIVQ_REQUIRE(d % M == 0, MIVQ_ERR_INVALID, "D must be divisible by M (number of subquantizers): d=%d M=%d", d, M);
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "pq_encode: nbits=%d not in [1, 8]", nbits);
    MIVQ_REQUIRE(prep != nullptr, MIVQ_ERR_INVALID, "pq_encode: prep is required (mivq_pq_prepare)");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && centroids && codes, MIVQ_ERR_INVALID, "pq_encode: null pointer");
    const size_t need = mivq_pq_encode_workspace_bytes(n, d, M, nbits);
    MIVQ_REQUIRE(workspace_bytes >= need && (need == 0 || workspace), MIVQ_ERR_WORKSPACE,
                 "pq_encode: workspace %zu < %zu bytes", workspace_bytes, need);
    const PqPrepLayout L = pq_prep_layout(d, M, nbits);
    const unsigned char* p = static_cast<const unsigned char*>(prep);
    const float* cn = reinterpret_cast<const float*>(p + L.cn);
    const float* ct = reinterpret_cast<const float*>(p + L.ct);
    hipStream_t st = as_stream(stream);
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    uint8_t* u8 = codes;
    size_t off = 0;
    if (nbits != 8) { u8 = ws; off = align_up((size_t)n * M, 256); }
    uint8_t* codesT = ws + off;
    off += align_up((size_t)n * M, 256);
    uint32_t* fl = reinterpret_cast<uint32_t*>(ws + off);  // legacy path
    void* items = ws + off;                                // cs path
    off += align_up(std::max((size_t)n * M * 8, (size_t)ceil_div(n, 32) * M * sizeof(uint32_t)), 256);
    void* counts = ws + off;
    off += align_up(cs_counts_bytes(n, M), 256);

    const bool aligned = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && (d % 4 == 0) && (L.dsub % 4 == 0);
    const bool exact_only = (flags_in & MIVQ_PQ_FORCE_EXACT) != 0;
    // (the code transpose after the filter stages (256 + 16) * M bytes of LDS: M <= 512)
    const bool cs_ok = L.mfma && aligned && !exact_only && L.ks <= 12 && cs_smem_bytes(L.ks, L.dsub) <= 160 * 1024 &&
                       M <= 512 && !(flags_in & MIVQ_PQ_LEGACY_MFMA);
    const bool mfma_ok = L.mfma && aligned && L.ks <= 8 && !exact_only && mfma_smem_bytes(L.ks, M) <= 160 * 1024;
    if (cs_ok) {
        // Calls above 2^20 rows run as consecutive 2^20-row slices on the same stream (the
        // workspace regions are reused, stream-ordered): the same codes, and a 10M x 1536 PQ16
        // call runs faster than in one piece (round 3: 13.85 vs 14.43 ms at 2^21-row slices,
        // tools/probe_chunked.py: a long filter-only stretch runs at a lower power-managed clock
        // than filters interleaved with their resolve launches; round 5: 2^20-row slices another
        // 1.2 % faster at 10M x 1536, equal at 6.65M x 1024, 2^19 / 2^22 no better,
        // profiles/r05_s28, r05_s29)
        constexpr int64_t kSlice = (int64_t)1 << 20;
        for (int64_t r0 = 0; r0 < n; r0 += kSlice) {
            const int64_t nc = std::min(kSlice, n - r0);
            const hipError_t e = launch_pq_encode_cs(L.ks, x + r0 * d, nc, d, M, L.dsub, centroids, cn, p + L.img,
                                                     reinterpret_cast<const float*>(p + L.hinit), p + L.bnd,
                                                     M <= kPdMaxM ? p + L.pd : nullptr, p + L.bnd2, codesT, items,
                                                     counts, u8 + r0 * M, st);
            if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "pq_encode_cs: %s", hipGetErrorString(e));
        }
    } else if (mfma_ok) {
        const half8* img = reinterpret_cast<const half8*>(p + L.img);
        const float* hinit = reinterpret_cast<const float*>(p + L.hinit);
        const float4* bnd = reinterpret_cast<const float4*>(p + L.bnd);
        hipError_t e = hipSuccess;
        switch (L.ks) {
            case 1: e = launch_mfma<1>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 2: e = launch_mfma<2>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 3: e = launch_mfma<3>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 4: e = launch_mfma<4>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 5: e = launch_mfma<5>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 6: e = launch_mfma<6>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 7: e = launch_mfma<7>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
            case 8: e = launch_mfma<8>(x, n, d, M, L.dsub, centroids, cn, img, hinit, bnd, u8, fl, st); break;
        }
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "pq_encode_mfma: %s", hipGetErrorString(e));
        const int64_t nwords = ceil_div(n, 32) * M;
        const int rgrid = (int)std::min<int64_t>(nwords, 4096);
        hipLaunchKernelGGL(pq_resolve_kernel, dim3(rgrid), dim3(256), (size_t)L.dsub * sizeof(float), st,
                           x, n, d, M, L.dsub, ct, cn, fl, nwords, u8);
        int rc = check_launch("pq_resolve");
        if (rc) return rc;
    } else if (L.ksub == 256 && L.dsub % 4 == 0 && aligned && !(flags_in & MIVQ_PQ_LEGACY_EXACT)) {
        hipLaunchKernelGGL(pq_encode_exact_tiled_kernel, dim3((unsigned)ceil_div(n, kXRows), (unsigned)M),
                           dim3(256), 0, st, x, n, d, M, L.dsub, ct, cn, u8);
        int rc = check_launch("pq_encode_exact_tiled");
        if (rc) return rc;
    } else {
        const size_t smem = (size_t)64 * (L.dsub + 1) * sizeof(float);
        MIVQ_REQUIRE(smem <= 160 * 1024, MIVQ_ERR_UNSUPPORTED, "pq_encode: dsub=%d too large", L.dsub);
        const dim3 grid((unsigned)ceil_div(n, 64), (unsigned)M);
        hipError_t e = hipSuccess;
#define MIVQ_EXACT(KG)                                                                                   \
    e = hipFuncSetAttribute((const void*)pq_encode_exact_kernel<KG>,                                    \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);                     \
    if (e == hipSuccess) {                                                                              \
        hipLaunchKernelGGL(pq_encode_exact_kernel<KG>, grid, dim3(64), smem, st, x, n, d, M, L.ksub,    \
                           L.dsub, ct, cn, u8);                                                         \
        e = hipGetLastError();                                                                          \
    }
        if (L.ksub % 8 == 0) { MIVQ_EXACT(8) }
        else if (L.ksub % 4 == 0) { MIVQ_EXACT(4) }
        else { MIVQ_EXACT(2) }
#undef MIVQ_EXACT
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "pq_encode_exact: %s", hipGetErrorString(e));
    }
    if (nbits != 8) {
        const int cs = pq_code_size(M, nbits);
        hipLaunchKernelGGL(pq_pack_kernel, dim3((unsigned)ceil_div(n * cs, 256)), dim3(256), 0, st, u8, n,
                           M, nbits, codes);
        return check_launch("pq_pack");
    }
    return MIVQ_OK;
}

extern "C" int mivq_pq_decode(const uint8_t* codes, int64_t n, int32_t d, int32_t M, int32_t nbits,
                              const float* centroids, float* out, void* stream) {
    MIVQ_REQUIRE(M > 0 && d > 0 && n >= 0 && d % M == 0, MIVQ_ERR_INVALID,
                 "pq_decode: bad sizes n=%lld d=%d M=%d", (long long)n, d, M);
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "pq_decode: nbits=%d not in [1, 8]", nbits);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(codes && centroids && out, MIVQ_ERR_INVALID, "pq_decode: null pointer");
    const int dsub = d / M;
    hipStream_t st = as_stream(stream);
    const int64_t total = n * (int64_t)d;
    const bool vec = dsub % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(centroids) % 16 == 0;
    if (vec)
        hipLaunchKernelGGL(pq_decode_kernel<4>, dim3((unsigned)ceil_div(total / 4, 256)), dim3(256), 0, st,
                           codes, n, d, M, nbits, dsub, centroids, out);
    else
        hipLaunchKernelGGL(pq_decode_kernel<1>, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st,
                           codes, n, d, M, nbits, dsub, centroids, out);
    return check_launch("pq_decode");
}

extern "C" int mivq_pq_unpack(const uint8_t* codes, int64_t n, int32_t M, int32_t nbits, uint8_t* out,
                              void* stream) {
    MIVQ_REQUIRE(M > 0 && n >= 0 && nbits >= 1 && nbits <= 8, MIVQ_ERR_INVALID, "pq_unpack: bad args");
    if (n == 0) return MIVQ_OK;
    hipStream_t st = as_stream(stream);
    if (nbits == 8) {
        hipError_t e = hipMemcpyAsync(out, codes, (size_t)n * M, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "pq_unpack: %s", hipGetErrorString(e));
        return MIVQ_OK;
    }
    hipLaunchKernelGGL(pq_unpack_kernel, dim3((unsigned)ceil_div(n * M, 256)), dim3(256), 0, st, codes, n, M,
                       nbits, out);
    return check_launch("pq_unpack");
}

extern "C" int mivq_kmeans_update(const float* x, int64_t n, int32_t d, int32_t M, int32_t ksub,
                                  const uint8_t* assign, float* centroids, int32_t* counts, void* stream) {
    MIVQ_REQUIRE(M > 0 && d > 0 && n >= 0 && d % M == 0, MIVQ_ERR_INVALID, "kmeans_update: bad sizes");
    MIVQ_REQUIRE(ksub >= 1 && ksub <= 256, MIVQ_ERR_UNSUPPORTED, "kmeans_update: ksub=%d", ksub);
    MIVQ_REQUIRE(d / M <= 256 * kKmDims, MIVQ_ERR_UNSUPPORTED, "kmeans_update: dsub=%d > %d", d / M, 256 * kKmDims);
    hipLaunchKernelGGL(kmeans_update_kernel, dim3(ksub, M), dim3(256), 0, as_stream(stream), x, n, d, M, ksub,
                       d / M, assign, centroids, counts);
    return check_launch("kmeans_update");
}
