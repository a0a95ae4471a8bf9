// opq.hip — OPQ rotation y = x . op(A) as a hand-written MFMA GEMM on gfx950.
//
// Replaces faiss.OPQMatrix.apply / reverse_transform used by OptimizedProductQuantizer
// (/root/reference/src/haag_vq/methods/optimized_product_quantization.py:26,31,34):
//   transpose == 0 : y = x . A^T   (LinearTransform::apply, A is d_out x d_in row-major)
//   transpose == 1 : y = x . A     (reverse_transform of an orthonormal A)
//
// Two kernels:
//
// 1. mivq_opq_rotate_prepared (the product path): fp32-accurate GEMM out of f16 MFMAs.
//    Every operand is split into two f16 terms, v = hi + lo with hi = f16(s v),
//    lo = f16(s v - hi) (the difference is exact in fp32), after a power-of-two scale s that
//    puts the largest |v| of the row (x) or of the matrix (A) at 2^13..2^14, inside f16's
//    range.  y = (x_hi b_hi + x_hi b_lo + x_lo b_hi) / (s_x s_b): each f16 x f16 product is
//    exact in the fp32 accumulator, and the terms left out (x_lo b_lo and the residuals of the
//    two splits) are <= ~3 * 2^-22 of |x_k b_k|, far below the fp32 accumulation rounding every
//    GEMM has (tests/test_opq_gpu.py checks 1e-5 of ||x|| ||a|| against fp64).  Three
//    v_mfma_f32_32x32x16_f16 per 32x32x16 block = 3 x 1/16 of the fp32-MFMA cost per flop.
//    mivq_opq_prepare builds the hi / lo images of B = op(A) once per matrix ([col][k] rows,
//    scaled); opq_row_scale_kernel computes x's row scales; opq_split_gemm_kernel splits x
//    while staging it (register-staged, 80-B padded rows, 256 x 256 or 128 x 128 tiles,
//    XCD-aware tile order so the column tiles of a row block share one L2, epilogue through
//    LDS as 16-B row stores).
//    No LDS DMA (global_load_lds_*): round 2's DMA-staged GEMM, while resident next to another
//    kernel's waves, corrupted lanes 48..63 of their packed-fp32 VALU results (v_pk_add_f32 /
//    v_pk_fma_f32 on LDS-loaded operands); a synthetic kernel that only overlaps LDS DMA with
//    MFMAs does the same, and neither does it without the MFMAs or without the DMA
//    (tools/probes/lut_stress.hip).  The library must not corrupt kernels it runs
//    beside (its own, torch's), so every shape takes the register-staged path.
// 2. opq_gemm_kernel (mivq_opq_rotate, no preparation, any d): plain fp32 MFMA
//    (v_mfma_f32_32x32x2_f32), 128 x 128 tiles, BK = 16 slices staged through LDS.
#include <math.h>

#include <algorithm>

#include "mivq_common.h"

namespace mivq {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ fp32 MFMA kernel
constexpr int BM = 128, BN = 128, BK = 16, PAD = 4;

__global__ __launch_bounds__(256) void opq_gemm_kernel(const float* __restrict__ x, int64_t n, int d,
                                                       const float* __restrict__ A, int transpose,
                                                       float* __restrict__ y) {
    __shared__ float xs[BK][BM + PAD];  // xs[k][i] = x[r0 + i][k0 + k]
    __shared__ float bs[BK][BN + PAD];  // bs[k][j] = B[k0 + k][c0 + j]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int64_t r0 = (int64_t)blockIdx.x * BM;
    const int c0 = blockIdx.y * BN;
    floatx16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

    const int kl = lane >> 5, il = lane & 31;
    for (int k0 = 0; k0 < d; k0 += BK) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + q * 256;
            const int i = e >> 4, kk = e & 15;
            const int64_t row = r0 + i;
            xs[kk][i] = (row < n && k0 + kk < d) ? x[row * d + k0 + kk] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + q * 256;
            if (transpose == 0) {  // B[k][j] = A[j][k]
                const int j = e >> 4, kk = e & 15;
                bs[kk][j] = (c0 + j < d && k0 + kk < d) ? A[(int64_t)(c0 + j) * d + k0 + kk] : 0.0f;
            } else {  // B[k][j] = A[k][j]
                const int kk = e >> 7, j = e & 127;
                bs[kk][j] = (c0 + j < d && k0 + kk < d) ? A[(int64_t)(k0 + kk) * d + c0 + j] : 0.0f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < BK; ks += 2) {
            float a0 = xs[ks + kl][wr * 64 + il];
            float a1 = xs[ks + kl][wr * 64 + 32 + il];
            float b0 = bs[ks + kl][wc * 64 + il];
            float b1 = bs[ks + kl][wc * 64 + 32 + il];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    // C layout: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                const int64_t gr = r0 + wr * 64 + a * 32 + row;
                const int gc = c0 + wc * 64 + b * 32 + (lane & 31);
                if (gr < n && gc < d) y[gr * d + gc] = acc[a][b][e];
            }
}

// ------------------------------------------------------------------ split-f16 kernel
constexpr int SBK = 32;
constexpr int SPITCH = SBK * 2 + 16;          // bytes per LDS row (64 B of halves + 16 B pad)
constexpr int kScaleShift = 14;               // largest |v| scaled into [2^13, 2^14]

// Tile geometry: WR x WC waves, each RB x CB blocks of 32 x 32 outputs; the workgroup tile is
// TM = 32 WR RB rows by TN = 32 WC CB columns.
template <int WR, int WC, int RB, int CB>
struct SplitTile {
    static constexpr int NT = WR * WC * 64;
    static constexpr int TM = 32 * WR * RB, TN = 32 * WC * CB;
    static constexpr int BUF = 2 * (TM + TN) * SPITCH;  // x hi, x lo, B hi, B lo planes
    static constexpr int SMEM = 2 * BUF;                // double-buffered
    static constexpr int U = TM * SBK / 4 / NT;          // 16-B loads of each kind per thread
    static_assert(TM * SBK / 4 == U * NT && 2 * TN * SBK / 8 == U * NT && TM == TN, "loads per thread");
};
using TileS = SplitTile<2, 2, 2, 2>;  // 128 x 128, 256 threads, 80 KiB (two per CU)
using TileL = SplitTile<4, 2, 2, 4>;  // 256 x 256, 512 threads, 160 KiB (half the L2 traffic per MFMA)
// Measured and removed: 256 x 256 with 4 waves of 128 x 128 (16.0 vs 14.8 ms per
// 1M x 1536 GEMM), a 4-wave software-pipelined kernel with sched_group_barrier interleaving
// (17.4 vs 16.2 ms), non-temporal x / B-image loads, and (round 5) row scales found inside the
// GEMM chunk by chunk instead of the row-scale pass (15.40 vs 14.65 ms: the per-chunk max and
// its 8-lane reduction in the staging cost more than the pass over x).

// Power-of-two scale 2^(14 - E) with max|v| = m 2^E, m in [0.5, 1); 1 for 0 / inf / NaN.
// Clamped to fp32's normal exponents (rows below 2^-112 lose relative accuracy).
__device__ __forceinline__ float pow2_scale(float amax) {
    if (!(amax > 0.0f) || !isfinite(amax)) return 1.0f;
    int e;
    (void)frexpf(amax, &e);
    const int sh = min(126, max(-126, kScaleShift - e));
    return ldexpf(1.0f, sh);
}

__device__ __forceinline__ void split2(float v, _Float16& hi, _Float16& lo) {
    hi = (_Float16)v;
    lo = (_Float16)(v - (float)hi);
}

// Per-row scale of x: one wave per row; d % 4 == 0 and 16-B aligned rows (the prepared path):
// 16-B loads, eight per lane in flight (round 2's dword loop waited on one 4-B load at a time).
__global__ __launch_bounds__(256) void opq_row_scale_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                float* __restrict__ rs) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    if (row >= n) return;
    const float4* xr = reinterpret_cast<const float4*>(x + row * d);
    const int q = d >> 2;
    float m = 0.0f;
    bool bad = false;
    for (int j0 = l; j0 < q; j0 += 8 * 64) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + 64 * u;
            v[u] = j < q ? xr[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            bad |= !isfinite(v[u].x) || !isfinite(v[u].y) || !isfinite(v[u].z) || !isfinite(v[u].w);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    bad = __any(bad);
    if (l == 0) rs[row] = bad ? 1.0f : pow2_scale(m);
}

// max |A| over the whole matrix -> header {s_b, 1 / s_b} of the prepared image (one workgroup).
__global__ __launch_bounds__(1024) void opq_absmax_kernel(const float* __restrict__ A, int64_t cnt,
                                                          float* __restrict__ hdr) {
    __shared__ float red[16];
    __shared__ int bad_any;
    if (threadIdx.x == 0) bad_any = 0;
    __syncthreads();
    float m = 0.0f;
    bool bad = false;
    for (int64_t i = threadIdx.x; i < cnt; i += 1024) {
        const float v = A[i];
        bad |= !isfinite(v);
        m = fmaxf(m, fabsf(v));
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&bad_any, 1);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = 0.0f;
        for (int i = 0; i < 16; ++i) mm = fmaxf(mm, red[i]);
        const float s = bad_any ? 1.0f : pow2_scale(mm);
        hdr[0] = s;
        hdr[1] = 1.0f / s;
    }
}

// B image: bimg[plane][j][k] = split(s_b * op(A)[k][j]), plane 0 = hi, 1 = lo; op(A)[k][j] =
// A[j][k] for transpose 0 (y = x A^T), A[k][j] for transpose 1.
__global__ __launch_bounds__(256) void opq_split_b_kernel(const float* __restrict__ A, int d, int transpose,
                                                          const float* __restrict__ hdr, _Float16* __restrict__ bimg) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t dd = (int64_t)d * d;
    if (e >= dd) return;
    const int j = (int)(e / d), k = (int)(e - (int64_t)j * d);
    const float v = (transpose == 0 ? A[(int64_t)j * d + k] : A[(int64_t)k * d + j]) * hdr[0];
    _Float16 hi, lo;
    split2(v, hi, lo);
    bimg[e] = hi;
    bimg[dd + e] = lo;
}

// LDS staging line (x row / B column) of staging thread-slot e, 8 slots of 8 B per 64-B line.
// A 16-lane ds_write_b64 group (or 8-lane ds_write_b128 group) covers two lines; with the 80-B
// pitch lines j and j + 1 overlap on 4 of the 32 store banks ((a/4) mod 32: 2-way conflicts on
// every staging store -- the ~577 M conflict cycles per 1M x 1536 rotation in PMC), lines j and
// j + 4 do not (80 B x 4 = 16 banks apart).  Against the round-3 order (line e / 8): 16.16 ->
// 16.01 ms per rotation.
__device__ __forceinline__ int stage_line(int e) {
    const int g = e >> 4, sub = (e >> 3) & 1;
    return (g >> 2) * 8 + (g & 3) + 4 * sub;
}

// Tile t of workgroup b: the workgroups of one XCD (b % 8, dealt round-robin) take a
// contiguous range of tiles, so consecutive tiles (the column tiles of one row block) share
// that XCD's L2.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t G) {
    const int64_t x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    return x * q + min(x, r) + j;
}

// Epilogue of both split GEMMs: y = acc / (s_x s_b) (powers of two: exact).  The wave's
// RB x CB blocks go out half a wave tile (32 rows) at a time through its own LDS slice
// (32 x 32 CB floats, the staging buffers being dead by then): accumulator layout in, rows of
// 16-B stores out (one 64-bit address per row instead of per element, no per-element
// bounds branches, one row-scale load per lane).  Callers pass the block after a barrier.
template <int RB, int CB>
__device__ __forceinline__ void store_tile(const floatx16 (&acc)[RB][CB], unsigned char* smem, int w, int l,
                                           int64_t rowbase, int colbase, int64_t n, int d,
                                           const float* __restrict__ rs, float binv, float* __restrict__ y) {
    constexpr int CW = CB * 32, LPR = CW / 4, RPIT = 64 / LPR;
    float* tw = reinterpret_cast<float*>(smem) + w * 32 * CW;
#pragma unroll
    for (int a = 0; a < RB; ++a) {
        const int64_t gra = rowbase + a * 32 + (l & 31);
        const float rsl = rs[gra < n ? gra : n - 1];
#pragma unroll
        for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e)
                tw[((e & 3) + 8 * (e >> 2) + 4 * (l >> 5)) * CW + b * 32 + (l & 31)] = acc[a][b][e];
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's own slice
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 32 / RPIT; ++it) {
            const int rl = it * RPIT + l / LPR, cl = 4 * (l % LPR);
            const float4 v = *reinterpret_cast<const float4*>(tw + rl * CW + cl);
            const float sc = binv / __shfl(rsl, rl);
            const int64_t gr = rowbase + a * 32 + rl;
            const int gc = colbase + cl;
            if (gr < n && gc < d)  // d % 8 == 0: the whole float4 is inside the row
                *reinterpret_cast<float4*>(y + gr * d + gc) = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
}

template <int WR, int WC, int RB, int CB>
__global__ __launch_bounds__(WR * WC * 64) void opq_split_gemm_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                      const float* __restrict__ rs,
                                                                      const _Float16* __restrict__ bimg,
                                                                      const float* __restrict__ hdr,
                                                                      float* __restrict__ y, int64_t ctiles) {
    using T = SplitTile<WR, WC, RB, CB>;
    constexpr int NT = T::NT, TM = T::TM, TN = T::TN;
    constexpr int XPL = TM * SPITCH, BPL = TN * SPITCH;  // plane sizes
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int wr = w / WC, wc = w % WC;
    const int64_t t = xcd_tile(blockIdx.x, gridDim.x);
    const int64_t r0 = (t / ctiles) * TM;
    const int c0 = (int)(t % ctiles) * TN;
    const int64_t dd = (int64_t)d * d;

    // staging geometry: x: U float4 per thread (row e / 8, k 4 (e % 8)); B: U x 16 B per
    // thread (plane e / (4 TN), column (e % 4 TN) / 4, k 8 (e % 4))
    constexpr int U = T::U;
    float sx[U];
    int xrow[U], xk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + NT * u;
        xrow[u] = stage_line(e);
        xk[u] = 4 * (e & 7);
        const int64_t gr = r0 + xrow[u];
        sx[u] = gr < n ? rs[gr] : 0.0f;
    }
    int bpl[U], bcol[U], bk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + NT * u;
        bpl[u] = e / (4 * TN);
        bcol[u] = stage_line(2 * (e % (4 * TN)));  // 4 lanes of 16 B per column
        bk[u] = 8 * (e & 3);
    }
    float4 xv[U];
    uint4 bv[U];
    // range-checked 16-B buffer loads (rows past n read zeros; a chunk past d gets an
    // out-of-range offset) instead of one guarded load per chunk, which compiled to a branch per
    // load (15.93 -> 14.80 ms per 1M x 1536 rotation, profiles/r04_s14); 32-bit offsets from the
    // tile's first row (4 d^2 < 2^31 checked at launch)
    constexpr int kOob = (int)0x80000000u;
    const int trows = (int)(n - r0 < TM ? n - r0 : TM);
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(x + r0 * d), 0, trows * d * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)bimg, 0, (int)(dd * 4), 0x00020000);
    auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + xk[u], gc = c0 + bcol[u], kb = k0 + bk[u];
            const int vx = k < d ? (xrow[u] * d + k) * 4 : kOob;
            const int vb = (gc < d && kb < d) ? (int)((bpl[u] * dd + (int64_t)gc * d + kb) * 2) : kOob;
            xv[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vx, 0, 0));
            bv[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(brs, vb, 0, 0));
        }
    };
    auto sstore = [&](unsigned char* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            half4 h, lo;
            const float v[4] = {xv[u].x * sx[u], xv[u].y * sx[u], xv[u].z * sx[u], xv[u].w * sx[u]};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                _Float16 a, b;
                split2(v[q], a, b);
                h[q] = a;
                lo[q] = b;
            }
            const int off = xrow[u] * SPITCH + 2 * xk[u];
            *reinterpret_cast<half4*>(buf + off) = h;
            *reinterpret_cast<half4*>(buf + XPL + off) = lo;
            *reinterpret_cast<uint4*>(buf + 2 * XPL + bpl[u] * BPL + bcol[u] * SPITCH + 2 * bk[u]) = bv[u];
        }
    };

    floatx16 acc[RB][CB];
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
        for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

    const int nsteps = (d + SBK - 1) / SBK;
    gload(0);
    sstore(smem);
    // stage first: step s + 1's chunks (loaded during step s - 1) go to LDS at the START of step
    // s, then step s + 2's loads are issued, then step s's MFMAs -- the loads have a whole step
    // to land and the store no longer sits between the MFMAs and the barrier (14.80 -> 14.27 ms,
    // r04_s22); loads past d read zeros (buffer loads), so no branch surrounds them (the last
    // steps' stores are never read)
    gload(SBK);
    __syncthreads();
    const int fr = l & 31, fk = 16 * (l >> 5);  // fragment row / col and byte offset of its k-group
    for (int s = 0; s < nsteps; ++s) {
        unsigned char* cur = smem + (s & 1) * T::BUF;
        sstore(smem + ((s + 1) & 1) * T::BUF);
        gload((s + 2) * SBK);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            half8 ah[RB], al[RB], bh[CB], bl[CB];
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const int ar = (wr * RB * 32 + i * 32 + fr) * SPITCH + 32 * kk + fk;
                ah[i] = *reinterpret_cast<const half8*>(cur + ar);
                al[i] = *reinterpret_cast<const half8*>(cur + XPL + ar);
            }
#pragma unroll
            for (int j = 0; j < CB; ++j) {
                const int bc = (wc * CB * 32 + j * 32 + fr) * SPITCH + 32 * kk + fk;
                bh[j] = *reinterpret_cast<const half8*>(cur + 2 * XPL + bc);
                bl[j] = *reinterpret_cast<const half8*>(cur + 2 * XPL + BPL + bc);
            }
            // small terms first; RB * CB independent accumulators between dependent MFMAs
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
                for (int b = 0; b < CB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
                for (int b = 0; b < CB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
                for (int b = 0; b < CB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue (the staging buffers are reused: every wave must be done with them)
    __syncthreads();
    store_tile<RB, CB>(acc, smem, w, l, r0 + wr * RB * 32, c0 + wc * CB * 32, n, d, rs, hdr[1], y);
}

// ------------------------------------------------------------ Procrustes Gram matrix (training)
// G = X^T Y in fp64 for the OPQ update (faiss OPQMatrix::train's X^T Yhat before its SVD,
// /root/reference/src/haag_vq/methods/optimized_product_quantization.py:21-28): X, Y (n, d) f32
// rows, each product exact in fp64 (24 + 24 bits), sums in fp64 on v_mfma_f64_16x16x4_f64.
// Split K: workgroup (tile, s) sums rows [s R, (s + 1) R) of a 128 x 128 tile of G into
// part[s]; opq_gram_reduce_kernel adds the parts in s order (deterministic).  4 waves of 64 x 64
// (4 x 4 blocks); f64 operand map as erq_rotate_kernel: A[l & 15][l >> 4], B[l >> 4][l & 15],
// D column l & 15, rows (l >> 4) + 4 g.
constexpr int GR_T = 128, GR_K = 16, GR_P = GR_T + 2;  // LDS rows of 130 doubles: [k][i]
typedef double f64x4g __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void opq_gram_kernel(const float* __restrict__ X, const float* __restrict__ Y,
                                                         int64_t n, int d, int64_t rows_per_split, int ctiles,
                                                         double* __restrict__ part) {
    __shared__ double As[2][GR_K * GR_P];
    __shared__ double Bs[2][GR_K * GR_P];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int tile = blockIdx.x, sp = blockIdx.y;
    const int i0 = (tile / ctiles) * GR_T, j0 = (tile % ctiles) * GR_T;
    const int64_t ra = (int64_t)sp * rows_per_split;
    const int64_t rb = min(n, ra + rows_per_split);
    f64x4g acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f64x4g){0.0, 0.0, 0.0, 0.0};
    // staging: thread t loads rows k = t >> 4 of the 16-row step, columns 8 (t & 15) .. +7 of the
    // tile (two float4 of X, two of Y); out-of-range rows / columns read as 0
    const int kr = tid >> 4, cc = 8 * (tid & 15);
    float xa[8], yb[8];
    auto gload = [&](int64_t r) __attribute__((always_inline)) {
        const int64_t row = r + kr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int ci = i0 + cc + u, cj = j0 + cc + u;
            xa[u] = (row < rb && ci < d) ? X[row * d + ci] : 0.0f;
            yb[u] = (row < rb && cj < d) ? Y[row * d + cj] : 0.0f;
        }
    };
    auto sstore = [&](int st) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            As[st][kr * GR_P + cc + u] = (double)xa[u];
            Bs[st][kr * GR_P + cc + u] = (double)yb[u];
        }
    };
    const int64_t nk = (rb - ra + GR_K - 1) / GR_K;
    if (nk <= 0) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int i = i0 + wr * 64 + a * 16 + (l >> 4) + 4 * g, j = j0 + wc * 64 + b * 16 + (l & 15);
                    if (i < d && j < d) part[((int64_t)sp * d + i) * d + j] = 0.0;
                }
        return;
    }
    gload(ra);
    sstore(0);
    __syncthreads();
    const int fi = l & 15, fk = l >> 4;
    for (int64_t ks = 0; ks < nk; ++ks) {
        const int st = (int)(ks & 1);
        if (ks + 1 < nk) gload(ra + (ks + 1) * GR_K);
#pragma unroll
        for (int k4 = 0; k4 < GR_K; k4 += 4) {
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) af[a] = As[st][(k4 + fk) * GR_P + wr * 64 + a * 16 + fi];
#pragma unroll
            for (int b = 0; b < 4; ++b) bf[b] = Bs[st][(k4 + fk) * GR_P + wc * 64 + b * 16 + fi];
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
                const int i = i0 + wr * 64 + a * 16 + fk + 4 * g, j = j0 + wc * 64 + b * 16 + fi;
                if (i < d && j < d) part[((int64_t)sp * d + i) * d + j] = acc[a][b][g];
            }
}

__global__ __launch_bounds__(256) void opq_gram_reduce_kernel(const double* __restrict__ part, int splits, int64_t dd,
                                                                double* __restrict__ G) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= dd) return;
    double s = part[e];
    for (int p = 1; p < splits; ++p) s += part[(int64_t)p * dd + e];
    G[e] = s;
}

int gram_splits(int64_t n, int d) {
    const int64_t tiles = ceil_div(d, GR_T) * ceil_div(d, GR_T);
    int64_t s = std::max<int64_t>(1, ceil_div(512, tiles));          // >= 2 rounds of workgroups
    s = std::min<int64_t>(s, std::max<int64_t>(1, ceil_div(n, 4 * GR_K)));  // >= 4 K steps each
    return (int)std::min<int64_t>(s, 64);
}

template <class T, int WR, int WC, int RB, int CB>
int launch_split(const float* x, int64_t n, int d, const float* rs, const _Float16* bimg, const float* hdr, float* y,
                 hipStream_t st) {
    static_assert(T::SMEM <= 160 * 1024, "LDS");
    auto kern = opq_split_gemm_kernel<WR, WC, RB, CB>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, T::SMEM);
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "opq_split_gemm: %s", hipGetErrorString(e));
    const int64_t ct = ceil_div(d, T::TN), tiles = ceil_div(n, T::TM) * ct;
    MIVQ_REQUIRE(tiles < ((int64_t)1 << 31), MIVQ_ERR_UNSUPPORTED, "opq_rotate_prepared: n=%lld too large for one call",
                 (long long)n);
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(T::NT), T::SMEM, st, x, n, d, rs, bimg, hdr, y, ct);
    return check_launch("opq_split_gemm");
}

size_t prep_bytes(int32_t d) { return 256 + (size_t)2 * d * d * sizeof(_Float16); }

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" int mivq_opq_rotate(const float* x, int64_t n, int32_t d, const float* A, int32_t transpose, float* y,
                               void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "opq_rotate: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(transpose == 0 || transpose == 1, MIVQ_ERR_INVALID, "opq_rotate: transpose must be 0 or 1");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && A && y && x != y, MIVQ_ERR_INVALID, "opq_rotate: null or aliased pointer");
    const dim3 grid((unsigned)ceil_div(n, BM), (unsigned)ceil_div(d, BN));
    hipLaunchKernelGGL(opq_gemm_kernel, grid, dim3(256), 0, as_stream(stream), x, n, d, A, transpose, y);
    return check_launch("opq_rotate");
}

extern "C" size_t mivq_opq_prep_bytes(int32_t d) { return d > 0 && d % 8 == 0 ? prep_bytes(d) : 0; }

extern "C" int mivq_opq_prepare(const float* A, int32_t d, int32_t transpose, void* prep, void* stream) {
    MIVQ_REQUIRE(d > 0, MIVQ_ERR_INVALID, "opq_prepare: bad size d=%d", d);
    MIVQ_REQUIRE(d % 8 == 0, MIVQ_ERR_UNSUPPORTED, "opq_prepare: d=%d must be a multiple of 8 (use mivq_opq_rotate)", d);
    MIVQ_REQUIRE(transpose == 0 || transpose == 1, MIVQ_ERR_INVALID, "opq_prepare: transpose must be 0 or 1");
    MIVQ_REQUIRE(A && prep, MIVQ_ERR_INVALID, "opq_prepare: null pointer");
    hipStream_t st = as_stream(stream);
    float* hdr = static_cast<float*>(prep);
    _Float16* bimg = reinterpret_cast<_Float16*>(static_cast<unsigned char*>(prep) + 256);
    hipLaunchKernelGGL(opq_absmax_kernel, dim3(1), dim3(1024), 0, st, A, (int64_t)d * d, hdr);
    int rc = check_launch("opq_absmax");
    if (rc) return rc;
    hipLaunchKernelGGL(opq_split_b_kernel, dim3((unsigned)ceil_div((int64_t)d * d, 256)), dim3(256), 0, st, A, d,
                       transpose, hdr, bimg);
    return check_launch("opq_split_b");
}

// Rows per GEMM launch (keeps the tile count of one launch far below 2^31).
constexpr int64_t kOpqChunk = (int64_t)1 << 20;

extern "C" size_t mivq_opq_rotate_workspace_bytes(int64_t n, int32_t d) {
    if (n <= 0 || d <= 0) return 0;
    return align_up((size_t)n * sizeof(float), 256);  // the row scales
}

extern "C" int mivq_opq_rotate_prepared(const float* x, int64_t n, int32_t d, const void* prep, void* workspace,
                                        size_t workspace_bytes, float* y, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "opq_rotate_prepared: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(d % 8 == 0, MIVQ_ERR_UNSUPPORTED, "opq_rotate_prepared: d=%d must be a multiple of 8", d);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && prep && y && x != y, MIVQ_ERR_INVALID, "opq_rotate_prepared: null or aliased pointer");
    MIVQ_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(prep) % 16 == 0,
                 MIVQ_ERR_INVALID, "opq_rotate_prepared: x and prep must be 16-byte aligned");
    const size_t need = mivq_opq_rotate_workspace_bytes(n, d);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "opq_rotate_prepared: workspace %zu < %zu",
                 workspace_bytes, need);
    MIVQ_REQUIRE(reinterpret_cast<uintptr_t>(workspace) % 16 == 0, MIVQ_ERR_INVALID,
                 "opq_rotate_prepared: workspace must be 16-byte aligned");
    // the split GEMM's buffer offsets are 32-bit: the B image is 4 d^2 bytes
    MIVQ_REQUIRE((int64_t)4 * d * d < ((int64_t)1 << 31), MIVQ_ERR_UNSUPPORTED,
                 "opq_rotate_prepared: d=%d too large", d);
    hipStream_t st = as_stream(stream);
    float* rs = static_cast<float*>(workspace);
    const float* hdr = static_cast<const float*>(prep);
    const _Float16* bimg = reinterpret_cast<const _Float16*>(static_cast<const unsigned char*>(prep) + 256);
    for (int64_t c0 = 0; c0 < n; c0 += kOpqChunk) {
        const int64_t cn = std::min(kOpqChunk, n - c0);
        const float* xc = x + c0 * d;
        float* yc = y + c0 * d;
        hipLaunchKernelGGL(opq_row_scale_kernel, dim3((unsigned)ceil_div(cn, 4)), dim3(256), 0, st, xc, cn, d,
                           rs + c0);
        int rc = check_launch("opq_row_scale");
        if (rc) return rc;
        // 256 x 256 tiles (512 threads, 160 KiB) wherever a row block spans at least one such
        // tile; the 128 x 128 kernel for narrow matrices (round 5: 128 x 128 everywhere, two
        // workgroups per CU whose barriers are independent: 18.0 vs 14.6 ms, profiles/r05_s27)
        if (d >= 256 && cn >= 256)
            rc = launch_split<TileL, 4, 2, 2, 4>(xc, cn, d, rs + c0, bimg, hdr, yc, st);
        else
            rc = launch_split<TileS, 2, 2, 2, 2>(xc, cn, d, rs + c0, bimg, hdr, yc, st);
        if (rc) return rc;
    }
    return MIVQ_OK;
}

extern "C" size_t mivq_opq_gram_workspace_bytes(int64_t n, int32_t d) {
    if (n <= 0 || d <= 0) return 0;
    return (size_t)gram_splits(n, d) * (size_t)d * d * sizeof(double);
}

extern "C" int mivq_opq_gram(const float* x, const float* y, int64_t n, int32_t d, void* workspace,
                             size_t workspace_bytes, double* G, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "opq_gram: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(G && (n == 0 || (x && y)), MIVQ_ERR_INVALID, "opq_gram: null pointer");
    hipStream_t st = as_stream(stream);
    const int64_t dd = (int64_t)d * d;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(G, 0, (size_t)dd * sizeof(double), st);
        return e == hipSuccess ? MIVQ_OK : set_error(MIVQ_ERR_HIP, "opq_gram: %s", hipGetErrorString(e));
    }
    const size_t need = mivq_opq_gram_workspace_bytes(n, d);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "opq_gram: workspace %zu < %zu",
                 workspace_bytes, need);
    const int splits = gram_splits(n, d);
    const int ct = (int)ceil_div(d, GR_T);
    const int64_t rps = ceil_div(n, splits);
    double* part = static_cast<double*>(workspace);
    hipLaunchKernelGGL(opq_gram_kernel, dim3((unsigned)(ct * ct), (unsigned)splits), dim3(256), 0, st, x, y, n, d, rps,
                       ct, part);
    int rc = check_launch("opq_gram");
    if (rc) return rc;
    hipLaunchKernelGGL(opq_gram_reduce_kernel, dim3((unsigned)ceil_div(dd, 256)), dim3(256), 0, st, part, splits, dd, G);
    return check_launch("opq_gram_reduce");
}
