// pq_encode_cs.hip — codebook-stationary fp16-MFMA PQ encode with exact re-check (gfx950).
//
// The hot kernel of ProductQuantizer.compress (/root/reference/src/haag_vq/methods/
// product_quantization.py:76-80 -> faiss ProductQuantizer::compute_codes).  Codes equal the
// canonical encode of include/mivq.h bit for bit; the filter window W is derived in pq.hip
// (pq_prep_mfma_kernel / the comment above pq_encode_mfma_kernel).
//
// Work decomposition.  Workgroup (chunk, m) owns subspace m for rows [chunk*R, (chunk+1)*R)
// (blockIdx = chunk*M + m).  The number of chunks is chosen so that the grid is a whole
// number of waves of workgroups over the CUs (one workgroup per CU: the LDS below).  For the
// workgroup's whole life LDS holds
//   cimg : the fp16 operand image of C_m, fragment order (8*KS KiB; ds_read_b128, no conflicts)
//   c32  : the exact fp32 C_m, rows padded to dsub+4 floats (conflict-free 16-B row reads)
//   hb   : the scaled accumulator init -|c|^2 * sigma * tau / 2
//   cnl  : the canonical norms |c|^2 of C_m
//   xsc  : one 2*HALF-float row scratch per wave (full canonical scans)
// 8 waves (2 per SIMD) each stream 32-row blocks ("vb"): 16-B loads of x straight to
// registers with the next vb prefetched (ping-pong register sets, no copies), 8*KS
// v_mfma_f32_32x32x16_f16 per vb, a packed top-3 per lane (one v_and_or_b32 + max + 2 med3
// per score), then
//   1 candidate in the window  -> done;
//   2 candidates               -> canonical fmaf chains of both, split across the lane pair,
//                                 centroids from c32, x from the registers;
//   >= 3, or a row the window cannot bound (fp16 overflow, NaN, tiny) -> canonical scan of all
//                                 256 centroids by the whole wave from c32.
// The only global loads inside the loop are the x prefetches: vmcnt retires in order, so any
// later global load (a norm, a re-read of x) would make the wave wait for the prefetch too.
// Codes go to a transposed (M, n) scratch (32 contiguous bytes per vb); a transpose kernel
// writes the (n, M) layout.
#include "pq_internal.h"

#include <math.h>

namespace mivq {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 8;  // 512 threads, 2 waves per SIMD
constexpr int kThreads = kWaves * 64;

// Keeps the three largest of a stream of packed scores.  Inline asm because the compiler
// quiets every packed value (v_max_f32 v, v, v) before fmaxf / fmed3 in IEEE mode: the
// values come out of integer bit operations.  They are never NaN here (a row whose scores
// could be is routed to the exact scan by the `bad` test), so the quieting is pure cost.
// The operands are plain VALU results, so no MFMA hazard is hidden from the compiler.
__device__ __forceinline__ void top3_insert(float& t1, float& t2, float& t3, float v) {
    float n1, n2, n3;
    asm("v_max_f32 %0, %1, %2" : "=v"(n1) : "v"(t1), "v"(v));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(n2) : "v"(t1), "v"(t2), "v"(v));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(n3) : "v"(t2), "v"(t3), "v"(v));
    t1 = n1; t2 = n2; t3 = n3;
}

// (v & 0xFFFFFF00) | k in ONE v_and_or_b32: gfx950's VOP3 takes no literal and one scalar
// operand, so the mask must live in a VGPR (opaque_mask hides the constant from the
// folder) and k comes from an SGPR.  Plain C, not inline asm: the compiler must see the
// read of the MFMA result to insert the MFMA->VALU hazard wait states.
__device__ __forceinline__ uint32_t opaque_mask() {
    uint32_t v;
    asm volatile("v_mov_b32 %0, 0xffffff00" : "=v"(v));
    return v;
}

__device__ __forceinline__ float pack_idx(float v, uint32_t vmask, uint32_t k) {
    return __uint_as_float((__float_as_uint(v) & vmask) | k);
}

__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t cvt2(float a, float b) {
    const half2v h = __builtin_convertvector((float2v){a, b}, half2v);
    return __builtin_bit_cast(uint32_t, h);
}

// V: profiling variants (tools/cs_variants.hip), 0 in the library.  Bits drop work and
// produce wrong codes: 1 the 2-candidate checks, 2 the full scans, 4 the top-3 (max only),
// 8 the MFMAs, 16 the whole filter, 32 all but the first 32 centroids.
template <int KS, int V = 0>
struct CsCtx {
    static constexpr int HALF = 8 * KS;
    static constexpr int NC = HALF / 4;  // float4 per lane-half
    const float* xsub;                   // x + m*dsub + h_begin
    int64_t d, n, r1;
    const half8* cimg;
    const float *c32, *hb, *cnl;
    float* scratch;
    uint8_t* codesT;
    int LDR, dsub, h_begin, nchunk, l, r, h, m;
    float sigma, wa, wb;
    uint32_t vmask;

    __device__ __forceinline__ void load(int64_t vb, float4* dst) const {
        const int64_t row = vb * 32 + r;
        const bool ok = row < r1;
        const float* src = xsub + (ok ? row : 0) * d;
#pragma unroll
        for (int i = 0; i < NC; ++i)
            dst[i] = (ok && i < nchunk) ? *reinterpret_cast<const float4*>(src + 4 * i)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }

    // Encode vb whose x half-rows are resident in xc; the loads of vb_next go into xn first.
    __device__ __forceinline__ void step(int64_t vb, const float4* xc, int64_t vb_next, int64_t vb_end,
                                         float4* xn) const {
        half8 bf[KS];
        float xx = 0.0f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const float4 a = xc[2 * ks], b = xc[2 * ks + 1];
            xx = __builtin_fmaf(a.x, a.x, xx); xx = __builtin_fmaf(a.y, a.y, xx);
            xx = __builtin_fmaf(a.z, a.z, xx); xx = __builtin_fmaf(a.w, a.w, xx);
            xx = __builtin_fmaf(b.x, b.x, xx); xx = __builtin_fmaf(b.y, b.y, xx);
            xx = __builtin_fmaf(b.z, b.z, xx); xx = __builtin_fmaf(b.w, b.w, xx);
            const uint32_t p0 = cvt2(sigma * a.x, sigma * a.y), p1 = cvt2(sigma * a.z, sigma * a.w);
            const uint32_t p2 = cvt2(sigma * b.x, sigma * b.y), p3 = cvt2(sigma * b.z, sigma * b.w);
            bf[ks] = __builtin_bit_cast(half8, make_uint4(p0, p1, p2, p3));
        }
        if (vb_next < vb_end) load(vb_next, xn);
        xx += __shfl_xor(xx, 32);

        float t1 = -INFINITY, t2 = -INFINITY, t3 = -INFINITY;
#pragma unroll
        for (int cb = 0; cb < ((V & 16) ? 0 : (V & 32) ? 1 : 8); ++cb) {
            half8 a[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) a[ks] = cimg[(cb * KS + ks) * 64 + l];
            floatx16 acc;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 hv = *reinterpret_cast<const float4*>(hb + cb * 32 + 8 * q + 4 * h);
                acc[4 * q + 0] = hv.x; acc[4 * q + 1] = hv.y;
                acc[4 * q + 2] = hv.z; acc[4 * q + 3] = hv.w;
            }
#pragma unroll
            for (int ks = 0; ks < ((V & 8) ? 0 : KS); ++ks) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks], bf[ks], acc, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if constexpr ((V & 4) != 0) asm("v_max_f32 %0, %0, %1" : "+v"(t1) : "v"(pack_idx(acc[i], vmask, (uint32_t)(cb * 32 + (i & 3) + 8 * (i >> 2)))));
                else top3_insert(t1, t2, t3, pack_idx(acc[i], vmask, (uint32_t)(cb * 32 + (i & 3) + 8 * (i >> 2))));
        }
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
        const float Xs = sigma * sqrtf(xx) * (1.0f + 1e-5f);
        const float W = wa * Xs + wb;
        const float thr = t1 - W;
        const bool bad = !(Xs < 65000.0f) || !(Xs > 1e-12f) || !isfinite(t1) || !isfinite(W);
        const int ncand = bad ? 3 : 1 + (t2 >= thr) + (t3 >= thr);
        const int k1 = (int)(__float_as_uint(t1) & 0xFFu);
        const int k2 = (int)(__float_as_uint(t2) & 0xFFu);
        int code = k1;
        if constexpr ((V & 16) != 0) {  // keep the loads and conversions alive
            uint32_t z = 0;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const uint4 u = __builtin_bit_cast(uint4, bf[ks]);
                z ^= u.x ^ u.y ^ u.z ^ u.w;
            }
            code ^= (int)(z & 0xFF);
        }
        if (!(V & 1) && __any(ncand == 2)) {
            const bool need = (ncand == 2);
            float carry = 0.0f, dot1 = 0.0f, dot2 = 0.0f;
#pragma unroll
            for (int phase = 0; phase < 3; ++phase) {
                // h0: k1 first half, then k2 first half; h1: k1 second half, then k2's
                const bool active = need && ((h == 0 && phase < 2) || (h == 1 && phase > 0));
                const int kk = (h == 0) ? (phase == 0 ? k1 : k2) : (phase == 1 ? k1 : k2);
                float acc = (h == 0) ? 0.0f : carry;
                if (active) {
                    const float* crow = c32 + kk * LDR + h_begin;
#pragma unroll
                    for (int i = 0; i < NC; ++i) {
                        if (i < nchunk) {
                            const float4 cv = *reinterpret_cast<const float4*>(crow + 4 * i);
                            acc = __builtin_fmaf(xc[i].x, cv.x, acc);
                            acc = __builtin_fmaf(xc[i].y, cv.y, acc);
                            acc = __builtin_fmaf(xc[i].z, cv.z, acc);
                            acc = __builtin_fmaf(xc[i].w, cv.w, acc);
                        }
                    }
                }
                const float other = __shfl_xor(acc, 32);
                if (h == 1) {
                    carry = other;
                    if (phase == 1) dot1 = acc;
                    if (phase == 2) dot2 = acc;
                }
            }
            if (need && h == 1) {
                const float s1 = __builtin_fmaf(-2.0f, dot1, cnl[k1]);
                const float s2 = __builtin_fmaf(-2.0f, dot2, cnl[k2]);
                code = (s2 < s1 || (s2 == s1 && k2 < k1)) ? k2 : k1;
            }
            code = __shfl(code, (l & 31) + 32);
        }
        unsigned long long full = (V & 2) ? 0ull : __ballot(ncand >= 3 && h == 0);
        while (full) {
            const int rr = __builtin_ctzll(full);
            full &= full - 1;
            if (r == rr) {
#pragma unroll
                for (int i = 0; i < NC; ++i) *reinterpret_cast<float4*>(scratch + h_begin + 4 * i) = xc[i];
            }
            lds_fence();
            float acc4[4] = {0.f, 0.f, 0.f, 0.f};
            for (int t = 0; t < dsub; t += 4) {
                const float4 xv = *reinterpret_cast<const float4*>(scratch + t);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float4 cv = *reinterpret_cast<const float4*>(c32 + (l + 64 * j) * LDR + t);
                    acc4[j] = __builtin_fmaf(xv.x, cv.x, acc4[j]);
                    acc4[j] = __builtin_fmaf(xv.y, cv.y, acc4[j]);
                    acc4[j] = __builtin_fmaf(xv.z, cv.z, acc4[j]);
                    acc4[j] = __builtin_fmaf(xv.w, cv.w, acc4[j]);
                }
            }
            float bs = INFINITY;
            int bk = l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float s = __builtin_fmaf(-2.0f, acc4[j], cnl[l + 64 * j]);
                if (s < bs) { bs = s; bk = l + 64 * j; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float os = __shfl_xor(bs, o);
                const int ok = __shfl_xor(bk, o);
                if (os < bs || (os == bs && ok < bk)) { bs = os; bk = ok; }
            }
            if (r == rr) code = (bs < INFINITY) ? bk : 0;
            lds_fence();
        }
        if (h == 0) {
            const int64_t row = vb * 32 + r;
            if (row < r1) codesT[(int64_t)m * n + row] = (uint8_t)code;
        }
    }
};

template <int KS, int V = 0>
__global__ __launch_bounds__(kThreads, 2) void pq_encode_cs_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub, int64_t rows_per_wg,
    const float* __restrict__ C, const float* __restrict__ cn, const half8* __restrict__ img,
    const float* __restrict__ hinit, const float4* __restrict__ bnd, uint8_t* __restrict__ codesT) {
    constexpr int FR = 8 * KS * 64;
    constexpr int HALF = 8 * KS;
    constexpr int NC = HALF / 4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int LDR = dsub + 4;
    half8* cimg = reinterpret_cast<half8*>(smem);
    float* c32 = reinterpret_cast<float*>(smem + FR * 16);
    float* hb = c32 + 256 * LDR;
    float* cnl = hb + 256;
    float* xsc = cnl + 256;

    const int tid = threadIdx.x;
    const int w = tid >> 6;
    const int m = (int)(blockIdx.x % M);
    const int64_t r0 = (int64_t)(blockIdx.x / M) * rows_per_wg;
    const int64_t r1 = min(n, r0 + rows_per_wg);
    if (r0 >= r1) return;

    {  // stage the subspace's codebook once per workgroup
        const half8* src = img + (int64_t)m * FR;
        for (int f = tid; f < FR; f += kThreads) cimg[f] = src[f];
        const float* Cm = C + (int64_t)m * 256 * dsub;
        const int q4 = dsub >> 2;
        for (int e = tid; e < 256 * q4; e += kThreads) {
            const int k = e / q4, q = e % q4;
            *reinterpret_cast<float4*>(c32 + k * LDR + 4 * q) =
                *reinterpret_cast<const float4*>(Cm + (int64_t)k * dsub + 4 * q);
        }
        if (tid < 256) {
            hb[tid] = hinit[(int64_t)m * 256 + tid];
            cnl[tid] = cn[(int64_t)m * 256 + tid];
        }
    }
    __syncthreads();

    CsCtx<KS, V> c;
    c.l = tid & 63;
    c.r = c.l & 31;
    c.h = c.l >> 5;
    c.m = m;
    c.d = d;
    c.n = n;
    c.r1 = r1;
    c.dsub = dsub;
    c.LDR = LDR;
    c.h_begin = c.h * HALF;
    c.nchunk = max(0, min(HALF, dsub - c.h_begin)) >> 2;
    c.xsub = x + (int64_t)m * dsub + c.h_begin;
    c.cimg = cimg;
    c.c32 = c32;
    c.hb = hb;
    c.cnl = cnl;
    c.scratch = xsc + w * 2 * HALF;
    c.codesT = codesT;
    const float4 bm = bnd[m];
    c.sigma = bm.x;
    c.wa = bm.y;
    c.wb = bm.z;
    c.vmask = opaque_mask();

    const int64_t vb_end = (r1 + 31) / 32;
    int64_t vb = r0 / 32 + w;
    float4 xa[NC], xb[NC];
    if (vb < vb_end) c.load(vb, xa);
    // two vbs per trip so that the prefetch target alternates between xa and xb
    for (; vb < vb_end; vb += 2 * kWaves) {
        c.step(vb, xa, vb + kWaves, vb_end, xb);
        if (vb + kWaves >= vb_end) break;
        c.step(vb + kWaves, xb, vb + 2 * kWaves, vb_end, xa);
    }
}

// (M, n) -> (n, M): one block per 256 rows, the tile goes through LDS.
__global__ __launch_bounds__(256) void pq_transpose_codes_kernel(const uint8_t* __restrict__ codesT, int64_t n, int M,
                                                                 uint8_t* __restrict__ codes) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];  // [256][M]
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    const int rows = (int)min<int64_t>(256, n - r0);
    for (int e = threadIdx.x; e < M * 256; e += 256) {
        const int mm = e / 256, rr = e % 256;
        if (rr < rows) tile[rr * M + mm] = codesT[(int64_t)mm * n + r0 + rr];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < rows * M; e += 256) codes[r0 * M + e] = tile[e];
}

int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    return cus;
}

// Chunk count for one workgroup per CU at a time: minimise the rounds of workgroups per row
// (ceil(chunks*M / CUs) / chunks), preferring fewer chunks, with at least 32*kWaves rows each.
int64_t pick_chunks(int64_t n, int M, int cus) {
    const int64_t cmax = std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 32 * kWaves), 4 * (int64_t)cus));
    int64_t best = 1;
    double best_cost = 1e300;
    for (int64_t c = 1; c <= cmax; ++c) {
        const double cost = (double)ceil_div(c * M, (int64_t)cus) / (double)c;
        if (cost < best_cost * (1.0 - 1e-9)) { best_cost = cost; best = c; }
    }
    return best;
}

template <int KS, int V = 0>
hipError_t launch_ks(const float* x, int64_t n, int d, int M, int dsub, const float* C, const float* cn,
                     const void* img, const float* hinit, const void* bnd, uint8_t* codesT, hipStream_t st) {
    const int smem = cs_smem_bytes(KS, dsub);
    auto kern = pq_encode_cs_kernel<KS, V>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    if (e != hipSuccess) return e;
    static thread_local int cus = 0;
    if (!cus) cus = device_cus();
    const int64_t chunks = pick_chunks(n, M, cus);
    const int64_t R = align_up(ceil_div(n, chunks), (int64_t)32);
    const int64_t grid = ceil_div(n, R) * M;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), smem, st, x, n, d, M, dsub, R, C, cn,
                       static_cast<const half8*>(img), hinit, static_cast<const float4*>(bnd), codesT);
    return hipGetLastError();
}

}  // namespace

int cs_smem_bytes(int KS, int dsub) {
    return 8 * KS * 64 * 16 + 256 * (dsub + 4) * 4 + 2 * 256 * 4 + kWaves * 2 * 8 * KS * 4;
}

hipError_t launch_pq_encode_cs(int KS, const float* x, int64_t n, int d, int M, int dsub, const float* C,
                               const float* cn, const void* img, const float* hinit, const void* bnd,
                               uint8_t* codesT, uint8_t* codes, hipStream_t st) {
    hipError_t e = hipErrorInvalidValue;
    switch (KS) {
        case 1: e = launch_ks<1>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        case 2: e = launch_ks<2>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        case 3: e = launch_ks<3>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        case 4: e = launch_ks<4>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        case 5: e = launch_ks<5>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        case 6: e = launch_ks<6>(x, n, d, M, dsub, C, cn, img, hinit, bnd, codesT, st); break;
        default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pq_transpose_codes_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), (size_t)256 * M, st,
                       codesT, n, M, codes);
    return hipGetLastError();
}

}  // namespace mivq
