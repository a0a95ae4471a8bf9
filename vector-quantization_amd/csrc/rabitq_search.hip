// rabitq_search.hip — RaBitQ estimator search (faiss IndexRaBitQ.search, qb query bits) for gfx950.
//
// GPU counterpart of RaBitQIndex.search_with_scores (/root/reference/src/haag_vq/methods/
// search/rabitq_index.py:42-70: faiss.IndexRaBitQ(D, metric), .qb = 4 by default, exhaustive
// search with the RaBitQ distance estimator).  The arithmetic is spelled out in
// oracle/mivq_oracle.c (oracle_rabitq_est) and include/mivq.h; faiss is absent here, so the
// restatement defines it (parity unpinned vs faiss) and the kernels are bit-exact against it.
//
//   rabitq_qprep_kernel     one workgroup per query: r = q - c, its min / max, the qb-bit
//                           quantised r' (int8, minus 128 when qb = 8), sum r', and the
//                           per-query factors {c1, c2, c34, ||r||^2, ||q||^2, 1/sqrt(d), off}.
//   rabitq_est_mfma_kernel  d % 32 == 0, qb >= 1: the integer dot <bits, r'> of 32 codes x 32
//                           queries on v_mfma_i32_32x32x32_i8.  The sign bits are expanded to
//                           int8 {0, 1} in registers (16 bits -> 16 bytes per lane and k-step:
//                           nibble * 0x204081 & 0x01010101), the queries' int8 rows sit in LDS.
//                           Integer sums are exact, so any accumulation order gives the oracle's
//                           dot; the epilogue applies the estimator in the oracle's fp32 order.
//   rabitq_est_generic_kernel  any d / qb = 0: one thread per (query, code).
// The (nq, m) key blocks go through launch_tiled_topk (segmented top-k + running merge), the
// same selection as the exact flat search: (key, id) ascending, ties to the smaller id.
#include "mivq_common.h"
#include "topk.h"

#include <math.h>

namespace mivq {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kQfStride = 8;  // floats per query: c1, c2, c34, qc, qn, 1/sqrt(d), off, 0

__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

// One workgroup (256 threads) per query.  qq: (nq, d) int8 (q' - off), qr: (nq, d) f32 r
// (qb = 0 only), qf: (nq, kQfStride) f32.
__global__ __launch_bounds__(256) void rabitq_qprep_kernel(const float* __restrict__ q, int d,
                                                           const float* __restrict__ centroid, int qb,
                                                           int8_t* __restrict__ qq, float* __restrict__ qr,
                                                           float* __restrict__ qf) {
    __shared__ float red_lo[256], red_hi[256];
    __shared__ int red_sum;
    const int tid = threadIdx.x;
    const int64_t a = blockIdx.x;
    const float* qrow = q + a * d;
    float lo = INFINITY, hi = -INFINITY;
    for (int j = tid; j < d; j += 256) {
        const float r = __fsub_rn(qrow[j], centroid ? centroid[j] : 0.0f);
        lo = fminf(lo, r);
        hi = fmaxf(hi, r);
        if (qb == 0) qr[a * d + j] = r;
    }
    red_lo[tid] = lo;
    red_hi[tid] = hi;
    if (tid == 0) red_sum = 0;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) {
            red_lo[tid] = fminf(red_lo[tid], red_lo[tid + s]);
            red_hi[tid] = fmaxf(red_hi[tid], red_hi[tid + s]);
        }
        __syncthreads();
    }
    const float vmin = red_lo[0], vmax = red_hi[0];
    const float isd = __fdiv_rn(1.0f, sqrtf((float)d));
    float delta = 0.0f;
    const int off = qb == 8 ? 128 : 0;
    if (qb > 0) {
        const int top = (1 << qb) - 1;
        delta = __fdiv_rn(__fsub_rn(vmax, vmin), (float)top);
        const float inv_delta = delta > 0.0f ? __fdiv_rn(1.0f, delta) : 0.0f;
        int part = 0;
        for (int j = tid; j < d; j += 256) {
            const float r = __fsub_rn(qrow[j], centroid ? centroid[j] : 0.0f);
            const float t = __fmul_rn(__fsub_rn(r, vmin), inv_delta);
            int v = (int)floorf(__fadd_rn(t, 0.5f));
            v = v < 0 ? 0 : (v > top ? top : v);
            part += v;
            qq[a * d + j] = (int8_t)(v - off);
        }
        atomicAdd(&red_sum, part);  // integer: order-free
    }
    __syncthreads();
    if (tid == 0) {
        // the oracle's sequential chains
        float qc = 0.0f, qn = 0.0f;
        for (int j = 0; j < d; ++j) {
            const float r = __fsub_rn(qrow[j], centroid ? centroid[j] : 0.0f);
            qc = __builtin_fmaf(r, r, qc);
            qn = __builtin_fmaf(qrow[j], qrow[j], qn);
        }
        float c1 = 0.0f, c2 = 0.0f, c34 = 0.0f;
        if (qb > 0) {
            c1 = __fmul_rn(__fmul_rn(2.0f, delta), isd);
            c2 = __fmul_rn(__fmul_rn(2.0f, vmin), isd);
            c34 = __fmul_rn(isd, __fadd_rn(__fmul_rn(delta, (float)red_sum), __fmul_rn((float)d, vmin)));
        }
        float* f = qf + a * kQfStride;
        f[0] = c1; f[1] = c2; f[2] = c34; f[3] = qc; f[4] = qn; f[5] = isd; f[6] = (float)off; f[7] = 0.0f;
    }
}

// The estimator epilogue shared by both kernels (oracle order).
__device__ __forceinline__ float rabitq_key(float fd, float f0, float f1, float qc, float qn, bool ip) {
    const float pre = __builtin_fmaf(__fmul_rn(-2.0f, f1), fd, __fadd_rn(f0, qc));
    return ip ? __fmul_rn(0.5f, __fsub_rn(pre, qn)) : pre;
}

__device__ __forceinline__ float load_f32(const unsigned char* p) {
    uint32_t u = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) u |= (uint32_t)p[b] << (8 * b);
    return __uint_as_float(u);
}

constexpr int kEstTiles = 8;  // 32-code tiles per wave (each workgroup: 4 waves x 256 codes)

// Grid (ceil(m / 1024), ceil(nq / 32)), 256 threads.  LDS: the 32 query rows (int8, pitch
// d + 16), per wave one 32-code staging tile (32 x cs bytes) and the codes' popcounts.
__global__ __launch_bounds__(256) void rabitq_est_mfma_kernel(const uint8_t* __restrict__ codes, int64_t m, int d,
                                                              const int8_t* __restrict__ qq,
                                                              const float* __restrict__ qf, int64_t nq, int metric,
                                                              float* __restrict__ buf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nb = d >> 3, cs = nb + 8;  // d % 32 == 0: cs % 4 == 0
    const int QP = d + 16;
    int8_t* qs = reinterpret_cast<int8_t*>(smem);
    unsigned char* cst_all = smem + 32 * QP;
    int* pop_all = reinterpret_cast<int*>(cst_all + 4 * 32 * cs);
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
    const int64_t q0 = (int64_t)blockIdx.y * 32;
    const int qch = d >> 4;
    for (int e = tid; e < 32 * qch; e += 256) {
        const int row = e / qch, c = e - row * qch;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q0 + row < nq) v = *reinterpret_cast<const uint4*>(qq + (q0 + row) * d + 16 * c);
        *reinterpret_cast<uint4*>(qs + row * QP + 16 * c) = v;
    }
    __syncthreads();
    const int64_t qa = q0 + r;
    const bool qok = qa < nq;
    float c1 = 0.0f, c2 = 0.0f, c34 = 0.0f, qc = 0.0f, qn = 0.0f;
    int off = 0;
    if (qok) {
        const float* f = qf + qa * kQfStride;
        c1 = f[0]; c2 = f[1]; c34 = f[2]; qc = f[3]; qn = f[4]; off = (int)f[6];
    }
    const bool ip = metric == MIVQ_METRIC_INNER_PRODUCT;
    unsigned char* cst = cst_all + w * 32 * cs;
    int* pops = pop_all + w * 64;
    const int nks = d >> 5;
    const int ndw = 8 * cs;  // dwords per 32-code tile
    for (int t = 0; t < kEstTiles; ++t) {
        const int64_t cb = ((int64_t)blockIdx.x * 4 * kEstTiles + w * kEstTiles + t) * 32;
        if (cb >= m) break;
        const int nc = (int)min<int64_t>(32, m - cb);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(codes + cb * cs);
        const int nvalid = nc * cs / 4;
        for (int e = l; e < ndw; e += 64) reinterpret_cast<uint32_t*>(cst)[e] = e < nvalid ? src[e] : 0u;
        lds_fence();
        v16i acc = {};
        int pc = 0;
        const unsigned char* crow = cst + r * cs + 2 * h;
        for (int s = 0; s < nks; ++s) {
            const uint32_t b16 = *reinterpret_cast<const uint16_t*>(crow + 4 * s);
            pc += __builtin_popcount(b16);
            v4i av;
#pragma unroll
            for (int j = 0; j < 4; ++j) av[j] = (int)(__umul24((b16 >> (4 * j)) & 0xFu, 0x204081u) & 0x01010101u);
            const v4i bq = *reinterpret_cast<const v4i*>(qs + r * QP + 32 * s + 16 * h);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bq, acc, 0, 0, 0);
        }
        pops[2 * r + h] = pc;
        lds_fence();
        if (qok) {
            float* orow = buf + qa * m + cb;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int ci = 8 * g + 4 * h + u;  // code row of accumulator 4g + u
                    if (ci < nc) {
                        const int pop = pops[2 * ci] + pops[2 * ci + 1];
                        const int dot = acc[4 * g + u] + off * pop;
                        const unsigned char* tr = cst + ci * cs + nb;
                        const float f0 = *reinterpret_cast<const float*>(tr);
                        const float f1 = *reinterpret_cast<const float*>(tr + 4);
                        const float fd = __builtin_fmaf(c1, (float)dot, __builtin_fmaf(c2, (float)pop, -c34));
                        orow[ci] = rabitq_key(fd, f0, f1, qc, qn, ip);
                    }
                }
            }
        }
        lds_fence();  // the next tile restages cst / pops
    }
}

// Any d, any qb: thread = code, blockIdx.y = query.
__global__ __launch_bounds__(256) void rabitq_est_generic_kernel(const uint8_t* __restrict__ codes, int64_t m, int d,
                                                                 const int8_t* __restrict__ qq,
                                                                 const float* __restrict__ qr,
                                                                 const float* __restrict__ qf, int qb, int metric,
                                                                 float* __restrict__ buf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t a = blockIdx.y;
    if (i >= m) return;
    const int nb = (d + 7) >> 3, cs = nb + 8;
    const uint8_t* code = codes + i * cs;
    const float* f = qf + a * kQfStride;
    float fd;
    int pop = 0;
    if (qb > 0) {
        const int8_t* qv = qq + a * d;
        const int off = (int)f[6];
        int dot = 0;
        for (int j = 0; j < d; ++j) {
            const int b = (code[j >> 3] >> (j & 7)) & 1;
            dot += b ? (int)qv[j] + off : 0;
            pop += b;
        }
        fd = __builtin_fmaf(f[0], (float)dot, __builtin_fmaf(f[1], (float)pop, -f[2]));
    } else {
        const float* rv = qr + a * d;
        float s = 0.0f;
        for (int j = 0; j < d; ++j) s = __fadd_rn(s, ((code[j >> 3] >> (j & 7)) & 1) ? rv[j] : -rv[j]);
        fd = __fmul_rn(s, f[5]);
    }
    buf[a * m + i] = rabitq_key(fd, load_f32(code + nb), load_f32(code + nb + 4), f[3], f[4],
                                metric == MIVQ_METRIC_INNER_PRODUCT);
}

struct RqLayout {
    size_t qq, qr, qf, tiled, total;
};

RqLayout rq_layout(int64_t nq, int64_t n, int d, int k) {
    RqLayout L{};
    size_t off = 0;
    L.qq = off;    off = align_up(off + (size_t)nq * d, 256);
    L.qr = off;    off = align_up(off + (size_t)nq * d * 4, 256);
    L.qf = off;    off = align_up(off + (size_t)nq * kQfStride * 4, 256);
    L.tiled = off; off = align_up(off + flat_tiled_workspace_bytes(nq, n, k), 256);
    L.total = off;
    return L;
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" size_t mivq_rabitq_search_workspace_bytes(int64_t nq, int64_t n, int32_t d, int32_t k) {
    if (nq < 0 || n < 0 || d <= 0 || k <= 0) return 0;
    return rq_layout(nq, n, d, k).total;
}

extern "C" int mivq_rabitq_search(const uint8_t* codes, int64_t n, int32_t d, const float* centroid, const float* q,
                                  int64_t nq, int32_t qb, int32_t metric, int32_t k, int64_t id_offset,
                                  void* workspace, size_t workspace_bytes, float* dists, uint32_t* ids,
                                  void* stream) {
    MIVQ_REQUIRE(n >= 0 && nq >= 0 && d > 0, MIVQ_ERR_INVALID, "rabitq_search: bad sizes n=%lld nq=%lld d=%d",
                 (long long)n, (long long)nq, d);
    MIVQ_REQUIRE(k >= 1 && k <= 256, MIVQ_ERR_UNSUPPORTED, "rabitq_search: k=%d not in [1, 256]", k);
    MIVQ_REQUIRE(qb >= 0 && qb <= 8, MIVQ_ERR_UNSUPPORTED, "rabitq_search: qb=%d not in [0, 8]", qb);
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "rabitq_search: metric %d", metric);
    if (nq == 0) return MIVQ_OK;
    MIVQ_REQUIRE(q && dists && ids && workspace, MIVQ_ERR_INVALID, "rabitq_search: null pointer");
    MIVQ_REQUIRE(n == 0 || codes, MIVQ_ERR_INVALID, "rabitq_search: null codes");
    const RqLayout L = rq_layout(nq, n, d, k);
    MIVQ_REQUIRE(workspace_bytes >= L.total, MIVQ_ERR_INVALID, "rabitq_search: workspace %zu < %zu bytes",
                 workspace_bytes, L.total);
    hipStream_t st = as_stream(stream);
    unsigned char* p = static_cast<unsigned char*>(workspace);
    int8_t* qq = reinterpret_cast<int8_t*>(p + L.qq);
    float* qr = reinterpret_cast<float*>(p + L.qr);
    float* qf = reinterpret_cast<float*>(p + L.qf);
    hipLaunchKernelGGL(rabitq_qprep_kernel, dim3((unsigned)nq), dim3(256), 0, st, q, d, centroid, qb, qq, qr, qf);
    int rc = check_launch("rabitq_qprep");
    if (rc) return rc;
    if (n == 0) {  // sentinel lists
        hipError_t e = launch_topk_merge(nullptr, nullptr, 0, nq, k, dists, ids, st);
        return e == hipSuccess ? MIVQ_OK : set_error(MIVQ_ERR_HIP, "rabitq_search: %s", hipGetErrorString(e));
    }
    const bool mfma = qb > 0 && (d % 32) == 0 && (reinterpret_cast<uintptr_t>(codes) % 4) == 0;
    const size_t smem = (size_t)32 * (d + 16) + (size_t)4 * 32 * (d / 8 + 8) + 4 * 64 * sizeof(int);
    if (mfma && smem > 160 * 1024) return set_error(MIVQ_ERR_UNSUPPORTED, "rabitq_search: d=%d too large", d);
    if (mfma) {
        hipError_t e = hipFuncSetAttribute((const void*)rabitq_est_mfma_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "rabitq_search: %s", hipGetErrorString(e));
    }
    const int nbytes = (d + 7) / 8 + 8;
    const hipError_t e = launch_tiled_topk(
        nq, n, k, id_offset, p + L.tiled, dists, ids, st, [&](int64_t c0, int64_t m, float* buf) {
            const uint8_t* cc = codes + c0 * nbytes;
            if (mfma)
                hipLaunchKernelGGL(rabitq_est_mfma_kernel, dim3((unsigned)ceil_div(m, 4 * kEstTiles * 32),
                                                                (unsigned)ceil_div(nq, 32)),
                                   dim3(256), smem, st, cc, m, d, qq, qf, nq, metric, buf);
            else
                hipLaunchKernelGGL(rabitq_est_generic_kernel, dim3((unsigned)ceil_div(m, 256), (unsigned)nq),
                                   dim3(256), 0, st, cc, m, d, qq, qr, qf, qb, metric, buf);
            return hipGetLastError();
        });
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "rabitq_search: %s", hipGetErrorString(e));
    return MIVQ_OK;
}
