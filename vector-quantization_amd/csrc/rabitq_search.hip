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

#include <type_traits>

namespace mivq {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));  // code rows are 4-B aligned

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
    if (tid < 64) {
        // the oracle's sequential chains, both in lane 0, over the row staged in LDS 1024
        // elements at a time by the whole wave: the global loads of a piece are in flight at
        // once instead of one round trip per element of a serial loop
        __shared__ __attribute__((aligned(16))) float s_q[1024], s_c[1024];
        float qc = 0.0f, qn = 0.0f;
        for (int j0 = 0; j0 < d; j0 += 1024) {
            const int nj = min(1024, d - j0);
            for (int t = tid; t < nj; t += 64) {
                s_q[t] = qrow[j0 + t];
                s_c[t] = centroid ? centroid[j0 + t] : 0.0f;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's own LDS stores
            __builtin_amdgcn_wave_barrier();
            if (tid == 0) {  // both chains in lane 0, 16-B LDS reads running ahead of the fmas
                int t = 0;
#pragma unroll 4
                for (; t + 4 <= nj; t += 4) {
                    const float4 qv = *reinterpret_cast<const float4*>(s_q + t);
                    const float4 cv = *reinterpret_cast<const float4*>(s_c + t);
                    float r = __fsub_rn(qv.x, cv.x); qc = __builtin_fmaf(r, r, qc); qn = __builtin_fmaf(qv.x, qv.x, qn);
                    r = __fsub_rn(qv.y, cv.y); qc = __builtin_fmaf(r, r, qc); qn = __builtin_fmaf(qv.y, qv.y, qn);
                    r = __fsub_rn(qv.z, cv.z); qc = __builtin_fmaf(r, r, qc); qn = __builtin_fmaf(qv.z, qv.z, qn);
                    r = __fsub_rn(qv.w, cv.w); qc = __builtin_fmaf(r, r, qc); qn = __builtin_fmaf(qv.w, qv.w, qn);
                }
                for (; t < nj; ++t) {
                    const float r = __fsub_rn(s_q[t], s_c[t]);
                    qc = __builtin_fmaf(r, r, qc);
                    qn = __builtin_fmaf(s_q[t], s_q[t], qn);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        float c1 = 0.0f, c2 = 0.0f, c34 = 0.0f;
        if (qb > 0) {
            c1 = __fmul_rn(__fmul_rn(2.0f, delta), isd);
            c2 = __fmul_rn(__fmul_rn(2.0f, vmin), isd);
            c34 = __fmul_rn(isd, __fadd_rn(__fmul_rn(delta, (float)red_sum), __fmul_rn((float)d, vmin)));
        }
        if (tid == 0) {
            float* f = qf + a * kQfStride;
            f[0] = c1; f[1] = c2; f[2] = c34; f[3] = qc; f[4] = qn; f[5] = isd; f[6] = (float)off; f[7] = 0.0f;
        }
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

constexpr int kEstWaves = 8;  // waves per workgroup (all share the query block in LDS)
constexpr int kEstTiles = 4;  // 32-code tiles per wave (each workgroup: 8 waves x 128 codes)
constexpr int kEstRegG = 24;  // 16-B groups of a code row held in registers (d <= 3072)

// Grid nqb * ceil(m / (32 kEstWaves kEstTiles)) (nqb = ceil(nq / 32)), 512 threads; the query
// block index runs fastest, so the nqb workgroups reading one chunk of codes run side by side
// and all but the first find it in L2 / MALL (the codes are read from HBM about once instead of
// once per query block).  LDS holds only the
// 32 query rows (int8, pitch d + 16), so two workgroups fit a CU up to d = 2048 and one up to
// d = 4096.  Lane (r, h) of a wave owns code r of the tile and, per 32-dim k-step s, the 16
// sign bits of dims 32s + 16h .. +16: the low (h = 0) or high half of the row's dword s, read
// straight from memory four k-steps (one 16-B load) ahead of use.  Popcounts and the two
// factors of code r move to the accumulator lanes by shuffles.
__global__ __launch_bounds__(kEstWaves * 64) void rabitq_est_mfma_kernel(
    const uint8_t* __restrict__ codes, int64_t m, int d, const int8_t* __restrict__ qq, const float* __restrict__ qf,
    int64_t nq, int metric, float* __restrict__ buf, unsigned nqb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nb = d >> 3, cs = nb + 8;  // d % 32 == 0: cs % 4 == 0
    const int QP = d + 16;
    int8_t* qs = reinterpret_cast<int8_t*>(smem);
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
    const unsigned qblk = blockIdx.x % nqb, cchunk = blockIdx.x / nqb;
    const int64_t q0 = (int64_t)qblk * 32;
    const int qch = d >> 4;
    for (int e = tid; e < 32 * qch; e += kEstWaves * 64) {
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
    const int nks = d >> 5;  // k-steps; nks % 4 handled by the dword tail
    const int8_t* qrow = qs + r * QP + 16 * h;
    const int sh = 16 * h;
    const int n4 = nks >> 2;
    // d <= 32 * 4 * kEstRegG: a tile's code bits (n4 16-B loads per lane) are all issued at once,
    // the next tile's right after the last k-step of this one (before the epilogue), so each
    // tile waits for memory about once instead of once per 16-B group
    const bool inreg = n4 <= kEstRegG;
    u32x4a4 cg[kEstRegG];
    auto tile_row = [&](int t, int& nc) -> const uint8_t* {
        const int64_t cb = (((int64_t)cchunk * kEstWaves + w) * kEstTiles + t) * 32;
        nc = (int)max<int64_t>(0, min<int64_t>(32, m - cb));
        // rows past the chunk read row 0 of the tile (in range) and are never written
        return codes + (cb + (r < nc ? r : 0)) * cs;
    };
    auto load_tile = [&](const uint8_t* crow) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < kEstRegG; ++g)
            if (g < n4) cg[g] = *reinterpret_cast<const u32x4a4*>(crow + 16 * g);
    };
    if (inreg) {
        int nc0;
        const uint8_t* row0 = tile_row(0, nc0);
        if (nc0 > 0) load_tile(row0);
    }
    for (int t = 0; t < kEstTiles; ++t) {
        const int64_t cb = (((int64_t)cchunk * kEstWaves + w) * kEstTiles + t) * 32;
        if (cb >= m) break;  // wave-uniform
        const int nc = (int)min<int64_t>(32, m - cb);
        // rows past the chunk read row 0 of the tile (in range) and are never written
        const uint8_t* crow = codes + (cb + (r < nc ? r : 0)) * cs;
        v16i acc = {};
        int pc = 0;
        auto kstep = [&](uint32_t dw, int s) __attribute__((always_inline)) {
            const uint32_t b16 = (dw >> sh) & 0xFFFFu;
            pc += __builtin_popcount(b16);
            v4i av;
#pragma unroll
            for (int j = 0; j < 4; ++j) av[j] = (int)(__umul24((b16 >> (4 * j)) & 0xFu, 0x204081u) & 0x01010101u);
            const v4i bq = *reinterpret_cast<const v4i*>(qrow + 32 * s);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bq, acc, 0, 0, 0);
        };
        if (inreg) {
#pragma unroll
            for (int g = 0; g < kEstRegG; ++g) {
                if (g < n4) {
                    kstep(cg[g][0], 4 * g + 0);
                    kstep(cg[g][1], 4 * g + 1);
                    kstep(cg[g][2], 4 * g + 2);
                    kstep(cg[g][3], 4 * g + 3);
                }
            }
        } else if (n4 > 0) {
            u32x4a4 cur = *reinterpret_cast<const u32x4a4*>(crow);  // cs % 4 == 0: 4-B aligned rows
            for (int g = 0; g < n4; ++g) {
                const u32x4a4 nxt = g + 1 < n4 ? *reinterpret_cast<const u32x4a4*>(crow + 16 * (g + 1)) : cur;
                kstep(cur[0], 4 * g + 0);
                kstep(cur[1], 4 * g + 1);
                kstep(cur[2], 4 * g + 2);
                kstep(cur[3], 4 * g + 3);
                cur = nxt;
            }
        }
        for (int s = 4 * n4; s < nks; ++s) kstep(*reinterpret_cast<const uint32_t*>(crow + 4 * s), s);
        const float fr = *reinterpret_cast<const float*>(crow + nb + 4 * h);  // h = 0: f0, h = 1: f1 of code r
        if (inreg && t + 1 < kEstTiles) {
            int nc1;
            const uint8_t* nrow = tile_row(t + 1, nc1);
            if (nc1 > 0) load_tile(nrow);
        }
        // every lane takes part in the shuffles (a bpermute from an inactive lane reads 0);
        // only the stores are guarded
        float* orow = buf + (qok ? qa : 0) * m + cb;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int ci = 8 * g + 4 * h + u;  // code row of accumulator 4g + u
                const int pop = __shfl(pc, ci) + __shfl(pc, ci + 32);
                const float f0 = __shfl(fr, ci), f1 = __shfl(fr, ci + 32);
                const int dot = acc[4 * g + u] + off * pop;
                const float fd = __builtin_fmaf(c1, (float)dot, __builtin_fmaf(c2, (float)pop, -c34));
                if (qok && ci < nc) orow[ci] = rabitq_key(fd, f0, f1, qc, qn, ip);
            }
        }
    }
}

// d % 512 == 0 (round 6): the same integer dot, 32 * NQB queries per workgroup.  rabitq_est_mfma_kernel
// spends ~20 VALU (the 16-bit sign expansion to int8) per v_mfma_i32_32x32x32_i8, because its LDS
// holds one 32-query block at full d; here the query bytes go through LDS in chunks of kEstKC
// dims (two stages, loaded a chunk ahead), and each expansion of a lane's 16 sign bits feeds NQB
// MFMAs, one per 32-query sub-block, whose accumulators stay in registers across the chunks.
// Wave w owns the 32-code tile w of the workgroup's 256 codes (lane (r, h): code r, k-half h, as
// above); its code bits for a chunk (kEstKC / 32 dwords of the row) are loaded a chunk ahead too.
// Integer sums: any order gives the oracle's dot; the epilogue is the estimator in fp32 order.
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations,
// not its global ones.  __syncthreads() is a workgroup release/acquire fence as well, so every
// chunk's barrier would also wait for the loads prefetching the next chunk and for the
// scattered key stores of the epilogue (vmcnt(0)).  The "memory" clobber keeps the compiler
// from moving memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int kEstKC = 512;                 // dims per LDS chunk
constexpr int kEstQP = kEstKC + 16;         // LDS pitch of a query row: 33 x 16 B, conflict-free b128 reads

// Screened key blocks (round 6, the multi-query kernel after the first column block): instead of
// the dense (nq, m) key block, a key is kept only when it ranks before the query's current k-th
// element (run_d / run_i: the running (nq, k) top-k of the blocks before, element k - 1), and is
// appended with its id to the query's candidate list (cnt[q] entries of row q, pitch ldc >= m, so
// no list can overflow).  Every key that can enter the final top-k passes the screen, so merging
// the lists into the running top-k gives the same (key, id) list as the dense block's top-k.
struct RqScreen {
    const float* run_d;
    const uint32_t* run_i;
    int k;
    uint32_t* cnt;
    float* cand_d;
    uint32_t* cand_i;
    int64_t ldc;
    uint32_t idbase;  // id of the block's column 0 (id_offset + c0, uint32 as in the dense path)
};

template <int NQB, bool SCREEN>
__global__ __launch_bounds__(kEstWaves * 64) void rabitq_est_mq_kernel(
    const uint8_t* __restrict__ codes, int64_t m, int d, const int8_t* __restrict__ qq, const float* __restrict__ qf,
    int64_t nq, int metric, float* __restrict__ buf, unsigned nqb, RqScreen scr) {
    constexpr int QR = 32 * NQB;                      // query rows per workgroup
    constexpr int STAGE = QR * kEstQP;                // bytes per LDS stage
    constexpr int NST = QR * (kEstKC / 16) / (kEstWaves * 64);  // 16-B staging pieces per thread
    static_assert(NST >= 2 && NST % 2 == 0 && QR * (kEstKC / 16) % (kEstWaves * 64) == 0, "staging split");
    constexpr int NG = kEstKC / 128;  // 16-B code-bit groups per chunk (4 k-steps each)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
    // persistent: workgroup b keeps query block b % nqb and walks the 256-code groups
    // b / nqb, + gridDim.x / nqb, ... (gridDim.x is a multiple of nqb), so the nqb workgroups of
    // a code group still run side by side (its code bits read from HBM once, then from L2)
    // (measured and not kept, profiles/r06_s14: the nqb workgroups of a code group placed on one
    // XCD; static priority for waves 4-7 -- both 1.5 % slower)
    const unsigned qblk = blockIdx.x % nqb;
    const int64_t gstep = gridDim.x / nqb;
    const int64_t ngroups = (m + kEstWaves * 32 - 1) / (kEstWaves * 32);
    const int64_t g0 = blockIdx.x / nqb;
    const int64_t q0 = (int64_t)qblk * QR;
    const int nb = d >> 3, cs = nb + 8;
    const int nch = d / kEstKC;  // d % kEstKC == 0 (host)
    const int64_t nit = g0 < ngroups ? ((ngroups - 1 - g0) / gstep + 1) * nch : 0;  // (group, chunk) steps
    // staging: piece i of this thread is query row e / 32, 16-B column e % 32 of the chunk; the
    // next chunk is staged in two halves (loaded at the start / middle of a step, stored at its
    // middle / end) so only half of it is held in registers at a time
    u32x4a4 qv[NST / 2];
    // range-checked buffer loads over this block's query rows: rows past nq read zeros (their keys
    // are never stored), the per-thread offset is one register and the piece / chunk offsets are
    // scalar (unconditional loads: a conditional load makes every later wait a vmcnt(0))
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(qq + q0 * d), 0, (int)(max<int64_t>(0, min<int64_t>(QR, nq - q0)) * d), 0x00020000);
    const int qvo = (tid >> 5) * d + 16 * (tid & 31);  // piece i: row (tid >> 5) + 16 i, column tid % 32
    static_assert((kEstWaves * 64) % 32 == 0, "staging pieces keep the thread's column");
    auto load_q = [&](int c, int half) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NST / 2; ++i) {
            const int pi = half * (NST / 2) + i;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(qrs, qvo, pi * (kEstWaves * 64 / 32) * d + c * kEstKC, 0);
            qv[i] = (u32x4a4){v[0], v[1], v[2], v[3]};
        }
    };
    auto store_q = [&](int st, int half) __attribute__((always_inline)) {
        unsigned char* sp = smem + st * STAGE;
#pragma unroll
        for (int i = 0; i < NST / 2; ++i) {
            const int e = tid + (half * (NST / 2) + i) * kEstWaves * 64, row = e >> 5, col = e & 31;
            *reinterpret_cast<uint4*>(sp + row * kEstQP + 16 * col) = make_uint4(qv[i][0], qv[i][1], qv[i][2], qv[i][3]);
        }
    };
    // this wave's code tile of group g; rows past m read row 0 (in range) and are never written
    auto tile = [&](int64_t g, int& nc) -> const uint8_t* {
        const int64_t cb = (g * kEstWaves + w) * 32;
        nc = (int)max<int64_t>(0, min<int64_t>(32, m - cb));
        return codes + (nc > 0 && r < nc ? cb + r : 0) * cs;
    };
    // the code bits of a chunk (NG 16-B groups of the row), loaded a whole step ahead
    u32x4a4 cg[NG], cgn[NG];
    auto load_c = [&](const uint8_t* crow, int c, u32x4a4 (&dst)[NG]) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < NG; ++g) dst[g] = *reinterpret_cast<const u32x4a4*>(crow + (c * kEstKC) / 8 + 16 * g);
    };
    v16i acc[NQB];
#pragma unroll
    for (int j = 0; j < NQB; ++j) acc[j] = (v16i){};
    int pc = 0;
    const int sh = 16 * h;
    const bool ip = metric == MIVQ_METRIC_INNER_PRODUCT;
    // per-query epilogue terms {c1, c2, c34, qc, qn, thd, off, thi} (thd / thi: the screen's
    // threshold, fixed for the launch) and per-wave code terms {pc of k-half 0, 1; f0; f1}, read
    // by the epilogue with b128 LDS reads instead of global loads and a shuffle per term
    float* qinfo = reinterpret_cast<float*>(smem + 2 * STAGE);
    float* cinfo = reinterpret_cast<float*>(smem + 2 * STAGE + QR * 32) + w * 128;
    if (tid < QR) {
        const int64_t qa = min<int64_t>(q0 + tid, nq - 1);
        float4 fa = *reinterpret_cast<const float4*>(qf + qa * kQfStride);
        float4 fb = *reinterpret_cast<const float4*>(qf + qa * kQfStride + 4);
        if constexpr (SCREEN) {
            fb.y = scr.run_d[qa * scr.k + scr.k - 1];
            fb.w = __uint_as_float(scr.run_i[qa * scr.k + scr.k - 1]);
        }
        *reinterpret_cast<float4*>(qinfo + tid * 8) = fa;
        *reinterpret_cast<float4*>(qinfo + tid * 8 + 4) = fb;
    }
    int64_t g = g0;
    int c = 0;
    int nc;
    const uint8_t* crow = tile(g, nc);
    if (nit > 0) {
        load_c(crow, 0, cg);
        load_q(0, 0);
        store_q(0, 0);
        load_q(0, 1);
        store_q(0, 1);
    }
    lds_barrier();
    for (int64_t it = 0; it < nit; ++it) {
        // the next step's chunk (the next group's first one at the end of a group)
        const bool more = it + 1 < nit;  // uniform
        const int cn = c + 1 < nch ? c + 1 : 0;
        const int64_t gn = c + 1 < nch ? g : g + gstep;
        int ncn = nc;
        const uint8_t* crown = crow;
        if (gn != g) crown = tile(gn, ncn);
        // unconditional (the last step reloads rows it already has), so every wait is counted;
        // the staging half first: its mid-step store then waits for it alone, not for the
        // code bits issued after it
        load_q(more ? cn : c, 0);
        load_c(more ? crown : crow, more ? cn : c, cgn);
        __builtin_amdgcn_sched_barrier(0);  // issue them here (the scheduler sinks loads to their use)
        constexpr int ks = kEstKC / 32;  // k-steps per chunk (d % kEstKC == 0)
        const int8_t* qs = reinterpret_cast<const int8_t*>(smem + (it & 1) * STAGE) + r * kEstQP + 16 * h;
        // the B operands (query bytes) of k-step s + 1 are read from LDS while step s's MFMAs run
        // (B reads two k-steps ahead: 1 % slower, profiles/r06_s21)
        v4i bq[NQB];
#pragma unroll
        for (int jb = 0; jb < NQB; ++jb) bq[jb] = *reinterpret_cast<const v4i*>(qs + jb * 32 * kEstQP);
#pragma unroll
        for (int gg = 0; gg < NG; ++gg) {
            {
                if (gg == NG / 2) {  // mid-chunk: first staging half out, second in
                    store_q((int)((it + 1) & 1), 0);  // unconditional: the last step's copy is never read
                    load_q(more ? cn : c, 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int s = 4 * gg + u;  // k-step within the chunk
                    const int sn = s + 1 < ks ? s + 1 : s;
                    v4i bqn[NQB];
#pragma unroll
                    for (int jb = 0; jb < NQB; ++jb) bqn[jb] = *reinterpret_cast<const v4i*>(qs + jb * 32 * kEstQP + 32 * sn);
                    // keeps those reads here, ahead of this step's MFMAs (the scheduler would sink
                    // them next to their use, exposing one LDS latency per MFMA)
                    __builtin_amdgcn_sched_barrier(0);
                    const uint32_t b16 = (cg[gg][u] >> sh) & 0xFFFFu;
                    pc += __builtin_popcount(b16);
                    v4i av;
#pragma unroll
                    for (int j = 0; j < 4; ++j) av[j] = (int)(__umul24((b16 >> (4 * j)) & 0xFu, 0x204081u) & 0x01010101u);
#pragma unroll
                    for (int jb = 0; jb < NQB; ++jb) acc[jb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bq[jb], acc[jb], 0, 0, 0);
#pragma unroll
                    for (int jb = 0; jb < NQB; ++jb) bq[jb] = bqn[jb];
                }
            }
        }
        if (c + 1 == nch && nc > 0) {  // the group's last chunk: estimator epilogue (wave-uniform)
            const int64_t cb = (g * kEstWaves + w) * 32;
            const float fr = *reinterpret_cast<const float*>(crow + nb + 4 * h);  // h = 0: f0, 1: f1 of code r
            // per code r of the tile: pop (both k-halves), (float)pop, f0 and -2 f1 (exact), so that
            // each (query, code) term below is 7 VALU: dot, 2 fma, convert, add, fma, compare
            cinfo[32 * h + r] = __int_as_float(pc);
            lds_fence();
            const int pop_r = __float_as_int(cinfo[r]) + __float_as_int(cinfo[32 + r]);
            if (h == 0) {
                cinfo[r] = __int_as_float(pop_r);
                cinfo[32 + r] = (float)pop_r;
                cinfo[64 + r] = fr;
            } else {
                cinfo[96 + r] = __fmul_rn(-2.0f, fr);
            }
            lds_fence();  // this wave's own LDS stores, read back below by other lanes
            auto epilogue = [&](auto ipc) __attribute__((always_inline)) {
                constexpr bool IP = decltype(ipc)::value;
#pragma unroll
                for (int jb = 0; jb < NQB; ++jb) {
                    const int64_t qa = q0 + 32 * jb + r;
                    const bool qok = qa < nq;
                    const float4 fa = *reinterpret_cast<const float4*>(qinfo + (32 * jb + r) * 8);
                    const float4 fb = *reinterpret_cast<const float4*>(qinfo + (32 * jb + r) * 8 + 4);
                    const float c1 = fa.x, c2 = fa.y, nc34 = -fa.z, qc = fa.w, qn = fb.x, thd = fb.y;
                    const int off = (int)fb.z;
                    float* orow = buf + (qok ? qa : 0) * m + cb;
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const int base = 8 * g4 + 4 * h;  // code rows of accumulators 4 g4 .. 4 g4 + 3
                        const int4 pv = *reinterpret_cast<const int4*>(cinfo + base);
                        const float4 pf = *reinterpret_cast<const float4*>(cinfo + 32 + base);
                        const float4 f0v = *reinterpret_cast<const float4*>(cinfo + 64 + base);
                        const float4 mf1 = *reinterpret_cast<const float4*>(cinfo + 96 + base);
                        const int pa[4] = {pv.x, pv.y, pv.z, pv.w};
                        const float pfa[4] = {pf.x, pf.y, pf.z, pf.w}, f0a[4] = {f0v.x, f0v.y, f0v.z, f0v.w},
                                    m2f1[4] = {mf1.x, mf1.y, mf1.z, mf1.w};
                        float key[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            // the oracle's order: fd = fmaf(c1, dot, fmaf(c2, pop, -c34)),
                            // pre = fmaf(-2 f1, fd, f0 + qc), IP: 0.5 (pre - qn)
                            const int dot = acc[jb][4 * g4 + u] + off * pa[u];
                            const float fd = __builtin_fmaf(c1, (float)dot, __builtin_fmaf(c2, pfa[u], nc34));
                            const float pre = __builtin_fmaf(m2f1[u], fd, __fadd_rn(f0a[u], qc));
                            key[u] = IP ? __fmul_rn(0.5f, __fsub_rn(pre, qn)) : pre;
                        }
                        if constexpr (SCREEN) {
                            // one compare per key; the exact (key, id) test (NaN -> +inf, ties by
                            // id, the row and query guards) only for keys not above the threshold
                            const bool any = !(key[0] > thd) || !(key[1] > thd) || !(key[2] > thd) || !(key[3] > thd);
                            if (any) {
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    const int ci = base + u;
                                    const float kk = key[u] != key[u] ? INFINITY : key[u];
                                    const uint32_t id = scr.idbase + (uint32_t)(cb + ci);
                                    if (qok && ci < nc && pair_less(kk, id, thd, __float_as_uint(fb.w))) {
                                        const int64_t slot = atomicAdd(scr.cnt + qa, 1u);
                                        scr.cand_d[qa * scr.ldc + slot] = kk;
                                        scr.cand_i[qa * scr.ldc + slot] = id;
                                    }
                                }
                            }
                        } else {
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (qok && base + u < nc) orow[base + u] = key[u];
                        }
                    }
                }
            };
            if (ip) epilogue(std::true_type{});
            else epilogue(std::false_type{});
        }
        if (c + 1 == nch) {
#pragma unroll
            for (int jb = 0; jb < NQB; ++jb) acc[jb] = (v16i){};
            pc = 0;
        }
        store_q((int)((it + 1) & 1), 1);
#pragma unroll
        for (int gg = 0; gg < NG; ++gg) cg[gg] = cgn[gg];
        lds_barrier();
        c = cn;
        g = gn;
        crow = crown;
        nc = ncn;
    }
}

// Merges each query's screened candidates (RqScreen) into its running top-k in place, one wave
// per query, and clears the query's count for the next block.  Exact in (key, id) whatever the
// order the candidates were appended in.
template <int R>
__global__ __launch_bounds__(256) void rq_screen_merge_kernel(float* __restrict__ run_d, uint32_t* __restrict__ run_i,
                                                              int64_t nq, int k, uint32_t* __restrict__ cnt,
                                                              const float* __restrict__ cand_d,
                                                              const uint32_t* __restrict__ cand_i, int64_t ldc) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const uint32_t nc = cnt[q];  // wave-uniform
    if (nc == 0) return;
    WaveTopK<R> top;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        top.d[r] = e < k ? run_d[q * k + e] : INFINITY;
        top.id[r] = e < k ? run_i[q * k + e] : kNoId;
    }
    float thr_d;
    uint32_t thr_i;
    top.kth(k, thr_d, thr_i);
    const float* cd = cand_d + q * ldc;
    const uint32_t* cix = cand_i + q * ldc;
    for (uint32_t j0 = 0; j0 < nc; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool valid = j < nc;
        const float dv = valid ? cd[j] : INFINITY;
        const uint32_t iv = valid ? cix[j] : kNoId;
        top.offer(valid, dv, iv, k, lane, thr_d, thr_i);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < k) { run_d[q * k + e] = top.d[r]; run_i[q * k + e] = top.id[r]; }
    }
    if (lane == 0) cnt[q] = 0;
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
    size_t qq, qr, qf, tiled, cand_d, cand_i, cnt, total;
};

// Columns of the dense first block of the screened search: its top-k gives every query a
// threshold (the k-th best of 8192 keys passes ~k / 8192 of the keys after it).
constexpr int64_t kRqFirstCols = 8192;
// Candidate-list entries (keys + ids, 8 B each) the screened blocks may use: a block is at most
// 2^27 / nq codes wide (~134k at 1000 queries), so no list can overflow whatever the codes' order.
constexpr int64_t kRqScreenEntries = (int64_t)1 << 27;

// Width of the screened blocks (0: no screened block), whole 256-code groups.
int64_t rq_screen_cols(int64_t nq, int64_t n) {
    const int64_t rest = n - std::min<int64_t>(n, kRqFirstCols);
    if (rest <= 0 || nq <= 0) return 0;
    const int64_t g = kEstWaves * 32;
    const int64_t w = std::max<int64_t>(4 * g, kRqScreenEntries / nq / g * g);  // >= 1024 codes
    return std::min<int64_t>(w, ceil_div(rest, g) * g);
}

// Screened search (d % 512 == 0): the dense first block's tiled top-k region, then the candidate
// lists (nq x rq_screen_cols keys and ids) and counts.  The dense search of other shapes uses the
// same offset for its full tiled region (the two layouts never coexist in one call).
RqLayout rq_layout(int64_t nq, int64_t n, int d, int k) {
    RqLayout L{};
    size_t off = 0;
    const bool screened = d % kEstKC == 0;
    L.qq = off;    off = align_up(off + (size_t)nq * d, 256);
    L.qr = off;    off = align_up(off + (size_t)nq * d * 4, 256);
    L.qf = off;    off = align_up(off + (size_t)nq * kQfStride * 4, 256);
    L.tiled = off;
    const size_t dense_all = align_up(off + flat_tiled_workspace_bytes(nq, n, k), 256);
    if (screened) {
        const size_t sc = (size_t)nq * rq_screen_cols(nq, n) * 4;
        off = align_up(off + flat_tiled_workspace_bytes(nq, std::min<int64_t>(n, kRqFirstCols), k), 256);
        L.cand_d = off; off = align_up(off + sc, 256);
        L.cand_i = off; off = align_up(off + sc, 256);
        L.cnt = off;    off = align_up(off + (size_t)nq * 4, 256);
    }
    L.total = std::max(off, dense_all);
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
    // the multi-query kernel for d % 512 == 0 (32, 64 or 128 queries per workgroup by nq)
#ifndef MIVQ_RQ_MQ
#define MIVQ_RQ_MQ 1
#endif
    const int nqb_mq = nq > 64 ? 4 : nq > 32 ? 2 : 1;
    const bool mq = MIVQ_RQ_MQ && mfma && (d % kEstKC) == 0;
    // multi-query kernel: two staging stages, the per-query and per-wave epilogue terms
    const size_t smem = mq ? (size_t)2 * 32 * nqb_mq * kEstQP + 32 * nqb_mq * 32 + kEstWaves * 512
                           : (size_t)32 * (d + 16);
    if (mfma && smem > 160 * 1024) return set_error(MIVQ_ERR_UNSUPPORTED, "rabitq_search: d=%d too large", d);
    using MqFn = void (*)(const uint8_t*, int64_t, int, const int8_t*, const float*, int64_t, int, float*, unsigned,
                          RqScreen);
    const MqFn mq_dense = nqb_mq == 4   ? rabitq_est_mq_kernel<4, false>
                          : nqb_mq == 2 ? rabitq_est_mq_kernel<2, false>
                                        : rabitq_est_mq_kernel<1, false>;
    const MqFn mq_screen = nqb_mq == 4   ? rabitq_est_mq_kernel<4, true>
                           : nqb_mq == 2 ? rabitq_est_mq_kernel<2, true>
                                         : rabitq_est_mq_kernel<1, true>;
    if (mfma) {
        for (const void* f : {mq ? (const void*)mq_dense : (const void*)rabitq_est_mfma_kernel, (const void*)mq_screen}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "rabitq_search: %s", hipGetErrorString(e));
        }
    }
    const int nbytes = (d + 7) / 8 + 8;
    // persistent grid of the multi-query kernel: a multiple of the query blocks, about one
    // workgroup per CU
    auto launch_mq = [&](MqFn fn, int64_t c0, int64_t m, float* buf, const RqScreen& scr) {
        const int64_t nqblk = ceil_div(nq, 32 * nqb_mq);
        const int64_t groups = ceil_div(m, kEstWaves * 32);
        const int64_t per = std::max<int64_t>(1, std::min<int64_t>(groups, 256 / std::max<int64_t>(1, nqblk)));
        hipLaunchKernelGGL(fn, dim3((unsigned)(per * nqblk)), dim3(kEstWaves * 64), smem, st, codes + c0 * nbytes, m,
                           d, qq, qf, nq, metric, buf, (unsigned)nqblk, scr);
        return hipGetLastError();
    };
    // the dense key blocks and their tiled top-k: the whole search, or the first block of the
    // screened one
    const int64_t n_dense = mq ? std::min<int64_t>(n, kRqFirstCols) : n;
    hipError_t e = launch_tiled_topk(
        nq, n_dense, k, id_offset, p + L.tiled, dists, ids, st, [&](int64_t c0, int64_t m, float* buf) {
            const uint8_t* cc = codes + c0 * nbytes;
            if (mq)
                return launch_mq(mq_dense, c0, m, buf, RqScreen{});
            if (mfma)
                hipLaunchKernelGGL(rabitq_est_mfma_kernel,
                                   dim3((unsigned)(ceil_div(m, kEstWaves * kEstTiles * 32) * ceil_div(nq, 32))),
                                   dim3(kEstWaves * 64), smem, st, cc, m, d, qq, qf, nq, metric, buf,
                                   (unsigned)ceil_div(nq, 32));
            else
                hipLaunchKernelGGL(rabitq_est_generic_kernel, dim3((unsigned)ceil_div(m, 256), (unsigned)nq),
                                   dim3(256), 0, st, cc, m, d, qq, qr, qf, qb, metric, buf);
            return hipGetLastError();
        });
    if (e == hipSuccess && n > n_dense) {
        // screened blocks growing 4x from 4 x the first block (the threshold is refreshed after
        // each: ~k x width / codes-so-far keys pass per query, and few queries' counters are
        // contended when nq is small), capped at rq_screen_cols; whole 256-code groups; each
        // followed by the merge of its candidates into (dists, ids)
        const int64_t cap = rq_screen_cols(nq, n);
        uint32_t* cnt = reinterpret_cast<uint32_t*>(p + L.cnt);
        RqScreen scr{dists, ids, k, cnt, reinterpret_cast<float*>(p + L.cand_d),
                     reinterpret_cast<uint32_t*>(p + L.cand_i), cap, 0u};
        int64_t cols = std::min<int64_t>(cap, 4 * kRqFirstCols);
        e = hipMemsetAsync(cnt, 0, (size_t)nq * 4, st);
        for (int64_t c0 = n_dense, m = 0; c0 < n && e == hipSuccess; c0 += m, cols = std::min<int64_t>(cap, 4 * cols)) {
            m = std::min<int64_t>(cols, n - c0);
            if (n - c0 - m < cols / 4) m = std::min<int64_t>(cap, n - c0);  // no sliver of a last block
            scr.idbase = (uint32_t)(id_offset + c0);
            e = launch_mq(mq_screen, c0, m, nullptr, scr);
            if (e != hipSuccess) break;
            const dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
            switch ((k + 63) / 64) {
                case 1: hipLaunchKernelGGL(rq_screen_merge_kernel<1>, grid, block, 0, st, dists, ids, nq, k, cnt, scr.cand_d, scr.cand_i, cap); break;
                case 2: hipLaunchKernelGGL(rq_screen_merge_kernel<2>, grid, block, 0, st, dists, ids, nq, k, cnt, scr.cand_d, scr.cand_i, cap); break;
                case 3: hipLaunchKernelGGL(rq_screen_merge_kernel<3>, grid, block, 0, st, dists, ids, nq, k, cnt, scr.cand_d, scr.cand_i, cap); break;
                default: hipLaunchKernelGGL(rq_screen_merge_kernel<4>, grid, block, 0, st, dists, ids, nq, k, cnt, scr.cand_d, scr.cand_i, cap); break;
            }
            e = hipGetLastError();
        }
    }
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "rabitq_search: %s", hipGetErrorString(e));
    return MIVQ_OK;
}
