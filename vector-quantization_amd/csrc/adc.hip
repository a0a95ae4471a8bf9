// adc.hip — flat ADC (asymmetric distance) search over PQ codes on gfx950.
//
// GPU counterpart of FlatQuantizedIndex.search_with_scores
// (/root/reference/src/haag_vq/methods/search/flat_quantized_index.py:45-76), which decodes
// every code and ranks ||q - x_hat||^2; here the same quantity is assembled from per-query
// lookup tables, sum_m ||q_m - c_{m,code_m}||^2 (canonical order in include/mivq.h):
//   adc_lut_kernel     one block per (subspace, 32 queries), one lane per centroid.
//   adc_scan_kernel    LUTs of QB queries live in LDS; each wavefront streams 64 code rows
//                      per step (one row per lane, 16-B loads), sums M table entries per
//                      (row, query) and keeps, per query, a wave-resident top-k (element e of
//                      the sorted list in lane e%64, register e/64) that a ballot screens and
//                      a shift-insert updates.  Exact (dist, id) order, so results are
//                      deterministic and identical for any row partition.
//   topk_merge_kernel  merges the per-wave partial lists (and, after the RCCL all-gather,
//                      the per-shard lists) into the final sorted top-k.
#include "mivq_common.h"
#include "topk.h"

namespace mivq {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));  // native vector: HIP's float4 struct copies can defeat SROA
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr int kScanWaves = 16;  // waves per scan workgroup (adc and flat)

// L2: lut[q][m][k] = fmaf chain over t of (q_t - c_t)^2;  IP: -(fmaf chain of q_t * c_t)
// grid (M, ceil(nq / kLutQ)), block 256: thread = centroid k of subspace m, looping over a
// block of kLutQ queries whose sub-vectors sit in LDS (broadcast reads).  The centroid row
// is read 4 floats at a time and every query's chain advances over those 4 dims in order,
// so each (query, k) chain is the canonical sequential one.  Stores are coalesced along k.
// 16 queries per workgroup (round 5: 57 -> 46 us for 1000 queries at M = 16 against 32 -- twice
// the workgroups to spread over the CUs; 8: 50 us; profiles/r05_s24)
constexpr int kLutQ = 16;

__global__ __launch_bounds__(256) void adc_lut_kernel(const float* __restrict__ q, int64_t nq, int d, int M, int ksub,
                                                       int dsub, const float* __restrict__ C, int metric,
                                                       int vec16, float* __restrict__ lut) {
    extern __shared__ __attribute__((aligned(16))) float qs[];  // [kLutQ][dsub]
    const int m = blockIdx.x;
    const int64_t q0 = (int64_t)blockIdx.y * kLutQ;
    const int nqb = (int)min<int64_t>(kLutQ, nq - q0);
    for (int e = threadIdx.x; e < nqb * dsub; e += blockDim.x) {
        const int qq = e / dsub, t = e - qq * dsub;
        qs[e] = q[(q0 + qq) * d + (int64_t)m * dsub + t];
    }
    __syncthreads();
    const int k = threadIdx.x;
    if (k >= ksub) return;
    const float* c = C + ((int64_t)m * ksub + k) * dsub;
    float acc[kLutQ];
#pragma unroll
    for (int qq = 0; qq < kLutQ; ++qq) acc[qq] = 0.0f;
    const bool l2 = metric == MIVQ_METRIC_L2;
    auto step = [&](float c0, float c1, float c2, float c3, int t0, int nt) __attribute__((always_inline)) {
#pragma unroll
        for (int qq = 0; qq < kLutQ; ++qq) {
            const float* qr = qs + qq * dsub + t0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float cj = j == 0 ? c0 : j == 1 ? c1 : j == 2 ? c2 : c3;
                if (j < nt) {
                    if (l2) {
                        const float df = __fsub_rn(qr[j], cj);
                        acc[qq] = __builtin_fmaf(df, df, acc[qq]);
                    } else {
                        acc[qq] = __builtin_fmaf(qr[j], cj, acc[qq]);
                    }
                }
            }
        }
    };
    if (vec16) {  // dsub % 4 == 0 and C 16-B aligned (host-side test: views may start anywhere)
        // 16-B loads of the centroid row, the next one in flight while this one is used.  (Round
        // 2 replaced these by dword loads while chasing a two-stream mismatch in lanes 48..63;
        // the cause was the LDS-DMA OPQ GEMM on the other stream corrupting packed-fp32 results,
        // since removed from the library: DESIGN §8.  The load form was never involved.)
        v4f cur = *reinterpret_cast<const v4f*>(c);
        for (int t0 = 0; t0 < dsub; t0 += 4) {
            const v4f nxt = (t0 + 4 < dsub) ? *reinterpret_cast<const v4f*>(c + t0 + 4) : cur;
            step(cur.x, cur.y, cur.z, cur.w, t0, 4);
            cur = nxt;
        }
    } else {
        for (int t0 = 0; t0 < dsub; t0 += 4) {
            const int nt = min(4, dsub - t0);
            const float c0 = c[t0], c1 = nt > 1 ? c[t0 + 1] : 0.0f;
            const float c2 = nt > 2 ? c[t0 + 2] : 0.0f, c3 = nt > 3 ? c[t0 + 3] : 0.0f;
            step(c0, c1, c2, c3, t0, nt);
        }
    }
#pragma unroll
    for (int qq = 0; qq < kLutQ; ++qq)
        if (qq < nqb) lut[((q0 + qq) * M + m) * ksub + k] = l2 ? acc[qq] : -acc[qq];
}

// ksub = 256, dsub % 4 == 0, C 16-B aligned (round 6): packed fp32.  Grid (M, ceil(nq / 8)),
// block 128: thread k takes centroids k and k + 128 as the two halves of v_pk_add_f32 /
// v_pk_fma_f32 (both chains exactly the scalar ones: the same sub, then fma, over t ascending),
// and the 8 queries' values come through the scalar cache as the broadcast operand -- no LDS,
// so no packed instruction reads an LDS-loaded register.  Half the VALU of the
// scalar kernel, and no LDS reads at all.
constexpr int kLutPkQ = 8;
template <bool L2, int DS>
__global__ __launch_bounds__(128) void adc_lut_pk_kernel(const float* __restrict__ q, int64_t nq, int d, int M,
                                                          int dsub, const float* __restrict__ C,
                                                          float* __restrict__ lut) {
    const int m = blockIdx.x;
    const int64_t q0 = (int64_t)blockIdx.y * kLutPkQ;
    const int nqb = (int)min<int64_t>(kLutPkQ, nq - q0);
    const int k = threadIdx.x;
    const float* ca = C + ((int64_t)m * 256 + k) * dsub;
    const float* cb = ca + (int64_t)128 * dsub;
    const float* qr[kLutPkQ];
#pragma unroll
    for (int qq = 0; qq < kLutPkQ; ++qq) qr[qq] = q + (q0 + min(qq, nqb - 1)) * d + (int64_t)m * dsub;  // in range
    float2v acc[kLutPkQ];
#pragma unroll
    for (int qq = 0; qq < kLutPkQ; ++qq) acc[qq] = (float2v){0.0f, 0.0f};
    auto body = [&](const v4f& a, const v4f& b, int t0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2v cc = {a[j], b[j]};
#pragma unroll
            for (int qq = 0; qq < kLutPkQ; ++qq) {
                const float qv = qr[qq][t0 + j];
                const float2v qq2 = {qv, qv};
                if constexpr (L2) {
                    const float2v df = qq2 - cc;
                    acc[qq] = __builtin_elementwise_fma(df, df, acc[qq]);
                } else {
                    acc[qq] = __builtin_elementwise_fma(qq2, cc, acc[qq]);
                }
            }
        }
    };
    if constexpr (DS > 0) {
        // compile-time dsub: both centroid rows are loaded up front (DS / 2 16-B loads per thread,
        // all in flight at once) and consumed in order as they land, instead of one 16-B step
        // ahead with a wait at every loop latch
        // (a window of W steps ahead instead spills: the scheduler hoists every load regardless)
        v4f ra[DS / 4], rb[DS / 4];
#pragma unroll
        for (int i = 0; i < DS / 4; ++i) {
            ra[i] = *reinterpret_cast<const v4f*>(ca + 4 * i);
            rb[i] = *reinterpret_cast<const v4f*>(cb + 4 * i);
        }
#pragma unroll
        for (int i = 0; i < DS / 4; ++i) body(ra[i], rb[i], 4 * i);
    } else {
    v4f a = *reinterpret_cast<const v4f*>(ca), b = *reinterpret_cast<const v4f*>(cb);
    for (int t0 = 0; t0 < dsub; t0 += 4) {
        const bool more = t0 + 4 < dsub;
        const v4f an = more ? *reinterpret_cast<const v4f*>(ca + t0 + 4) : a;
        const v4f bn = more ? *reinterpret_cast<const v4f*>(cb + t0 + 4) : b;
        body(a, b, t0);
        a = an;
        b = bn;
    }
    }
#pragma unroll
    for (int qq = 0; qq < kLutPkQ; ++qq) {
        if (qq < nqb) {
            float* o = lut + ((q0 + qq) * M + m) * 256;
            o[k] = L2 ? acc[qq].x : -acc[qq].x;
            o[k + 128] = L2 ? acc[qq].y : -acc[qq].y;
        }
    }
}

// Table group mk (= m*ksub + code) holds the QB queries' entries of (m, code) side by side.
// For QB = 8 a lookup is two ds_read_b128 of the group's 16-B halves, and odd lanes read the
// halves in the opposite order: in each 16-lane group of a ds_read_b128 the 8 even lanes then
// hit even 16-B slots of the 256-B bank row and the 8 odd lanes odd ones, two independent
// 8-into-8 draws instead of one 16-into-16 (random codes: 2.94 instead of 3.08 expected LDS
// cycles per lane group).  The lane keeps its two half-sums in lane order (lo = the half read
// first) and swaps them back once per row; each query's sum still runs over m in order.
template <int QB>
__device__ __forceinline__ void lut_add(const float* tab, uint32_t mk, float (&dist)[QB], uint32_t par) {
    const float* g = tab + (size_t)mk * QB;
    if constexpr (QB == 8) {
        const float4 t0 = *reinterpret_cast<const float4*>(g + 4 * par);
        const float4 t1 = *reinterpret_cast<const float4*>(g + 4 * (par ^ 1u));
        dist[0] += t0.x; dist[1] += t0.y; dist[2] += t0.z; dist[3] += t0.w;
        dist[4] += t1.x; dist[5] += t1.y; dist[6] += t1.z; dist[7] += t1.w;
    } else if constexpr (QB >= 4) {
#pragma unroll
        for (int v = 0; v < QB / 4; ++v) {
            const float4 t = *reinterpret_cast<const float4*>(g + 4 * v);
            dist[4 * v + 0] += t.x; dist[4 * v + 1] += t.y; dist[4 * v + 2] += t.z; dist[4 * v + 3] += t.w;
        }
    } else if constexpr (QB == 2) {
        const float2 t = *reinterpret_cast<const float2*>(g);
        dist[0] += t.x; dist[1] += t.y;
    } else {
        dist[0] += g[0];
    }
}

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f32x4v lds_f4;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4v lds_u4;
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u32x2v lds_u2;

// Undoes the odd lanes' half order of lut_add<8> (identity for other QB).
template <int QB>
__device__ __forceinline__ void lut_unswap(float (&dist)[QB], uint32_t par) {
    if constexpr (QB == 8) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float a = dist[q], b = dist[q + 4];
            dist[q] = par ? b : a;
            dist[q + 4] = par ? a : b;
        }
    }
}

// grid (nchunks, ceil(nq / QB)), block kScanWaves waves sharing the QB LUTs in LDS (so the
// CU keeps 4 waves per SIMD despite the 128 KiB of tables).  Part index = chunk*kScanWaves + wave.
// MC > 0 (M = 16 MC, ksub = 256, 16-B aligned code rows): each lane's row of codes is MC
// 16-B loads issued one wave-step ahead, so the LDS lookups never wait on the code fetch
// (MC = 0: 4-B code words loaded in the step that uses them).
template <int R, int QB, int MC>
__device__ __forceinline__ void adc_scan_block(
    const float* __restrict__ lut, int64_t nq, const uint8_t* __restrict__ codes, int64_t n, int M,
    int ksub, int k, int64_t id_offset, int64_t chunk_rows, float* __restrict__ part_d,
    uint32_t* __restrict__ part_i, const int* __restrict__ qlist, const int* __restrict__ qcount, int64_t yb) {
    if constexpr (MC > 0) {
        M = 16 * MC;
        ksub = 256;
    }
    // qlist (the exact re-run of queries the filtered search could not certify, below): query
    // slot s of this launch is query qlist[s], s < *qcount; the lists are written per slot
    // [M][ksub][QB]: the QB queries' entries of one (m, code) are adjacent, so one 16-B LDS
    // read serves 4 queries (random codes: ~2x fewer bank-conflict cycles per lookup than
    // QB separate 4-B reads)
    extern __shared__ __attribute__((aligned(16))) float tab[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t q0 = yb * QB;
    int nqb = (int)min<int64_t>(QB, nq - q0);
    if (qlist != nullptr) {
        const int cnt = *qcount;
        if (q0 >= cnt) return;  // whole workgroup (the caller's loop ends too)
        nqb = (int)min<int64_t>(QB, cnt - q0);
    }
    const int64_t tab_elems = (int64_t)M * ksub;
    for (int64_t e = tid; e < tab_elems * QB; e += kScanWaves * 64) {
        const int64_t mk = e / QB;
        const int qq = (int)(e - mk * QB);
        const int64_t qsrc = qq < nqb ? (qlist != nullptr ? (int64_t)qlist[q0 + qq] : q0 + qq) : 0;
        tab[e] = qq < nqb ? lut[qsrc * tab_elems + mk] : 0.0f;
    }
    __syncthreads();

    WaveTopK<R> top[QB];
    float thr_d[QB];     // element k-1 of each list (wave-uniform)
    uint32_t thr_i[QB];
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        top[qq].init();
        thr_d[qq] = INFINITY;
        thr_i[qq] = kNoId;
    }

    const int64_t rbeg = (int64_t)blockIdx.x * chunk_rows;
    const int64_t rend = min(n, rbeg + chunk_rows);
    const bool words = (M % 4) == 0;
    const uint32_t par = (uint32_t)lane & 1u;
    const uint32_t tbase = (uint32_t)(uintptr_t)tab + 16u * par;  // LDS byte address of the half read first
    uint4 cw[MC > 0 ? MC : 1];
    auto fetch = [&](int64_t row) __attribute__((always_inline)) {
        if constexpr (MC > 0) {
            const uint4* cr = reinterpret_cast<const uint4*>(codes + row * (16 * MC));
#pragma unroll
            for (int c = 0; c < MC; ++c) cw[c] = row < rend ? cr[c] : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    fetch(rbeg + (int64_t)wv * 64 + lane);
    for (int64_t base = rbeg + (int64_t)wv * 64; base < rend; base += kScanWaves * 64) {
        const int64_t row = base + lane;
        const bool valid = row < rend;
        float dist[QB];
#pragma unroll
        for (int qq = 0; qq < QB; ++qq) dist[qq] = 0.0f;
        if constexpr (MC > 0) {
            uint4 cur[MC];
#pragma unroll
            for (int c = 0; c < MC; ++c) cur[c] = cw[c];
            fetch(row + kScanWaves * 64);
            // one word (4 sub-codes) per iteration, the queue of words rotating through
            // registers (a rolled loop: unrolled, the 16 MC lookups' reads and addresses
            // outgrow the 128 registers of the 16-wave workgroup)
            uint32_t wq[4 * MC];
#pragma unroll
            for (int c = 0; c < MC; ++c) {
                wq[4 * c + 0] = cur[c].x; wq[4 * c + 1] = cur[c].y;
                wq[4 * c + 2] = cur[c].z; wq[4 * c + 3] = cur[c].w;
            }
#pragma unroll 1
            for (int jw = 0; jw < 4 * MC; ++jw) {
                const uint32_t wrd = wq[0];
                if constexpr (QB == 8) {
                    // byte offsets: group (4 jw + b, code) at 32 (256 (4 jw + b) + code); the half
                    // read first at +16 par, the other at that ^ 16; the b term (a multiple of 32)
                    // goes to the instruction's offset field: 3 VALU per lookup for addresses
                    const uint32_t wofs = tbase + (uint32_t)jw * (4u * 256u * 32u);
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        // inline asm keeps the three ops as written (left to itself the compiler
                        // re-derives o2 from the pieces with more adds)
                        uint32_t cb, o1, o2;
                        asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(cb) : "v"(wrd), "i"(8 * b));
                        asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(o1) : "v"(cb), "v"(wofs));
                        asm("v_xor_b32 %0, 16, %1" : "=v"(o2) : "v"(o1));
                        const f32x4v t0 = *(reinterpret_cast<const lds_f4*>((uintptr_t)o1) + b * 512);
                        const f32x4v t1 = *(reinterpret_cast<const lds_f4*>((uintptr_t)o2) + b * 512);
                        dist[0] += t0.x; dist[1] += t0.y; dist[2] += t0.z; dist[3] += t0.w;
                        dist[4] += t1.x; dist[5] += t1.y; dist[6] += t1.z; dist[7] += t1.w;
                    }
                } else {
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        lut_add<QB>(tab, (uint32_t)((4 * jw + b) * 256) + ((wrd >> (8 * b)) & 0xFFu), dist, par);
                }
#pragma unroll
                for (int t = 0; t + 1 < 4 * MC; ++t) wq[t] = wq[t + 1];
            }
            lut_unswap<QB>(dist, par);
        } else if (valid) {
            const uint8_t* cr = codes + row * M;
            if (words) {
                for (int m0 = 0; m0 < M; m0 += 4) {
                    const uint32_t wrd = *reinterpret_cast<const uint32_t*>(cr + m0);
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t code = (wrd >> (8 * b)) & 0xFFu;
                        lut_add<QB>(tab, (uint32_t)((m0 + b) * ksub) + code, dist, par);
                    }
                }
            } else {
                for (int m = 0; m < M; ++m) lut_add<QB>(tab, (uint32_t)(m * ksub + cr[m]), dist, par);
            }
            lut_unswap<QB>(dist, par);
        }
        const uint32_t gid = (uint32_t)(id_offset + row);
#pragma unroll
        for (int qq = 0; qq < QB; ++qq) {
            if (qq >= nqb) break;
            float dv = dist[qq];
            if (dv != dv) dv = INFINITY;  // NaN ranks with +inf
            // screen against the cached k-th element; it only moves when something is inserted
            unsigned long long mask = __ballot(valid && pair_less(dv, gid, thr_d[qq], thr_i[qq]));
            while (mask) {
                const int src = __builtin_ctzll(mask);
                mask &= mask - 1;
                const float cd = __shfl(dv, src);
                const uint32_t ci = __shfl(gid, src);
                if (!pair_less(cd, ci, thr_d[qq], thr_i[qq])) continue;
                top[qq].insert(cd, ci, k, lane);
                top[qq].kth(k, thr_d[qq], thr_i[qq]);
            }
        }
    }
    const int64_t part = (int64_t)blockIdx.x * kScanWaves + wv;
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        if (qq >= nqb) break;
        float* od = part_d + (part * nq + q0 + qq) * k;
        uint32_t* oi = part_i + (part * nq + q0 + qq) * k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = r * 64 + lane;
            if (e < k) { od[e] = top[qq].d[r]; oi[e] = top[qq].id[r]; }
        }
    }
}

// Query block blockIdx.y (fp32 scan of every query), or -- qlist, the re-run of the queries
// the filtered search could not certify -- list slots blockIdx.y, + gridDim.y, ... while they
// exist: a small grid whatever the count (0 failures: every workgroup returns at once).
template <int R, int QB, int MC>
__global__ __launch_bounds__(kScanWaves * 64) void adc_scan_kernel(
    const float* __restrict__ lut, int64_t nq, const uint8_t* __restrict__ codes, int64_t n, int M,
    int ksub, int k, int64_t id_offset, int64_t chunk_rows, float* __restrict__ part_d,
    uint32_t* __restrict__ part_i, const int* __restrict__ qlist, const int* __restrict__ qcount) {
    if (qlist == nullptr) {
        adc_scan_block<R, QB, MC>(lut, nq, codes, n, M, ksub, k, id_offset, chunk_rows, part_d, part_i, qlist, qcount,
                                  (int64_t)blockIdx.y);
        return;
    }
    const int cnt = *qcount;
    for (int64_t yb = blockIdx.y; yb * QB < cnt; yb += gridDim.y) {
        adc_scan_block<R, QB, MC>(lut, nq, codes, n, M, ksub, k, id_offset, chunk_rows, part_d, part_i, qlist, qcount,
                                  yb);
        __syncthreads();  // the next block's table overwrites this one's
    }
}

// Exact brute force over an f32 database: grid (nchunks, ceil(nq / QB)), block 256.  The QB
// query vectors live in LDS; lane = database row, distances are sequential fmaf chains over t
// (16-B loads of the row), ranked with the same wave-resident top-k as adc_scan_kernel.
template <int R, int QB>
__global__ __launch_bounds__(kScanWaves * 64) void flat_scan_kernel(
    const float* __restrict__ q, int64_t nq, const float* __restrict__ x, int64_t n, int d, int metric, int k,
    int64_t id_offset, int64_t chunk_rows, float* __restrict__ part_d, uint32_t* __restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float qv[];  // [QB][d]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t q0 = (int64_t)blockIdx.y * QB;
    const int nqb = (int)min<int64_t>(QB, nq - q0);
    for (int64_t e = tid; e < (int64_t)nqb * d; e += kScanWaves * 64) qv[e] = q[q0 * d + e];
    __syncthreads();
    WaveTopK<R> top[QB];
    float thr_d[QB];
    uint32_t thr_i[QB];
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        top[qq].init();
        thr_d[qq] = INFINITY;
        thr_i[qq] = kNoId;
    }
    const int64_t rbeg = (int64_t)blockIdx.x * chunk_rows;
    const int64_t rend = min(n, rbeg + chunk_rows);
    const bool vec = (d % 4) == 0;
    for (int64_t base = rbeg + (int64_t)wv * 64; base < rend; base += kScanWaves * 64) {
        const int64_t row = base + lane;
        const bool valid = row < rend;
        float dist[QB];
#pragma unroll
        for (int qq = 0; qq < QB; ++qq) dist[qq] = 0.0f;
        if (valid) {
            const float* xr = x + row * d;
            if (vec) {
                for (int t = 0; t < d; t += 4) {
                    const float4 xv = *reinterpret_cast<const float4*>(xr + t);
#pragma unroll
                    for (int qq = 0; qq < QB; ++qq) {
                        const float4 qf = *reinterpret_cast<const float4*>(qv + qq * d + t);
                        if (metric == MIVQ_METRIC_L2) {
                            float df = __fsub_rn(qf.x, xv.x); dist[qq] = __builtin_fmaf(df, df, dist[qq]);
                            df = __fsub_rn(qf.y, xv.y); dist[qq] = __builtin_fmaf(df, df, dist[qq]);
                            df = __fsub_rn(qf.z, xv.z); dist[qq] = __builtin_fmaf(df, df, dist[qq]);
                            df = __fsub_rn(qf.w, xv.w); dist[qq] = __builtin_fmaf(df, df, dist[qq]);
                        } else {
                            dist[qq] = __builtin_fmaf(qf.x, xv.x, dist[qq]);
                            dist[qq] = __builtin_fmaf(qf.y, xv.y, dist[qq]);
                            dist[qq] = __builtin_fmaf(qf.z, xv.z, dist[qq]);
                            dist[qq] = __builtin_fmaf(qf.w, xv.w, dist[qq]);
                        }
                    }
                }
            } else {
                for (int t = 0; t < d; ++t) {
                    const float xs = xr[t];
#pragma unroll
                    for (int qq = 0; qq < QB; ++qq) {
                        if (metric == MIVQ_METRIC_L2) {
                            const float df = __fsub_rn(qv[qq * d + t], xs);
                            dist[qq] = __builtin_fmaf(df, df, dist[qq]);
                        } else {
                            dist[qq] = __builtin_fmaf(qv[qq * d + t], xs, dist[qq]);
                        }
                    }
                }
            }
        }
        const uint32_t gid = (uint32_t)(id_offset + row);
#pragma unroll
        for (int qq = 0; qq < QB; ++qq) {
            if (qq >= nqb) break;
            float dv = metric == MIVQ_METRIC_L2 ? dist[qq] : -dist[qq];
            if (dv != dv) dv = INFINITY;
            unsigned long long mask = __ballot(valid && pair_less(dv, gid, thr_d[qq], thr_i[qq]));
            while (mask) {
                const int src = __builtin_ctzll(mask);
                mask &= mask - 1;
                const float cd = __shfl(dv, src);
                const uint32_t ci = __shfl(gid, src);
                if (!pair_less(cd, ci, thr_d[qq], thr_i[qq])) continue;
                top[qq].insert(cd, ci, k, lane);
                top[qq].kth(k, thr_d[qq], thr_i[qq]);
            }
        }
    }
    const int64_t part = (int64_t)blockIdx.x * kScanWaves + wv;
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        if (qq < nqb) {
            float* od = part_d + (part * nq + q0 + qq) * k;
            uint32_t* oi = part_i + (part * nq + q0 + qq) * k;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int e = r * 64 + lane;
                if (e < k) { od[e] = top[qq].d[r]; oi[e] = top[qq].id[r]; }
            }
        }
    }
}

// One wave per query: the parts*k candidates (lists laid out (parts, nq, k)) stream through
// a wave-resident top-k, 64 at a time, screened against the cached k-th element.
template <int R>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ in_d, const uint32_t* __restrict__ in_i,
                                                         int parts, int64_t nq, int k, float* __restrict__ out_d,
                                                         uint32_t* __restrict__ out_i, const int* __restrict__ qlist,
                                                         const int* __restrict__ qcount) {
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;  // whole wave
    if (qlist != nullptr && qi >= *qcount) return;
    const int64_t qo = qlist != nullptr ? (int64_t)qlist[qi] : qi;  // output row of list slot qi
    WaveTopK<R> top;
    top.init();
    float thr_d = INFINITY;
    uint32_t thr_i = kNoId;
    const int64_t total = (int64_t)parts * k;
    for (int64_t e0 = 0; e0 < total; e0 += 64) {
        const int64_t e = e0 + lane;
        const bool valid = e < total;
        float cd = INFINITY;
        uint32_t ci = kNoId;
        if (valid) {
            const int64_t p = e / k, j = e - p * k;
            cd = in_d[(p * nq + qi) * k + j];
            ci = in_i[(p * nq + qi) * k + j];
            if (cd != cd) cd = INFINITY;
        }
        unsigned long long mask = __ballot(valid && pair_less(cd, ci, thr_d, thr_i));
        while (mask) {
            const int src = __builtin_ctzll(mask);
            mask &= mask - 1;
            const float vd = __shfl(cd, src);
            const uint32_t vi = __shfl(ci, src);
            if (!pair_less(vd, vi, thr_d, thr_i)) continue;
            top.insert(vd, vi, k, lane);
            top.kth(k, thr_d, thr_i);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < k) { out_d[qo * k + e] = top.d[r]; out_i[qo * k + e] = top.id[r]; }
    }
}

// ---------------------------------------------------------------------------------------------
// Filtered ADC search (M = 16 / 32, ksub = 256): the same canonical fp32 top-k, found in two
// passes.
//
// 1. adc_qstats_kernel / adc_qtab_kernel quantise every query's LUT to 6-bit integers:
//      q[m][c] = min(63, floor((lut[m][c] - min_m) / delta)),  delta = min(range, 2 w) / 63
//    (range = max_m range_m, w = the largest mean offset above min_m: the grid is fine where the
//    rows near the top live, entries above it clamp), one byte per query, 16 queries per 16-B
//    table entry.  A row's sum S = sum_m q[m][code_m] < 2^11 (M <= 32).
// 2. adc_qscan_kernel: four lookups add up inside the bytes (4 x 63 < 256) before one v_perm
//    unpack to u16 pairs, so a (query, row) costs M / 8 byte-adds + M / 4 unpacks + M / 4
//    16-bit adds; every lane keeps, per query, the three smallest keys (S << 16 | step) of its
//    own rows (v_med3 / v_min, registers only), and each wave ("part") finally lists the
//    candidates below a ballot-searched threshold plus its bound B (every unlisted row of the
//    part has S >= B).
// 3. adc_rerank_kernel (one wave per query) evaluates the canonical fp32 distance (the sum over
//    m in order of the fp32 LUT entries, include/mivq.h) of every listed row and keeps the exact
//    top-k.  It is the canonical answer if no row outside the lists can beat its k-th element
//    (E_k): a row part p did not list has S >= B(p), and, with q*delta <= lut - min, its
//    canonical distance is >= LB(S) = base + delta * S - margin (base = sum_m min_m, margin >=
//    the fp32 summation error gamma_M * sum_m max_c |lut[m][c]| plus fp64 slack).  So the query
//    is certified when LB(B(p)) > E_k for every part p; a query that is not (or whose LUT is
//    not finite) is listed for
// 4. the fp32 scan (adc_scan_kernel) re-run on the listed queries only (query indirection; the
//    workgroups of empty slots return at once) and its merge.
// Results are identical to the fp32 scan's for every input.
struct AdcQStat {
    double base, delta, margin;
    int bad, pad;
};

// Integer table: 6-bit entries in bytes (round 5, A/B-measured against 8- and 7-bit entries and
// u16 entries: 6 bits lets four lookups share one unpack, and certified as many queries once the
// grid span followed the mean offset); lanes keep 3 keys per query (2 left ~2 % of the queries
// uncertified on Gaussian rows, 3 none).
// (5 bits, eight lookups per unpack: 3-5 % faster on clustered rows and the config #5 shape, but
// 1.6x slower on 1M x 1536 Gaussian rows, whose queries it mostly fails to certify; r05_s22)
constexpr int kAdcBits = 6;
// (round 6, with the scan VALU-bound: 2 keys -- one v_med3 less per row and query -- measured
// 2.4x / 1.23x slower at 1000 x 1M / the config #5 shape: the uncertified queries' fp32 re-runs)
constexpr int kLaneKeys = 3;
constexpr double kAdcSpan = 2.0;  // the grid's span in mean offsets above the minimum
__host__ __device__ constexpr int adc_qmax(int) { return (1 << kAdcBits) - 1; }

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// grid nq, block 256: per (query, m) the minimum and range (mins[q][m] = min_m), then the
// query's {base, delta, margin, bad}.
__global__ __launch_bounds__(256) void adc_qstats_kernel(const float* __restrict__ lut, int64_t nq, int M,
                                                         float* __restrict__ mins, AdcQStat* __restrict__ qs) {
    __shared__ double s_min[64], s_rng[64], s_abs[64], s_wid[64];
    __shared__ int s_bad;
    const int64_t qi = blockIdx.x;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    for (int m = w; m < M; m += 4) {
        const float4 v = *reinterpret_cast<const float4*>(lut + (qi * M + m) * 256 + 4 * l);
        const bool fin = isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w);
        const float mn = wave_min(fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
        const float mx = wave_max(fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
        const float ab = wave_max(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        // mean offset above the minimum (the scale the rows near the top live on)
        const float wid = wave_sum((v.x - mn) + (v.y - mn) + (v.z - mn) + (v.w - mn)) * (1.0f / 256.0f);
        const bool bad = __ballot(!fin) != 0ull;
        if (l == 0) {
            s_min[m] = mn;
            s_wid[m] = wid;
            s_rng[m] = (double)mx - (double)mn;
            s_abs[m] = ab;
            mins[qi * M + m] = mn;
            if (bad) s_bad = 1;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double base = 0.0, rng = 0.0, mag = 0.0, wid = 0.0;
        for (int m = 0; m < M; ++m) {
            base += s_min[m];
            rng = fmax(rng, s_rng[m]);
            mag += s_abs[m];
            wid = fmax(wid, s_wid[m]);
        }
        AdcQStat st;
        st.base = base;
        // the integer grid spans kAdcSpan x the largest mean offset: entries above it clamp to
        // QMAX (a clamped q still has q delta <= lut - min, so every bound stays a lower bound),
        // and the rows near the top -- small entries in most subspaces -- get a finer grid than
        // the full range would give (round 5: range / 255 certified too few queries on
        // k-means codebooks, whose far centroids stretch the range)
        const double span = fmin(rng, kAdcSpan * wid);
        st.delta = span > 0.0 ? span / (double)adc_qmax(M) : (rng > 0.0 ? rng / (double)adc_qmax(M) : 1.0);
        // fp32 canonical sum: |fl(sum) - sum| <= gamma_{M-1} sum |t| <= gamma_M mag; 2x that, plus
        // fp64 slack for base and delta * S
        st.margin = 2.0 * (double)M * 5.9604644775390625e-8 * mag + 1e-12 * (mag + fabs(base));
        st.bad = s_bad || !isfinite(base) || !isfinite(mag) || !(st.delta > 0.0);
        st.pad = 0;
        qs[qi] = st;
    }
}

// grid (ceil(nq / QB), M), block 256 (code c): one 16-B entry per (m, c) holding the 16 queries'
// bytes; dword w holds queries (4w, 4w + 2, 4w + 1, 4w + 3) in bytes 0..3, so the two byte-pair
// unpacks give the u16 pairs (4w, 4w + 1) and (4w + 2, 4w + 3).  q <= (lut - min) / delta (the
// ratio is shrunk by 2^-50 before the floor, so fp64 rounding never rounds it up past an
// integer).  Entry order (round 6): [m / 16][c][m % 16] -- the 16 subspaces of a half side by
// side in one 256-B bank row per code, so that lanes reading 16 DIFFERENT subspaces hit 16
// different bank slots whatever their codes (adc_qscan_kernel).
template <int QB>
__global__ __launch_bounds__(256) void adc_qtab_kernel(const float* __restrict__ lut, int64_t nq, int M,
                                                       const float* __restrict__ mins,
                                                       const AdcQStat* __restrict__ qs, uint32_t* __restrict__ tab) {
    constexpr int NWD = QB / 4;
    const int64_t qb = blockIdx.x;
    const int m = blockIdx.y, c = threadIdx.x;
    const int qmax = adc_qmax(M);
    uint32_t w[NWD];
#pragma unroll
    for (int j = 0; j < NWD; ++j) w[j] = 0u;
    // every load of the block's QB queries first (rows past nq clamped to the last query, their
    // bytes zeroed below), then the arithmetic: one memory round trip instead of one per query
    // behind the per-query branches
    float lv[QB], mv[QB];
    double dl[QB];
    int bd[QB];
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        const int64_t qi = min(qb * QB + qq, nq - 1);
        lv[qq] = lut[(qi * M + m) * 256 + c];
        mv[qq] = mins[qi * M + m];
        dl[qq] = qs[qi].delta;
        bd[qq] = qs[qi].bad;
    }
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        const double x = ((double)lv[qq] - (double)mv[qq]) / dl[qq] * (1.0 - 8.881784197001252e-16);
        uint32_t v = x >= (double)qmax ? (uint32_t)qmax : x > 0.0 ? (uint32_t)floor(x) : 0u;
        if (qb * QB + qq >= nq || bd[qq]) v = 0u;
        const int r = qq & 3;
        w[qq >> 2] |= v << (8 * (((r & 1) << 1) | (r >> 1)));
    }
    uint32_t* dst = tab + (((qb * (M / 16) + (m >> 4)) * 256 + c) * 16 + (m & 15)) * NWD;
    if constexpr (NWD >= 4) {
#pragma unroll
        for (int j = 0; j < NWD; j += 4) *reinterpret_cast<uint4*>(dst + j) = make_uint4(w[j], w[j + 1], w[j + 2], w[j + 3]);
    } else {
        *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
    }
}

constexpr int kQB = 16;  // queries per integer-table block

// grid (nchunks, ceil(nq / 16)), block kScanWaves waves (the fp32 scan's structure): the byte
// tables of 16 queries in LDS (M * 4 KiB), M = 16 MC, each lane one row per wave-step with its
// code row loaded a step ahead.  No wave-level list during the scan: every lane keeps, per
// query, the kLaneKeys smallest keys (S << 16 | wave-step) of its own rows (v_med3 + v_min per
// row and query, registers only).  At the end each wave ("part") selects from its 192 lane
// candidates per query those with S below T = the largest value with at most K1 candidates
// below it (binary search on ballot counts), writes them (float(S), id) -- the rest of the K1
// slots sentinels -- and its bound B = min(T, min over lanes of the lane's last key's S): every
// row of the part that is not listed has S >= B (a lane's other rows are >= its last kept
// key, a dropped candidate is >= T).  (The round-5 first cut kept wave-resident exact lists
// updated by ballot + shuffle inserts: those inserts were most of its LDS instructions.)

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int MC, bool PIN>
__global__ __launch_bounds__(kScanWaves * 64) void adc_qscan_kernel(
    const uint32_t* __restrict__ qtab, int64_t nq, const uint8_t* __restrict__ codes, int64_t n, int k1,
    int64_t id_offset, int64_t chunk_rows, float* __restrict__ part_d, uint32_t* __restrict__ part_i,
    float* __restrict__ part_b) {
    constexpr int M = 16 * MC;
    constexpr int QB = kQB;
    constexpr int NWD = QB / 4;   // dwords per (m, code) entry (u8 per query)
    constexpr int NACC = QB / 2;  // u16-pair accumulators (queries 2j, 2j + 1)
    extern __shared__ __attribute__((aligned(16))) uint32_t qt[];  // [M][256][NWD]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t q0 = (int64_t)blockIdx.y * QB;
    const int nqb = (int)min<int64_t>(QB, nq - q0);
    {
        const uint4* src = reinterpret_cast<const uint4*>(qtab + (int64_t)blockIdx.y * M * 256 * NWD);
        uint4* dst = reinterpret_cast<uint4*>(qt);
        for (int e = tid; e < M * 256 * NWD / 4; e += kScanWaves * 64) dst[e] = src[e];
    }
    __syncthreads();

    // per query: the lane's kLaneKeys smallest keys (S << 16 | step) in increasing order, ~0u = none
    uint32_t mk[kLaneKeys][QB];
#pragma unroll
    for (int t = 0; t < kLaneKeys; ++t)
#pragma unroll
        for (int qq = 0; qq < QB; ++qq) mk[t][qq] = 0xFFFFFFFFu;

    const int64_t rbeg = (int64_t)blockIdx.x * chunk_rows;
    const int64_t rend = min(n, rbeg + chunk_rows);
    uint4 cw[MC];
    auto fetch = [&](int64_t row) __attribute__((always_inline)) {
        const uint4* cr = reinterpret_cast<const uint4*>(codes + row * (16 * MC));
#pragma unroll
        for (int c = 0; c < MC; ++c) cw[c] = row < rend ? cr[c] : make_uint4(0u, 0u, 0u, 0u);
    };
    // Conflict-free lookups (round 6).  A ds_read_b128 is served in four 16-lane groups, one LDS
    // cycle per group when its 16 lanes hit 16 different 16-B slots of the 256-B bank row
    // (MI355X_MICROARCH.md §LDS); with the table [m][code], slot = code % 16 is random and a group
    // took ~3 cycles.  With the table [m / 16][code][m % 16] the slot is m % 16, so at every
    // lookup step the lanes of a group read 16 different subspaces: lane l (r = l % 16, rd = r / 4,
    // rb = r % 4; every 16-lane group of ds_read_b128 holds each r once) takes at step (word k,
    // byte b) subspace mm = 4 ((k + rd) % 4) + (b + rb) % 4 of the half.  The integer sums do
    // not depend on the order of their terms.  Per lookup the address is still ONE VALU: a
    // v_perm builds code << 8 | mm << 4 from the code word (byte (b + rb) % 4 of its dword
    // rotated by rd) and a per-lane register of the four mm << 4 values of word k.
    const uint32_t rl = (uint32_t)lane & 15u, rd = rl >> 2, rb = rl & 3u;
    uint32_t mo[4], psel[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t v = 0u;
#pragma unroll
        for (int b = 0; b < 4; ++b) v |= ((4u * ((k + rd) & 3u) + ((b + rb) & 3u)) << 4) << (8 * b);
        mo[k] = v;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)  // byte0 <- mo byte b (S1), byte1 <- code byte (b + rb) % 4 (S0), bytes 2, 3 <- 0
        psel[b] = (uint32_t)b | ((4u + ((b + rb) & 3u)) << 8) | 0x0C0C0000u;
#ifndef MIVQ_QSCAN_BUF
#define MIVQ_QSCAN_BUF 1
#endif
    // M = 16 (MC = 1): the code row's dwords come rotated by rd straight from memory: four dword buffer loads per
    // 16-B half with per-lane offsets fixed for the whole kernel (the lane's row and rotation)
    // and the wave-step in the scalar soffset, range-checked over the chunk (rows past it read
    // zeros), so neither the rotation nor the row address costs VALU.  (M = 32: the select
    // rotation below; eight such loads per row spilled there.)
    // (M = 32: the buffer path in the pinned kernel only -- the unpinned one spills with it --
    // and launch_qscan always takes the pinned kernel at M = 32: 2-3 % faster at 1000 / 4000 x 1M
    // and 10,000 x 6.65M, profiles/r06_s34)
#ifndef MIVQ_QSCAN_M32BUF
#define MIVQ_QSCAN_M32BUF 1
#endif
    constexpr bool kBuf = MIVQ_QSCAN_BUF && (MC == 1 || (MIVQ_QSCAN_M32BUF && MC == 2 && PIN));
    // the even-query unpack (bytes 0 and 2 -> the u16 pair) is a mask: with the mask in an SGPR it
    // is a 32-bit v_and instead of a 64-bit v_perm (the scan is VALU-issue bound, DESIGN 3.3;
    // 1.2-1.5 % faster at M = 16 / 32, 1000 x 1M and the config #5 shape, profiles/r06_s35)
    uint32_t mlo;
    asm volatile("s_mov_b32 %0, 0xff00ff" : "=s"(mlo));
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(codes + rbeg * (16 * MC)), 0, (int)(max<int64_t>(0, rend - rbeg) * (16 * MC)), 0x00020000);
    int voffc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voffc[i] = (wv * 64 + lane) * (16 * MC) + 4 * (int)((i + rd) & 3u);
    auto fetchb_to = [&](int64_t base, uint4 (&dst)[MC]) __attribute__((always_inline)) {
        const int so = (int)(base - rbeg) * (16 * MC);
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            dst[c].x = __builtin_amdgcn_raw_buffer_load_b32(crs, voffc[0], so + 16 * c, 0);
            dst[c].y = __builtin_amdgcn_raw_buffer_load_b32(crs, voffc[1], so + 16 * c, 0);
            dst[c].z = __builtin_amdgcn_raw_buffer_load_b32(crs, voffc[2], so + 16 * c, 0);
            dst[c].w = __builtin_amdgcn_raw_buffer_load_b32(crs, voffc[3], so + 16 * c, 0);
        }
    };
    auto fetchb = [&](int64_t base) __attribute__((always_inline)) { fetchb_to(base, cw); };
    // the code row's dwords rotated by rd within each 16-B half (two select levels)
    auto rot = [&](uint4 w) __attribute__((always_inline)) {
        const bool r1 = (rd & 1u) != 0u, r2 = (rd & 2u) != 0u;
        const uint32_t t0 = r1 ? w.y : w.x, t1 = r1 ? w.z : w.y, t2 = r1 ? w.w : w.z, t3 = r1 ? w.x : w.w;
        return make_uint4(r2 ? t2 : t0, r2 ? t3 : t1, r2 ? t0 : t2, r2 ? t1 : t3);
    };
    // entries of kAdcBits < 8 bits: 2^(8 - bits) lookups add up in the bytes themselves (no carry
    // crosses a byte) before one unpack to the u16 pairs
    constexpr int UNP = 1 << (8 - kAdcBits);
    static_assert(UNP == 1 || UNP == 2 || UNP == 4 || UNP == 8, "entry bits");
    const int64_t first = rbeg + (int64_t)wv * 64;
    if constexpr (kBuf) fetchb(rbeg);
    else fetch(first + lane);
    uint32_t step = 0;
    for (int64_t base = first; base < rend; base += kScanWaves * 64, ++step) {
        const int64_t row = base + lane;
        uint32_t acc[NACC];
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = 0u;
        uint4 cur[MC];
#pragma unroll
        for (int c = 0; c < MC; ++c) cur[c] = cw[c];
        if constexpr (kBuf) fetchb(base - (int64_t)wv * 64 + kScanWaves * 64);
        else fetch(row + kScanWaves * 64);
        // PIN (round 6): the next row's loads issue here, at the top of the step, so they have the
        // whole step to land (the compiler otherwise places them ~30 % into it, and the copy at
        // the loop latch waits for them): 8 % faster at the config #5 shape, 2 % slower when one
        // round of workgroups covers the search (1000 x 1M), so launch_qscan picks it by shape
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        uint32_t wq[4 * MC];
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            if constexpr (!kBuf) cur[c] = rot(cur[c]);
            wq[4 * c + 0] = cur[c].x; wq[4 * c + 1] = cur[c].y;
            wq[4 * c + 2] = cur[c].z; wq[4 * c + 3] = cur[c].w;
        }
        // unrolled over the code words (round 5: 0.560 -> 0.531 ms per 1000 x 1M at M = 16,
        // profiles/r05_s20): word jw is read straight from its register wq[jw]
        uint32_t a8[4] = {0u, 0u, 0u, 0u};  // byte sums of up to UNP lookups (across words)
#pragma unroll
        for (int jw = 0; jw < 4 * MC; ++jw) {
            const uint32_t wrd = wq[jw];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                // code << 8 | mm << 4 in ONE v_perm; the half's 64 KiB (M = 32) is one more op
                // (the ds_read offset field holds 16 bits); qt is this kernel's only LDS, so the
                // dynamic segment starts at address 0 (guarded at the bound store below)
                uint32_t o1 = __builtin_amdgcn_perm(wrd, mo[jw & 3], psel[b]);
                if (jw >= 4) o1 |= (uint32_t)(jw >> 2) << 16;
                const u32x4v t0 = *(reinterpret_cast<const lds_u4*>((uintptr_t)o1));
                const uint32_t tv[4] = {t0.x, t0.y, t0.z, t0.w};
#pragma unroll
                for (int wd = 0; wd < 4; ++wd) a8[wd] = ((4 * jw + b) % UNP == 0) ? tv[wd] : a8[wd] + tv[wd];
                if ((4 * jw + b + 1) % UNP == 0) {
#pragma unroll
                    for (int wd = 0; wd < 4; ++wd) {  // bytes (4w, 4w+2, 4w+1, 4w+3) -> u16 pairs
                        acc[2 * wd] += a8[wd] & mlo;
                        acc[2 * wd + 1] += __builtin_amdgcn_perm(a8[wd], a8[wd], 0x0C030C01u);
                    }
                }
            }
        }
        // a row past the chunk takes part in nothing (the last step only)
        const uint32_t inval = row < rend ? 0u : 0xFFFFFFFFu;
        auto insert = [&](int qq, uint32_t key) __attribute__((always_inline)) {
            // sorted insert into (m0 <= m1 [<= m2]): med3 / min per slot
            if constexpr (kLaneKeys == 3) mk[2][qq] = umed3(mk[1][qq], mk[2][qq], key);
            mk[1][qq] = umed3(mk[0][qq], mk[1][qq], key);
            mk[0][qq] = min(mk[0][qq], key);
        };
        // the row's low half once per row: each key is then one v_lshl_or / v_and_or
        const uint32_t lo16 = step | inval;
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            insert(2 * j, (acc[j] << 16) | lo16);                 // query 2j
            insert(2 * j + 1, (acc[j] & 0xFFFF0000u) | lo16);     // query 2j + 1
        }
    }
    // per query: select the candidates below T, the bound B, write K1 slots.  A lane's unlisted
    // rows have keys >= its last kept key, so B = min(T, min over lanes of that key's S).
    const int64_t part = (int64_t)blockIdx.x * kScanWaves + wv;
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
        if (qq >= nqb) continue;
        uint32_t sv[kLaneKeys];
#pragma unroll
        for (int t = 0; t < kLaneKeys; ++t) sv[t] = mk[t][qq] >> 16;  // 0xFFFF: no candidate
        // T: the largest t in [0, 0xFFFF] with #{candidates with S < t} <= k1.  Real sums are at
        // most kSMax = M * QMAX (keys of rows past the chunk have S = 0xFFFF: never candidates),
        // so the search runs over [0, kSMax + 1] (11 steps at M = 16 instead of 16) and a result
        // of kSMax + 1 (every kept key listed) stands for 0xFFFF
        constexpr uint32_t kSMax = (uint32_t)M * ((1u << kAdcBits) - 1u);
        uint32_t lo = 0, hi = kSMax + 1;
        while (lo < hi) {  // wave-uniform
            const uint32_t mid = (lo + hi + 1) >> 1;
            int cnt = 0;
#pragma unroll
            for (int t = 0; t < kLaneKeys; ++t) cnt += __popcll(__ballot(sv[t] < mid));
            if (cnt <= k1) lo = mid; else hi = mid - 1;
        }
        const uint32_t T = lo > kSMax ? 0xFFFFu : lo;
        // min over lanes of the last kept key's S: a wave reduction, not a ballot search
        uint32_t blo = sv[kLaneKeys - 1];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) blo = min(blo, (uint32_t)__shfl_xor((int)blo, o));
        const uint32_t B = min(T, blo);
        float* od = part_d + (part * nq + q0 + qq) * k1;
        uint32_t* oi = part_i + (part * nq + q0 + qq) * k1;
        int used = 0;
#pragma unroll
        for (int t = 0; t < kLaneKeys; ++t) {
            const bool take = sv[t] < T;
            const uint64_t bt = __ballot(take);
            if (take) {
                const int at = used + __popcll(bt & below);
                od[at] = (float)sv[t];
                oi[at] = (uint32_t)(id_offset + first + (int64_t)(mk[t][qq] & 0xFFFFu) * (kScanWaves * 64) + lane);
            }
            used += __popcll(bt);
        }
        for (int e = used + lane; e < k1; e += 64) { od[e] = INFINITY; oi[e] = kNoId; }
        // B = 0xFFFF: every row of the part is listed
        // (the lookups take the table at LDS address 0, i.e. no static LDS in this kernel; were
        // there any, every bound reads 0 and every query goes to the fp32 re-run: slow, never wrong)
        if (lane == 0)
            part_b[part * nq + q0 + qq] = __builtin_amdgcn_groupstaticsize() != 0 ? 0.0f : B >= 0xFFFFu ? INFINITY : (float)B;
    }
}

// The rerank's first 64 entries all beat the empty list's +inf threshold: instead of ~28
// sequential wave inserts (each a ballot and four cross-lane moves in a dependent chain) they are
// sorted at once -- bitonic, 21 compare-exchange stages on (dist, id) -- and become the list
// (R = 1, k <= 64: element e in lane e).  The k smallest pairs are unique, so the list equals the
// one the inserts build.
__device__ __forceinline__ void rr_seed(WaveTopK<1>& top, bool valid, float dv, uint32_t id, int k, int lane,
                                        float& thr_d, uint32_t& thr_i) {
    float d = valid ? dv : INFINITY;
    uint32_t i = valid ? id : kNoId;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const float od = __shfl_xor(d, stride);
            const uint32_t oi = (uint32_t)__shfl_xor((int)i, stride);
            const bool up = (lane & size) == 0 || size == 64;  // ascending run
            const bool lower = (lane & stride) == 0;
            const bool take = lower == up ? pair_less(od, oi, d, i) : pair_less(d, i, od, oi);
            d = take ? od : d;
            i = take ? oi : i;
        }
    }
    top.d[0] = d;
    top.id[0] = i;
    top.kth(k, thr_d, thr_i);
}

// One wave per query: canonical fp32 distances of the listed rows, exact top-k, certificate.
template <int R, int MC>
__global__ __launch_bounds__(256) void adc_rerank_kernel(const float* __restrict__ lut, int64_t nq,
                                                         const uint8_t* __restrict__ codes, int64_t id_offset,
                                                         const uint32_t* __restrict__ pi, const float* __restrict__ pb,
                                                         int parts, int k1, int k, const AdcQStat* __restrict__ qs,
                                                         float* __restrict__ out_d, uint32_t* __restrict__ out_i,
                                                         int* __restrict__ fail_list, int* __restrict__ fail_count,
                                                         int lut16) {
    constexpr int M = 16 * MC;
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;  // whole wave
    const AdcQStat st = qs[qi];
    WaveTopK<R> top;
    top.init();
    float thr_d = INFINITY;
    uint32_t thr_i = kNoId;
    // the wave's query LUT staged in LDS (coalesced), so the candidates' M lookups each are LDS
    // reads instead of random 4-B global reads (wave-private region: no workgroup barrier;
    // round 5: 0.478 -> 0.468 ms per 1000 x 1M search at M = 16, 0.826 -> 0.794 at M = 32,
    // 3.07 -> 2.95 ms at the config #5 shape, profiles/r05_s32)
    extern __shared__ __attribute__((aligned(16))) float rls[];
    float* lq = rls + (threadIdx.x >> 6) * M * 256;
    {
        const float* src = lut + qi * M * 256;
        if (lut16) {
#pragma unroll
            for (int i = 0; i < M; ++i)
                reinterpret_cast<float4*>(lq)[i * 64 + lane] = reinterpret_cast<const float4*>(src)[i * 64 + lane];
        } else {
            for (int i = lane; i < M * 256; i += 64) lq[i] = src[i];
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's own stores
        __builtin_amdgcn_wave_barrier();
    }
    const int64_t total = (int64_t)parts * k1;
    auto eval = [&](bool valid, const uint4 (&cw)[MC]) __attribute__((always_inline)) {
        float dv = INFINITY;
        if (valid) {
            float t[M];
#pragma unroll
            for (int c = 0; c < MC; ++c) {
                const uint32_t wd[4] = {cw[c].x, cw[c].y, cw[c].z, cw[c].w};
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    t[16 * c + j] = lq[(16 * c + j) * 256 + ((wd[j >> 2] >> (8 * (j & 3))) & 0xFFu)];
            }
            dv = 0.0f;
#pragma unroll
            for (int m = 0; m < M; ++m) dv += t[m];  // the canonical order
            if (dv != dv) dv = INFINITY;
        }
        return dv;
    };
    auto offer = [&](bool first, bool valid, float dv, uint32_t id) __attribute__((always_inline)) {
        // (round 6 split, profiling builds traced in r06_s39: 33 us per 1000 x 1M search, of which
        // ~12.5 us were the sequential wave inserts -- the first step's now one sort, r06_s40)
        if constexpr (R == 1) {
            if (first) rr_seed(top, valid, dv, id, k, lane, thr_d, thr_i);
            else top.offer(valid, dv, id, k, lane, thr_d, thr_i);
        } else {
            top.offer(valid, dv, id, k, lane, thr_d, thr_i);
        }
    };
    // (round 6: ids and code rows by range-checked buffer loads in chunks of 8 steps -- all of a
    // chunk's gathers in flight at once -- measured 26.5 -> 23.9 us here but neutral to 0.3 %
    // slower end to end at M = 32 and the config #5 shape, r06_s41: not kept)
    // three-stage pipeline over the list in steps of 64 entries (round 6): the ids two steps
    // ahead and the code rows (which need those ids) one step ahead are in flight while a step
    // is evaluated, instead of an id load -> row gather -> lookups round trip per step
    auto ld_id = [&](int64_t e0) __attribute__((always_inline)) {
        const int64_t e = e0 + lane;
        uint32_t id = kNoId;
        if (e < total) {
            const int64_t p = e / k1, j = e - p * k1;
            id = pi[(p * nq + qi) * k1 + j];
        }
        return id;
    };
    auto ld_row = [&](uint32_t id, uint4 (&cw)[MC]) __attribute__((always_inline)) {
        const uint4* cr = reinterpret_cast<const uint4*>(codes + ((int64_t)(id != kNoId ? id : (uint32_t)id_offset) - id_offset) * M);
#pragma unroll
        for (int c = 0; c < MC; ++c) cw[c] = id != kNoId ? cr[c] : make_uint4(0u, 0u, 0u, 0u);
    };
    uint32_t id_cur = ld_id(0), id_nxt = ld_id(64);
    uint4 cw_cur[MC];
    ld_row(id_cur, cw_cur);
    for (int64_t e0 = 0; e0 < total; e0 += 64) {
        const uint32_t id_far = ld_id(e0 + 128);
        uint4 cw_nxt[MC];
        ld_row(id_nxt, cw_nxt);
        const uint32_t id = id_cur;
        const bool valid = id != kNoId;
        offer(e0 == 0, valid, eval(valid, cw_cur), id);
        id_cur = id_nxt;
        id_nxt = id_far;
#pragma unroll
        for (int c = 0; c < MC; ++c) cw_cur[c] = cw_nxt[c];
    }
    // certificate: every part's bound B (its unlisted rows have S >= B) must put them above E_k
    bool ok = !st.bad;
    for (int p0 = 0; p0 < parts; p0 += 64) {
        const int p = p0 + lane;
        bool f = false;
        if (p < parts) {
            const float B = pb[(int64_t)p * nq + qi];
            if (B < INFINITY) {
                const double lb = st.base + st.delta * (double)B - st.margin;
                f = !(lb > (double)thr_d);
            }
        }
        if (__ballot(f) != 0ull) ok = false;
    }
    if (ok) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = r * 64 + lane;
            if (e < k) { out_d[qi * k + e] = top.d[r]; out_i[qi * k + e] = top.id[r]; }
        }
    } else if (lane == 0) {
        fail_list[atomicAdd(fail_count, 1)] = (int)qi;
    }
}

int adc_qb(int M, int ksub) {
    const int64_t per = (int64_t)M * ksub * 4;
    const int64_t budget = 128 * 1024;
    if (per * 8 <= budget) return 8;
    if (per * 4 <= budget) return 4;
    if (per * 2 <= budget) return 2;
    if (per <= 160 * 1024) return 1;
    return 0;
}

// Row chunks per query block.  The scan workgroups (16 waves, up to 128 KiB of LDS) run one
// per CU, so the grid of nch * qblocks workgroups takes ceil(nch * qblocks / 256) rounds, each
// as long as one workgroup's table fill (about half a wave-step of 1024 rows) plus its
// ceil(n / nch / 1024) wave-steps: pick the nch of least total time (the smallest on ties:
// fewer partial lists; a larger count must gain 2 %: the model is coarse, and every chunk adds
// a part list per query).  nq = 1000 at QB = 8, n = 1M: 2 chunks, 250 workgroups in one round,
// instead of 625 in three of which the last is 44 % full.
int64_t adc_chunks(int64_t nq, int64_t n, int QB) {
    const int64_t qblocks = ceil_div(nq, QB);
    const int64_t step_rows = 64 * kScanWaves;
    const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(1024, ceil_div(n, step_rows)));
    int64_t best = 1;
    double best_cost = 0.0;
    for (int64_t nch = 1; nch <= cap; ++nch) {
        const double cost = (double)ceil_div(nch * qblocks, 256) * ((double)ceil_div(ceil_div(n, nch), step_rows) + 0.5);
        if (nch == 1 || cost < best_cost * 0.98) { best = nch; best_cost = cost; }
    }
    return best;
}

template <int R, int QB>
hipError_t launch_scan(const float* lut, int64_t nq, const uint8_t* codes, int64_t n, int M, int ksub, int k,
                       int64_t id_offset, int64_t nch, float* pd, uint32_t* pi, hipStream_t st,
                       const int* qlist = nullptr, const int* qcount = nullptr, bool small_grid = false) {
    const size_t smem = (size_t)QB * M * ksub * sizeof(float);
    const bool vec = ksub == 256 && reinterpret_cast<uintptr_t>(codes) % 16 == 0;
    auto kern = vec && M == 16 ? adc_scan_kernel<R, QB, 1> : vec && M == 32 ? adc_scan_kernel<R, QB, 2>
                                                                             : adc_scan_kernel<R, QB, 0>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    const int64_t chunk_rows = ceil_div(n, nch);
    // the re-run of uncertified queries: one round of workgroups looping over the list slots
    // (small_grid, a test hook: one column, so every workgroup walks several slot blocks)
    const int64_t qgrid = qlist != nullptr ? (small_grid ? 1 : std::max<int64_t>(1, std::min<int64_t>(ceil_div(nq, QB), 256 / nch)))
                                           : ceil_div(nq, QB);
    hipLaunchKernelGGL(kern, dim3((unsigned)nch, (unsigned)qgrid), dim3(kScanWaves * 64), smem, st, lut, nq, codes,
                       n, M, ksub, k, id_offset, chunk_rows, pd, pi, qlist, qcount);
    return hipGetLastError();
}

// Row chunks of the re-run of uncertified queries: ~32k rows each (one failed query costs a
// few tens of microseconds, not a whole-database workgroup), as long as the re-run's part
// lists -- sized for every query, since the host does not know how many fail -- stay within
// kRerunListBytes: (16 parts per chunk) x nq x k x 8 B per chunk.  At nq = 10,000, k = 32 that
// is 40 MB per chunk, so 6 chunks (a failed query then scans ~1/6 of the rows per workgroup:
// slower, never wrong); below 1,000 queries at k = 10 the 256 chunks fit.  (the
// unbounded form sized 10.5 GB at n = 10M, nq = 10k, k = 32.)
constexpr size_t kRerunListBytes = size_t(256) << 20;
int64_t adc_fallback_chunks(int64_t nq, int64_t n, int k) {
    const int64_t want = std::max<int64_t>(1, std::min<int64_t>(256, ceil_div(n, 32768)));
    const size_t per_chunk = (size_t)kScanWaves * (size_t)std::max<int64_t>(nq, 1) * (size_t)k * 8u;
    return std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)(kRerunListBytes / per_chunk)));
}

template <int R>
hipError_t launch_scan_r(int QB, const float* lut, int64_t nq, const uint8_t* codes, int64_t n, int M, int ksub,
                         int k, int64_t id_offset, int64_t nch, float* pd, uint32_t* pi, hipStream_t st,
                         const int* qlist = nullptr, const int* qcount = nullptr, bool sg = false) {
    switch (QB) {
        case 8: return launch_scan<R, 8>(lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg);
        case 4: return launch_scan<R, 4>(lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg);
        case 2: return launch_scan<R, 2>(lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg);
        default: return launch_scan<R, 1>(lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg);
    }
}

int flat_qb(int d) {
    const int64_t per = (int64_t)d * 4;
    if (per * 8 <= 96 * 1024) return 8;
    if (per * 4 <= 96 * 1024) return 4;
    if (per * 2 <= 96 * 1024) return 2;
    if (per <= 160 * 1024) return 1;
    return 0;
}

template <int R, int QB>
hipError_t launch_flat(const float* q, int64_t nq, const float* x, int64_t n, int d, int metric, int k,
                       int64_t id_offset, int64_t nch, float* pd, uint32_t* pi, hipStream_t st) {
    const size_t smem = (size_t)QB * d * sizeof(float);
    auto kern = flat_scan_kernel<R, QB>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)nch, (unsigned)ceil_div(nq, QB)), dim3(kScanWaves * 64), smem, st, q, nq, x, n, d,
                       metric, k, id_offset, ceil_div(n, nch), pd, pi);
    return hipGetLastError();
}

template <int R>
hipError_t launch_flat_r(int QB, const float* q, int64_t nq, const float* x, int64_t n, int d, int metric, int k,
                         int64_t id_offset, int64_t nch, float* pd, uint32_t* pi, hipStream_t st) {
    switch (QB) {
        case 8: return launch_flat<R, 8>(q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st);
        case 4: return launch_flat<R, 4>(q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st);
        case 2: return launch_flat<R, 2>(q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st);
        default: return launch_flat<R, 1>(q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st);
    }
}

// Filtered path eligibility by shape (the workspace is sized on shape alone; the diagnostic
// flag MIVQ_ADC_FORCE_EXACT runs the fp32 scan for every query in the same workspace).
// (queries per table block: the variants whose lists fit the 128 registers of the 16-wave scan)
// Part lists keep K1 = k + kListSlack entries (at most 256): the certificate bounds the rows a
// part did NOT list by its K1-th entry, so a part holding some of the k best rows still
// certifies when its K1-th row is clearly worse (with K1 = k, the part holding the best row of
// a k = 1 search never could).
constexpr int kListSlack = 4;
int adc_k1(int k) { return k + kListSlack; }
// k <= 32: a part's 192 lane candidates (kLaneKeys = 3 per lane) carry the k best rows with room to spare;
// for larger k the per-lane bound (a lane's second-best) sits too close to the k-th distance to
// certify, and the fp32 scan serves those searches
bool adc_filtered_shape(int M, int ksub, int k) { return ksub == 256 && (M == 16 || M == 32) && k <= 32; }
int adc_fqb(int M, int k) { return kQB; }

// Row chunks of the filtered (integer) scan: the cost model's, then, when its grid fits one round
// of the CUs, at least 4 chunks and at most 1024 wave-steps per chunk (the grid then takes several
// rounds and launch_qscan the pinned-prefetch kernel).  Measured (round 6, profiles/r06_s30, 1M
// rows unless noted; results identical): 2000 queries 0.99 -> 0.79 ms, 4000 queries 1.77 ->
// 1.44 ms, 1000 x 6.65M 2.65 -> 2.20 ms, 3000 x 6.65M 6.57 -> 6.18 ms, while 500 / 1000 queries
// over 1M-4M rows (model already at 4+ chunks, <= 1024 steps) and the multi-round config #5 grid
// keep the model's count (more chunks there measured 1-17 % slower).
int64_t adc_qscan_chunks(int64_t nq, int64_t n, int QB) {
    int64_t nch = adc_chunks(nq, n, QB);
    const int64_t qblocks = ceil_div(nq, QB), step_rows = 64 * kScanWaves;
    const int64_t most = std::max<int64_t>(1, std::min<int64_t>(1024, ceil_div(n, step_rows)));
    if (nch * qblocks <= 256)
        while (nch < most && (nch < 4 || ceil_div(ceil_div(n, nch), step_rows) > 1024)) nch = std::min(most, 2 * nch);
    return nch;
}

struct AdcFilteredLayout {
    size_t stats, mins, tab, p1d, p1i, p1b, fail, total;
    int64_t nch, parts;
    int k1;
};

AdcFilteredLayout adc_filtered_layout(int64_t nq, int64_t n, int M, int k, size_t off) {
    AdcFilteredLayout L{};
    const int QB = adc_fqb(M, k);
    L.k1 = adc_k1(k);
    // the part lists stay within ~1 GiB where the chunk model would ask for more (100k queries:
    // 2 chunks instead of 12, at the same modelled time), and a lane's step index is 16 bits: at
    // most 65535 wave-steps (of 1024 rows) per chunk
    const size_t per_chunk = (size_t)kScanWaves * (size_t)nq * (size_t)L.k1 * 8u;
    const int64_t cap = std::max<int64_t>(1, (int64_t)((size_t(1) << 30) / per_chunk));
    L.nch = std::max<int64_t>(std::min<int64_t>(adc_qscan_chunks(nq, n, QB), cap), ceil_div(n, (int64_t)65535 * kScanWaves * 64));
    L.parts = L.nch * kScanWaves;
    L.stats = off;  off = align_up(off + (size_t)nq * sizeof(AdcQStat), 256);
    L.mins = off;   off = align_up(off + (size_t)nq * M * sizeof(float), 256);
    L.tab = off;    off = align_up(off + (size_t)ceil_div(nq, QB) * M * 256 * QB, 256);
    L.p1d = off;    off = align_up(off + (size_t)L.parts * nq * L.k1 * sizeof(float), 256);
    L.p1i = off;    off = align_up(off + (size_t)L.parts * nq * L.k1 * sizeof(uint32_t), 256);
    L.p1b = off;    off = align_up(off + (size_t)L.parts * nq * sizeof(float), 256);
    L.fail = off;   off = align_up(off + (size_t)(nq + 1) * sizeof(int), 256);
    L.total = off;
    return L;
}

template <int MC>
hipError_t launch_qscan(const uint32_t* tab, int64_t nq, const uint8_t* codes, int64_t n, int k1, int64_t id_offset,
                        const AdcFilteredLayout& L, float* p1d, uint32_t* p1i, float* p1b, hipStream_t st) {
    constexpr int M = 16 * MC;
    // the pinned prefetch when the workgroups take more than one round of the chip's CUs
#ifndef MIVQ_QSCAN_PIN_MODE
#define MIVQ_QSCAN_PIN_MODE 2  // 0: never, 1: always, 2: by shape
#endif
    const bool pin = MIVQ_QSCAN_PIN_MODE == 1 || (MIVQ_QSCAN_PIN_MODE == 2 && L.nch * ceil_div(nq, kQB) > 256) ||
                     (MIVQ_QSCAN_M32BUF && MC == 2);
    auto kern = pin ? adc_qscan_kernel<MC, true> : adc_qscan_kernel<MC, false>;
    const int smem = M * 256 * kQB;
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)L.nch, (unsigned)ceil_div(nq, kQB)), dim3(kScanWaves * 64), smem, st, tab,
                       nq, codes, n, k1, id_offset, ceil_div(n, L.nch), p1d, p1i, p1b);
    return hipGetLastError();
}

hipError_t launch_filtered(int M, const float* lut, int64_t nq, const uint8_t* codes, int64_t n, int k,
                           int64_t id_offset, unsigned char* ws, const AdcFilteredLayout& L, float* dists,
                           uint32_t* ids, hipStream_t st) {
    const int QB = adc_fqb(M, k), k1 = L.k1;
    auto* qs = reinterpret_cast<AdcQStat*>(ws + L.stats);
    auto* mins = reinterpret_cast<float*>(ws + L.mins);
    auto* tab = reinterpret_cast<uint32_t*>(ws + L.tab);
    auto* p1d = reinterpret_cast<float*>(ws + L.p1d);
    auto* p1i = reinterpret_cast<uint32_t*>(ws + L.p1i);
    auto* p1b = reinterpret_cast<float*>(ws + L.p1b);
    int* fail_count = reinterpret_cast<int*>(ws + L.fail);
    int* fail_list = fail_count + 1;
    hipError_t e = hipMemsetAsync(fail_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    // (round 6: the two launches fused into one workgroup per 16-query block measured slower --
    // 0.422 vs 0.406 ms per 1000 x 1M search: 63 workgroups leave most CUs idle; profiles/r06_s5)
    hipLaunchKernelGGL(adc_qstats_kernel, dim3((unsigned)nq), dim3(256), 0, st, lut, nq, M, mins, qs);
    const dim3 tgrid((unsigned)ceil_div(nq, QB), (unsigned)M);
    if (QB == 16)
        hipLaunchKernelGGL(adc_qtab_kernel<16>, tgrid, dim3(256), 0, st, lut, nq, M, mins, qs, tab);
    else
        hipLaunchKernelGGL(adc_qtab_kernel<8>, tgrid, dim3(256), 0, st, lut, nq, M, mins, qs, tab);
    e = M == 16 ? launch_qscan<1>(tab, nq, codes, n, k1, id_offset, L, p1d, p1i, p1b, st)
                : launch_qscan<2>(tab, nq, codes, n, k1, id_offset, L, p1d, p1i, p1b, st);
    if (e != hipSuccess) return e;
    const int R = (k + 63) / 64;
    const dim3 rgrid((unsigned)ceil_div(nq, 4));
    const int lut16 = reinterpret_cast<uintptr_t>(lut) % 16 == 0;
    const size_t rsm = (size_t)4 * M * 256 * sizeof(float);  // four query LUTs: 64 / 128 KiB
    // the buffer-load rerank needs 32-bit byte offsets into the codes and into the part lists
#define MIVQ_RR(RR, MM)                                                                                              \
    {                                                                                                                \
        e = hipFuncSetAttribute((const void*)adc_rerank_kernel<RR, MM>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)rsm);                                                                           \
        if (e != hipSuccess) return e;                                                                               \
        hipLaunchKernelGGL((adc_rerank_kernel<RR, MM>), rgrid, dim3(256), rsm, st, lut, nq, codes, id_offset, p1i,  \
                           p1b, (int)L.parts, k1, k, qs, dists, ids, fail_list, fail_count, lut16);                  \
    }
    (void)R;  // k <= 32: one list register
    if (M == 16) MIVQ_RR(1, 1)
    else MIVQ_RR(1, 2)
#undef MIVQ_RR
    return hipGetLastError();
}

}  // namespace

hipError_t launch_topk_merge(const float* pd, const uint32_t* pi, int parts, int64_t nq, int k, float* od, uint32_t* oi,
                        hipStream_t st, const int* qlist, const int* qcount) {
    const dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
    switch ((k + 63) / 64) {
        case 1: hipLaunchKernelGGL(topk_merge_kernel<1>, grid, block, 0, st, pd, pi, parts, nq, k, od, oi, qlist, qcount); break;
        case 2: hipLaunchKernelGGL(topk_merge_kernel<2>, grid, block, 0, st, pd, pi, parts, nq, k, od, oi, qlist, qcount); break;
        case 3: hipLaunchKernelGGL(topk_merge_kernel<3>, grid, block, 0, st, pd, pi, parts, nq, k, od, oi, qlist, qcount); break;
        default: hipLaunchKernelGGL(topk_merge_kernel<4>, grid, block, 0, st, pd, pi, parts, nq, k, od, oi, qlist, qcount); break;
    }
    return hipGetLastError();
}

}  // namespace mivq

using namespace mivq;

// The tiled path (pairwise chains on packed VALU + segmented top-k) wins once there are
// enough queries to fill a 128-row tile; the streaming scan keeps the small-batch cases.
static bool flat_use_tiled(int64_t nq, int64_t n) { return nq >= 16 && n >= 4096; }

extern "C" size_t mivq_flat_search_workspace_bytes(int64_t nq, int64_t n, int32_t d, int32_t k) {
    if (nq <= 0 || n <= 0 || d <= 0 || k <= 0) return 0;
    if (flat_use_tiled(nq, n)) return flat_tiled_workspace_bytes(nq, n, k);
    const int QB = flat_qb(d);
    if (QB == 0) return 0;
    const int64_t parts = adc_chunks(nq, n, QB) * kScanWaves;
    return align_up((size_t)parts * nq * k * sizeof(float), 256) + align_up((size_t)parts * nq * k * 4, 256);
}

extern "C" int mivq_flat_search(const float* q, int64_t nq, const float* x, int64_t n, int32_t d, int32_t metric,
                                int32_t k, int64_t id_offset, void* workspace, size_t workspace_bytes, float* dists,
                                uint32_t* ids, void* stream) {
    MIVQ_REQUIRE(nq >= 0 && n >= 0 && d > 0 && k > 0, MIVQ_ERR_INVALID, "flat_search: bad sizes");
    MIVQ_REQUIRE(k <= 256, MIVQ_ERR_UNSUPPORTED, "flat_search: k=%d > 256", k);
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "flat_search: metric %d", metric);
    const int QB = flat_qb(d);
    MIVQ_REQUIRE(QB > 0 || flat_use_tiled(nq, n), MIVQ_ERR_UNSUPPORTED, "flat_search: d=%d too large for LDS", d);
    MIVQ_REQUIRE(id_offset >= 0 && id_offset + n <= (int64_t)kNoId, MIVQ_ERR_INVALID, "flat_search: ids overflow");
    if (nq == 0) return MIVQ_OK;
    hipStream_t st = as_stream(stream);
    MIVQ_REQUIRE(dists && ids, MIVQ_ERR_INVALID, "flat_search: null pointer");
    if (n == 0) {
        const hipError_t e = launch_topk_merge(nullptr, nullptr, 0, nq, k, dists, ids, st);
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "flat_search(empty): %s", hipGetErrorString(e));
        return MIVQ_OK;
    }
    MIVQ_REQUIRE(q && x, MIVQ_ERR_INVALID, "flat_search: null pointer");
    const size_t need = mivq_flat_search_workspace_bytes(nq, n, d, k);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "flat_search: workspace %zu < %zu",
                 workspace_bytes, need);
    if (flat_use_tiled(nq, n)) {
        const hipError_t et = launch_flat_tiled(q, nq, x, n, d, metric, k, id_offset, workspace, dists, ids, st);
        if (et != hipSuccess) return set_error(MIVQ_ERR_HIP, "flat_search (tiled): %s", hipGetErrorString(et));
        return MIVQ_OK;
    }
    const int64_t nch = adc_chunks(nq, n, QB);
    const int parts = (int)(nch * kScanWaves);
    float* pd = static_cast<float*>(workspace);
    uint32_t* pi = reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) +
                                               align_up((size_t)parts * nq * k * sizeof(float), 256));
    const int R = (k + 63) / 64;
    hipError_t e;
    switch (R) {
        case 1: e = launch_flat_r<1>(QB, q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st); break;
        case 2: e = launch_flat_r<2>(QB, q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st); break;
        case 3: e = launch_flat_r<3>(QB, q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st); break;
        default: e = launch_flat_r<4>(QB, q, nq, x, n, d, metric, k, id_offset, nch, pd, pi, st); break;
    }
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "flat_scan: %s", hipGetErrorString(e));
    e = launch_topk_merge(pd, pi, parts, nq, k, dists, ids, st);
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "topk_merge: %s", hipGetErrorString(e));
    return MIVQ_OK;
}

extern "C" int mivq_adc_lut(const float* q, int64_t nq, int32_t d, int32_t M, int32_t nbits,
                            const float* centroids, int32_t metric, float* lut, void* stream) {
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "adc_lut: metric %d", metric);
    MIVQ_REQUIRE(nq >= 0 && M > 0 && d > 0 && d % M == 0, MIVQ_ERR_INVALID, "adc_lut: bad sizes");
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "adc_lut: nbits=%d", nbits);
    if (nq == 0) return MIVQ_OK;
    MIVQ_REQUIRE(q && centroids && lut, MIVQ_ERR_INVALID, "adc_lut: null pointer");
    const int ksub = 1 << nbits;
#ifndef MIVQ_LUT_PK
#define MIVQ_LUT_PK 1
#endif
    if (MIVQ_LUT_PK && ksub == 256 && (d / M) % 4 == 0 && reinterpret_cast<uintptr_t>(centroids) % 16 == 0) {
        const dim3 grid((unsigned)M, (unsigned)ceil_div(nq, kLutPkQ));
        const int ds = d / M;
        // compile-time dsub for the benchmarked shapes (round 6, profiles/r06_s36; bit-exact tests, r06_s37):
        // 1000 queries, dsub 96 35.5 -> 34 us, 10,000 queries dsub 64 224 -> 197 us, dsub 48
        // 33.5 -> 26.5 us
        const int dsk = ds == 48 || ds == 64 || ds == 96 ? ds : 0;
#define MIVQ_LUT_GO(L2V, DSV)                                                                                  \
    hipLaunchKernelGGL((adc_lut_pk_kernel<L2V, DSV>), grid, dim3(128), 0, as_stream(stream), q, nq, d, M, ds, \
                       centroids, lut)
        const bool l2 = metric == MIVQ_METRIC_L2;
        switch (dsk) {
            case 48: if (l2) MIVQ_LUT_GO(true, 48); else MIVQ_LUT_GO(false, 48); break;
            case 64: if (l2) MIVQ_LUT_GO(true, 64); else MIVQ_LUT_GO(false, 64); break;
            case 96: if (l2) MIVQ_LUT_GO(true, 96); else MIVQ_LUT_GO(false, 96); break;
            default: if (l2) MIVQ_LUT_GO(true, 0); else MIVQ_LUT_GO(false, 0); break;
        }
#undef MIVQ_LUT_GO
        return check_launch("adc_lut");
    }
    const size_t smem = (size_t)kLutQ * (d / M) * sizeof(float);
    MIVQ_REQUIRE(smem <= 64 * 1024, MIVQ_ERR_UNSUPPORTED, "adc_lut: dsub=%d too large", d / M);
    hipLaunchKernelGGL(adc_lut_kernel, dim3((unsigned)M, (unsigned)ceil_div(nq, kLutQ)), dim3(256), smem,
                       as_stream(stream), q, nq, d, M, ksub, d / M, centroids, metric,
                       (d / M) % 4 == 0 && reinterpret_cast<uintptr_t>(centroids) % 16 == 0 ? 1 : 0, lut);
    return check_launch("adc_lut");
}

extern "C" size_t mivq_adc_search_workspace_bytes(int64_t nq, int64_t n, int32_t M, int32_t nbits, int32_t k) {
    if (nq <= 0 || n <= 0 || M <= 0 || k <= 0 || nbits < 1 || nbits > 8) return 0;
    const int QB = adc_qb(M, 1 << nbits);
    if (QB == 0) return 0;
    int64_t parts = adc_chunks(nq, n, QB) * kScanWaves;
    if (adc_filtered_shape(M, 1 << nbits, k)) parts = std::max<int64_t>(parts, adc_fallback_chunks(nq, n, k) * kScanWaves);
    // the fp32 scan's part lists (every query, or the filtered path's uncertified ones) ...
    const size_t exact = align_up((size_t)parts * nq * k * sizeof(float), 256) + align_up((size_t)parts * nq * k * 4, 256);
    // ... then the filtered path's regions
    if (!adc_filtered_shape(M, 1 << nbits, k)) return exact;
    return adc_filtered_layout(nq, n, M, k, exact).total;
}

extern "C" int mivq_adc_search(const float* lut, int64_t nq, const uint8_t* codes, int64_t n, int32_t M,
                               int32_t nbits, int32_t k, int64_t id_offset, void* workspace,
                               size_t workspace_bytes, float* dists, uint32_t* ids, uint32_t flags, void* stream) {
    MIVQ_REQUIRE(nq >= 0 && n >= 0 && M > 0 && k > 0, MIVQ_ERR_INVALID,
                 "adc_search: bad sizes nq=%lld n=%lld M=%d k=%d", (long long)nq, (long long)n, M, k);
    MIVQ_REQUIRE((flags & ~(MIVQ_ADC_FORCE_EXACT | MIVQ_ADC_NO_RERUN | MIVQ_ADC_SMALL_RERUN_GRID)) == 0,
                 MIVQ_ERR_INVALID, "adc_search: unknown flags 0x%x", flags);
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "adc_search: nbits=%d", nbits);
    MIVQ_REQUIRE(k <= 256, MIVQ_ERR_UNSUPPORTED, "adc_search: k=%d > 256", k);
    const int ksub = 1 << nbits;
    const int QB = adc_qb(M, ksub);
    MIVQ_REQUIRE(QB > 0, MIVQ_ERR_UNSUPPORTED, "adc_search: M*ksub=%d tables do not fit LDS", M * ksub);
    MIVQ_REQUIRE(id_offset >= 0 && id_offset + n <= (int64_t)kNoId, MIVQ_ERR_INVALID,
                 "adc_search: global ids must fit uint32");
    if (nq == 0) return MIVQ_OK;
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        // nothing to rank: every slot is the sentinel
        MIVQ_REQUIRE(dists && ids, MIVQ_ERR_INVALID, "adc_search: null pointer");
        const hipError_t e = launch_topk_merge(nullptr, nullptr, 0, nq, k, dists, ids, st);
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "adc_search(empty): %s", hipGetErrorString(e));
        return MIVQ_OK;
    }
    MIVQ_REQUIRE(lut && codes && dists && ids, MIVQ_ERR_INVALID, "adc_search: null pointer");
    const size_t need = mivq_adc_search_workspace_bytes(nq, n, M, nbits, k);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "adc_search: workspace %zu < %zu",
                 workspace_bytes, need);
    const bool fshape = adc_filtered_shape(M, ksub, k);
    const int64_t nch_exact = adc_chunks(nq, n, QB), nch_fb = adc_fallback_chunks(nq, n, k);
    const int64_t parts_ws = std::max<int64_t>(nch_exact, fshape ? nch_fb : 0) * kScanWaves;
    float* pd = static_cast<float*>(workspace);
    const size_t exact_bytes = align_up((size_t)parts_ws * nq * k * sizeof(float), 256) +
                               align_up((size_t)parts_ws * nq * k * 4, 256);
    uint32_t* pi = reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) +
                                               align_up((size_t)parts_ws * nq * k * sizeof(float), 256));
    // the filtered path (integer-LUT scan + exact re-rank + certificate; the fp32 scan re-runs
    // only the uncertified queries): same results, ~half the LDS traffic per (query, row)
    const bool filtered = fshape && reinterpret_cast<uintptr_t>(codes) % 16 == 0 &&
                          reinterpret_cast<uintptr_t>(lut) % 16 == 0 && !(flags & MIVQ_ADC_FORCE_EXACT);
    const int* qlist = nullptr;
    const int* qcount = nullptr;
    hipError_t e;
    const bool no_fallback = (flags & MIVQ_ADC_NO_RERUN) != 0;  // test hook: certified queries only, the others NaN
    if (filtered) {
        const AdcFilteredLayout FL = adc_filtered_layout(nq, n, M, k, exact_bytes);
        unsigned char* ws = static_cast<unsigned char*>(workspace);
        if (no_fallback) {
            e = hipMemsetAsync(dists, 0xFF, (size_t)nq * k * sizeof(float), st);
            if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "adc_search: %s", hipGetErrorString(e));
        }
        e = launch_filtered(M, lut, nq, codes, n, k, id_offset, ws, FL, dists, ids, st);
        if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "adc_search (filtered): %s", hipGetErrorString(e));
        qcount = reinterpret_cast<const int*>(ws + FL.fail);
        qlist = qcount + 1;
        if (no_fallback) return MIVQ_OK;
    }
    const int64_t nch = filtered ? nch_fb : nch_exact;
    const int parts = (int)(nch * kScanWaves);
    const bool sg = filtered && (flags & MIVQ_ADC_SMALL_RERUN_GRID) != 0;
    const int R = (k + 63) / 64;
    switch (R) {
        case 1: e = launch_scan_r<1>(QB, lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg); break;
        case 2: e = launch_scan_r<2>(QB, lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg); break;
        case 3: e = launch_scan_r<3>(QB, lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg); break;
        default: e = launch_scan_r<4>(QB, lut, nq, codes, n, M, ksub, k, id_offset, nch, pd, pi, st, qlist, qcount, sg); break;
    }
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "adc_scan: %s", hipGetErrorString(e));
    e = launch_topk_merge(pd, pi, parts, nq, k, dists, ids, st, qlist, qcount);
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "topk_merge: %s", hipGetErrorString(e));
    return MIVQ_OK;
}

extern "C" int mivq_topk_merge(const float* dists_in, const uint32_t* ids_in, int32_t parts, int64_t nq, int32_t k,
                               float* dists_out, uint32_t* ids_out, void* stream) {
    MIVQ_REQUIRE(parts >= 0 && nq >= 0 && k > 0, MIVQ_ERR_INVALID, "topk_merge: bad sizes");
    if (nq == 0) return MIVQ_OK;
    MIVQ_REQUIRE((parts == 0 || (dists_in && ids_in)) && dists_out && ids_out, MIVQ_ERR_INVALID,
                 "topk_merge: null pointer");
    MIVQ_REQUIRE(k <= 256, MIVQ_ERR_UNSUPPORTED, "topk_merge: k=%d > 256", k);
    const hipError_t e = launch_topk_merge(dists_in, ids_in, parts, nq, k, dists_out, ids_out, as_stream(stream));
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "topk_merge: %s", hipGetErrorString(e));
    return MIVQ_OK;
}
