// ivf.hip — coarse quantizer, inverted lists and IVF-PQ search on gfx950.
//
// GPU counterpart of FaissIvfPqIndex (/root/reference/src/haag_vq/methods/search/
// faiss_ivfpq_index.py:46-76: faiss IndexIVFPQ over an IndexFlatL2 / IndexFlatIP coarse
// quantizer, residual PQ) and of the IVF build timed in benchmarks/ivf_benchmark.py:170-204.
//
//   pairwise_kernel        exact coarse distances (the quantizer's exhaustive search and the
//                          k-means assignment): 128 x 64 (row, centroid) tile per 256-thread
//                          workgroup, 8 x 4 per thread as 16 v_pk chains, k-slices of 16
//                          staged transposed in LDS (double-buffered, prefetched into
//                          registers one slice ahead).  Every (row, centroid) value is one
//                          sequential fmaf chain over t, the same as mivq_flat_search.
//   topk_rows_kernel       per-row (value, column) top-k (wave per row; k = 1 is a plain
//                          lane-strided argmin plus one wave reduction).
//   bucket_*               stable counting sort of list assignments (per-block histograms,
//                          column prefix, block-local ranks by wave match loops), giving
//                          list offsets and the row order inside every list.
//   centroid_update        k-means update from the sort: ascending-row sums per list.
//   ivfpq_terms_kernel     per-vector L2 term tau_i (faiss' precomputed table folded per
//                          code, so a search needs only the query's own M x ksub LUT).
//   ivfpq_scan_kernel      one workgroup per (query, probe slice); 16 waves share the
//                          query's LUT in LDS and scan whole lists, 64 codes per step, into
//                          wave-resident top-k lists that topk_merge_kernel merges.
#include "mivq_common.h"
#include "topk.h"

namespace mivq {
namespace {

typedef float float2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int PBM = 128, PBN = 64, PBK = 16, PPAD = 4;

// out[i][j] = L2: fmaf chain over t of (x_i[t] - y_j[t])^2;  IP: -(fmaf chain of x_i[t] y_j[t])
template <bool IP, bool VEC>
__global__ __launch_bounds__(256) void pairwise_kernel(const float* __restrict__ x, int64_t n,
                                                       const float* __restrict__ y, int64_t m, int d,
                                                       float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float xs[2][PBK][PBM + PPAD];
    __shared__ __attribute__((aligned(16))) float ys[2][PBK][PBN + PPAD];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int64_t r0 = (int64_t)blockIdx.x * PBM;
    const int64_t c0 = (int64_t)blockIdx.y * PBN;

    // global -> register slice loads: x slice = 128 rows x 16 t (2 float4 per thread),
    // y slice = 64 rows x 16 t (1 float4 per thread); out-of-range values are 0, which
    // leaves every chain unchanged (fmaf(0, 0, a) == a)
    f32x4 px[2], py;
    auto fetch = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int f = tid + 256 * u, row = f >> 2, q4 = f & 3;
            const int64_t gr = r0 + row;
            const int t = k0 + 4 * q4;
            if (VEC) {
                px[u] = (gr < n && t < d) ? *reinterpret_cast<const f32x4*>(x + gr * d + t) : (f32x4){0.f, 0.f, 0.f, 0.f};
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) px[u][j] = (gr < n && t + j < d) ? x[gr * d + t + j] : 0.0f;
            }
        }
        {
            const int row = tid >> 2, q4 = tid & 3;
            const int64_t gc = c0 + row;
            const int t = k0 + 4 * q4;
            if (VEC) {
                py = (gc < m && t < d) ? *reinterpret_cast<const f32x4*>(y + gc * d + t) : (f32x4){0.f, 0.f, 0.f, 0.f};
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) py[j] = (gc < m && t + j < d) ? y[gc * d + t + j] : 0.0f;
            }
        }
    };
    auto stash = [&](int b) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int f = tid + 256 * u, row = f >> 2, q4 = f & 3;
#pragma unroll
            for (int j = 0; j < 4; ++j) xs[b][4 * q4 + j][row] = px[u][j];
        }
        const int row = tid >> 2, q4 = tid & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) ys[b][4 * q4 + j][row] = py[j];
    };

    // scalar fp32 chains: packed fp32 math must not consume LDS-loaded registers (DESIGN.md §8,
    // tools/isa_audit.py)
    float acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0.0f;

    fetch(0);
    stash(0);
    __syncthreads();
    int b = 0;
    for (int k0 = 0; k0 < d; k0 += PBK) {
        const bool more = k0 + PBK < d;
        if (more) fetch(k0 + PBK);
#pragma unroll
        for (int t = 0; t < PBK; ++t) {
            const f32x4 xa = *reinterpret_cast<const f32x4*>(&xs[b][t][ty * 8]);
            const f32x4 xb = *reinterpret_cast<const f32x4*>(&xs[b][t][ty * 8 + 4]);
            const f32x4 yv = *reinterpret_cast<const f32x4*>(&ys[b][t][tx * 4]);
            const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
            const float yy[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
            for (int i = 0; i < 8; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (IP) {
                        acc[i][j] = __builtin_fmaf(xv[i], yy[j], acc[i][j]);
                    } else {
                        const float df = __fsub_rn(xv[i], yy[j]);
                        acc[i][j] = __builtin_fmaf(df, df, acc[i][j]);
                    }
                }
            }
        }
        if (more) {
            stash(b ^ 1);
            __syncthreads();
            b ^= 1;
        }
    }
    const int64_t gc = c0 + tx * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t gr = r0 + ty * 8 + i;
        if (gr >= n) continue;
        f32x4 v = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
        if (IP) v = -v;
        float* o = out + gr * m + gc;
        if ((m & 3) == 0 && gc + 3 < m) {
            *reinterpret_cast<f32x4*>(o) = v;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (gc + j < m) o[j] = v[j];
        }
    }
}

// Per row: the k smallest (value, column) pairs.  Wave per row, 4 rows per block.
template <int R>
__global__ __launch_bounds__(256) void topk_rows_kernel(const float* __restrict__ dist, int64_t n, int64_t m, int k,
                                                        float* __restrict__ od, uint32_t* __restrict__ oi) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;  // whole wave
    const float* dr = dist + row * m;
    if (R == 0) {  // k == 1: lane-strided argmin, then the wave minimum
        float bd = INFINITY;
        uint32_t bi = kNoId;
        for (int64_t j = lane; j < m; j += 64) {
            float v = dr[j];
            if (v != v) v = INFINITY;
            if (pair_less(v, (uint32_t)j, bd, bi)) { bd = v; bi = (uint32_t)j; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float vd = __shfl_xor(bd, o);
            const uint32_t vi = __shfl_xor(bi, o);
            if (pair_less(vd, vi, bd, bi)) { bd = vd; bi = vi; }
        }
        if (lane == 0) { od[row] = bd; oi[row] = bi; }
        return;
    }
    constexpr int RR = R > 0 ? R : 1;
    WaveTopK<RR> top;
    top.init();
    float thr_d = INFINITY;
    uint32_t thr_i = kNoId;
    for (int64_t j0 = 0; j0 < m; j0 += 64) {
        const int64_t j = j0 + lane;
        const bool valid = j < m;
        float v = valid ? dr[j] : INFINITY;
        if (v != v) v = INFINITY;
        top.offer(valid, v, (uint32_t)j, k, lane, thr_d, thr_i);
    }
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const int e = r * 64 + lane;
        if (e < k) { od[row * k + e] = top.d[r]; oi[row * k + e] = top.id[r]; }
    }
}

// ---------------------------------------------------------------- stable bucket sort
constexpr int kBucketRows = 1024;  // rows per sort block (histogram and scatter agree)

__global__ __launch_bounds__(256) void bucket_hist_kernel(const uint32_t* __restrict__ a, int64_t n, int K,
                                                          uint32_t* __restrict__ cnt) {
    extern __shared__ uint32_t h[];
    for (int l = threadIdx.x; l < K; l += 256) h[l] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * kBucketRows;
    for (int r = threadIdx.x; r < kBucketRows; r += 256) {
        const int64_t row = b0 + r;
        if (row < n) atomicAdd(&h[a[row]], 1u);
    }
    __syncthreads();
    uint32_t* dst = cnt + (int64_t)blockIdx.x * K;
    for (int l = threadIdx.x; l < K; l += 256) dst[l] = h[l];
}

// cnt[b][l] -> exclusive prefix over blocks b; tot[l] = bucket size
__global__ __launch_bounds__(256) void bucket_colscan_kernel(uint32_t* __restrict__ cnt, int64_t nb, int K,
                                                             int64_t* __restrict__ tot) {
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l >= K) return;
    int64_t run = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const uint32_t c = cnt[b * K + l];
        cnt[b * K + l] = (uint32_t)run;
        run += c;
    }
    tot[l] = run;
}

// offsets[l] = sum of tot[< l], offsets[K] = n (one block)
__global__ __launch_bounds__(1024) void bucket_offsets_kernel(const int64_t* __restrict__ tot, int K,
                                                              int64_t* __restrict__ offsets) {
    __shared__ int64_t part[1024];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < K; base += 1024) {
        const int l = base + threadIdx.x;
        const int64_t v = l < K ? tot[l] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
            const int64_t add = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (l < K) offsets[l] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) offsets[K] = carry;
}

// One wave per sort block: rows in ascending order get consecutive slots of their bucket.
__global__ __launch_bounds__(64) void bucket_scatter_kernel(const uint32_t* __restrict__ a, int64_t n, int K,
                                                            const uint32_t* __restrict__ cnt,
                                                            const int64_t* __restrict__ offsets,
                                                            uint32_t* __restrict__ order) {
    extern __shared__ int64_t pos[];  // next slot per bucket for this block
    const int lane = threadIdx.x;
    const uint32_t* cb = cnt + (int64_t)blockIdx.x * K;
    for (int l = lane; l < K; l += 64) pos[l] = offsets[l] + cb[l];
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * kBucketRows;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int r0 = 0; r0 < kBucketRows; r0 += 64) {
        const int64_t row = b0 + r0 + lane;
        const bool valid = row < n;
        const uint32_t mine = valid ? a[row] : 0u;
        bool pending = valid;
        for (;;) {  // one iteration per distinct bucket among the pending lanes
            const unsigned long long act = __ballot(pending);
            if (!act) break;
            const uint32_t lead = __shfl(mine, __builtin_ctzll(act));
            const unsigned long long same = __ballot(pending && mine == lead);
            const int64_t p0 = pos[lead];
            if (pending && mine == lead) {
                order[p0 + __popcll(same & below)] = (uint32_t)row;
                pending = false;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) pos[lead] = p0 + __popcll(same);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// centroids[l][t] = (sum over the bucket's rows, ascending, of x[row][t]) / count
__global__ __launch_bounds__(256) void centroid_update_kernel(const float* __restrict__ x, int d,
                                                              const int64_t* __restrict__ offsets,
                                                              const uint32_t* __restrict__ order,
                                                              float* __restrict__ centroids,
                                                              int32_t* __restrict__ counts) {
    __shared__ uint32_t rows[256];
    const int l = blockIdx.x;
    const int64_t beg = offsets[l], end = offsets[l + 1];
    constexpr int TPT = 8;  // dims per thread per pass
    for (int t0 = 0; t0 < d; t0 += 256 * TPT) {
        float s[TPT];
#pragma unroll
        for (int u = 0; u < TPT; ++u) s[u] = 0.0f;
        for (int64_t c = beg; c < end; c += 256) {
            const int nc = (int)min<int64_t>(256, end - c);
            __syncthreads();
            if (threadIdx.x < nc) rows[threadIdx.x] = order[c + threadIdx.x];
            __syncthreads();
            for (int q = 0; q < nc; ++q) {
                const float* xr = x + (int64_t)rows[q] * d;
#pragma unroll
                for (int u = 0; u < TPT; ++u) {
                    const int t = t0 + u * 256 + threadIdx.x;
                    if (t < d) s[u] = __fadd_rn(s[u], xr[t]);
                }
            }
        }
        const int64_t cntl = end - beg;
        if (cntl > 0) {
#pragma unroll
            for (int u = 0; u < TPT; ++u) {
                const int t = t0 + u * 256 + threadIdx.x;
                if (t < d) centroids[(int64_t)l * d + t] = __fdiv_rn(s[u], (float)cntl);
            }
        }
    }
    if (threadIdx.x == 0) counts[l] = (int32_t)(end - beg);
}

__global__ __launch_bounds__(256) void residual_kernel(const float* __restrict__ x, int64_t n, int d,
                                                       const float* __restrict__ c, const uint32_t* __restrict__ a,
                                                       float* __restrict__ r) {
    const int64_t total = n * (int64_t)d;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t row = e / d;
        const int t = (int)(e - row * d);
        r[e] = __fsub_rn(x[e], c[(int64_t)a[row] * d + t]);
    }
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const uint32_t* __restrict__ src, int64_t words,
                                                          const uint32_t* __restrict__ order, int64_t n,
                                                          uint32_t* __restrict__ dst) {
    const int64_t total = n * words;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t i = e / words, w = e - i * words;
        dst[e] = src[(int64_t)order[i] * words + w];
    }
}

// tau_i = sum over m ascending of (cn[m][k] + 2 * (fmaf chain over t of cc[t] * C[m][k][t]))
__global__ __launch_bounds__(256) void ivfpq_terms_kernel(const uint8_t* __restrict__ codes, int64_t n, int d, int M,
                                                          int ksub, const float* __restrict__ C,
                                                          const float* __restrict__ cn,
                                                          const float* __restrict__ coarse,
                                                          const uint32_t* __restrict__ a, float* __restrict__ tau) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int dsub = d / M;
    const float* cc = coarse + (int64_t)a[i] * d;
    float acc = 0.0f;
    for (int m = 0; m < M; ++m) {
        const int k = codes[i * M + m];
        const float* cm = C + ((int64_t)m * ksub + k) * dsub;
        const float* cs = cc + m * dsub;
        float p = 0.0f;
        for (int t = 0; t < dsub; ++t) p = __builtin_fmaf(cs[t], cm[t], p);
        acc = __fadd_rn(acc, __fadd_rn(cn[m * ksub + k], __fmul_rn(2.0f, p)));
    }
    tau[i] = acc;
}

constexpr int kIvfWaves = 16;

// grid (nsplit, nq); workgroup: query q, probes [s*pps, (s+1)*pps); wave w takes every 16th.
template <int R, bool L2>
__global__ __launch_bounds__(kIvfWaves * 64) void ivfpq_scan_kernel(
    const float* __restrict__ lut, int M, int ksub, const float* __restrict__ probe_d,
    const uint32_t* __restrict__ probe_l, int nprobe, int pps, const int64_t* __restrict__ offsets,
    const uint8_t* __restrict__ codes, const uint32_t* __restrict__ ids, const float* __restrict__ tau, int k,
    int64_t nq, float* __restrict__ part_d, uint32_t* __restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float tab[];  // [M][ksub]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t q = blockIdx.y;
    const int tabn = M * ksub;
    for (int e = tid; e < tabn; e += kIvfWaves * 64) tab[e] = lut[q * tabn + e];
    __syncthreads();
    WaveTopK<R> top;
    top.init();
    float thr_d = INFINITY;
    uint32_t thr_i = kNoId;
    const int p0 = blockIdx.x * pps, p1 = min(nprobe, p0 + pps);
    const bool words = (M & 3) == 0;
    for (int p = p0 + wv; p < p1; p += kIvfWaves) {
        const uint32_t l = probe_l[q * nprobe + p];
        if (l == kNoId) continue;  // wave-uniform
        const float base = probe_d[q * nprobe + p];
        const int64_t beg = offsets[l], end = offsets[l + 1];
        for (int64_t r0 = beg; r0 < end; r0 += 64) {
            const int64_t row = r0 + lane;
            const bool valid = row < end;
            float dv = INFINITY;
            uint32_t gid = kNoId;
            if (valid) {
                const uint8_t* cr = codes + row * M;
                float s = 0.0f;
                if (words) {
                    for (int m0 = 0; m0 < M; m0 += 4) {
                        const uint32_t w = *reinterpret_cast<const uint32_t*>(cr + m0);
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) s = __fadd_rn(s, tab[(m0 + bb) * ksub + ((w >> (8 * bb)) & 0xFFu)]);
                    }
                } else {
                    for (int m = 0; m < M; ++m) s = __fadd_rn(s, tab[m * ksub + cr[m]]);
                }
                dv = L2 ? __fadd_rn(__fadd_rn(base, tau[row]), __fmul_rn(2.0f, s)) : __fadd_rn(base, s);
                if (dv != dv) dv = INFINITY;
                gid = ids[row];
            }
            top.offer(valid, dv, gid, k, lane, thr_d, thr_i);
        }
    }
    const int64_t part = (int64_t)blockIdx.x * kIvfWaves + wv;
    float* od = part_d + (part * nq + q) * k;
    uint32_t* oi = part_i + (part * nq + q) * k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < k) { od[e] = top.d[r]; oi[e] = top.id[r]; }
    }
}

// Segmented row top-k for the tiled exact search: the (rows, S*L) block is read as rows*S
// segments of L columns; segment (row, s) writes its k best (value, base + s*L + col) to part
// part0 + s of the (parts, rows, k) list layout that topk_merge_kernel consumes.
template <int R>
__global__ __launch_bounds__(256) void topk_seg_kernel(const float* __restrict__ dist, int64_t rows, int64_t ld,
                                                       int64_t ncols, int L, int S, int k, int64_t base,
                                                       int part0, float* __restrict__ part_d,
                                                       uint32_t* __restrict__ part_i) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= rows * S) return;
    const int64_t row = g / S;
    const int s = (int)(g - row * S);
    const int64_t c0 = (int64_t)s * L;
    const int64_t c1 = min<int64_t>(ncols, c0 + L);
    const float* dr = dist + row * ld;
    WaveTopK<R> top;
    top.init();
    float thr_d = INFINITY;
    uint32_t thr_i = kNoId;
    // 256 columns per step, four coalesced dword loads per lane, the next step's in flight while
    // this one is screened; a step none of whose values beats the current k-th element costs one
    // ballot (round 6: the loop was one dependent 4-B load per 64 columns).  The list is exact
    // in (dist, id), so the order the candidates are offered in does not change it.
    float v[4], vn[4];
    auto ldv = [&](int64_t j0, float (&dst)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t j = j0 + 64 * t + lane;
            dst[t] = j < c1 ? dr[j] : INFINITY;
        }
    };
    ldv(c0, v);
    for (int64_t j0 = c0; j0 < c1; j0 += 256) {
        ldv(j0 + 256, vn);
        bool any = false;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t j = j0 + 64 * t + lane;
            if (v[t] != v[t]) v[t] = INFINITY;
            any = any || (j < c1 && pair_less(v[t], (uint32_t)(base + j), thr_d, thr_i));
        }
        if (__ballot(any) != 0ull) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int64_t j = j0 + 64 * t + lane;
                top.offer(j < c1, v[t], (uint32_t)(base + j), k, lane, thr_d, thr_i);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = vn[t];
    }
    float* od = part_d + ((int64_t)(part0 + s) * rows + row) * k;
    uint32_t* oi = part_i + ((int64_t)(part0 + s) * rows + row) * k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < k) { od[e] = top.d[r]; oi[e] = top.id[r]; }
    }
}

// columns per segment (round 6: 16384 measured 3 % faster on the 1000 x 1M estimator search,
// 1024 30 % slower, profiles/r06_s6; 4096 kept: flat_tiled_cols never goes below one segment,
// so a longer segment would also raise the distance buffer's floor to nq x kSegL floats)
constexpr int kSegL = 4096;

int64_t flat_tiled_cols(int64_t nq, int64_t n) {
    int64_t bc = ((int64_t)1 << 26) / std::max<int64_t>(nq, 1);  // <= 256 MiB of distances per chunk
    bc = std::max<int64_t>(kSegL, bc / kSegL * kSegL);
    return std::min<int64_t>(bc, ceil_div(n, kSegL) * kSegL);
}

template <int R>
hipError_t launch_topk_seg(const float* dist, int64_t rows, int64_t ld, int64_t ncols, int S, int k, int64_t base,
                           int part0, float* pd, uint32_t* pi, hipStream_t st) {
    hipLaunchKernelGGL(topk_seg_kernel<R>, dim3((unsigned)ceil_div(rows * S, 4)), dim3(256), 0, st, dist, rows, ld,
                       ncols, kSegL, S, k, base, part0, pd, pi);
    return hipGetLastError();
}

}  // namespace

int64_t tiled_topk_cols(int64_t nq, int64_t n) { return flat_tiled_cols(nq, n); }

size_t flat_tiled_workspace_bytes(int64_t nq, int64_t n, int k) {
    const int64_t bc = flat_tiled_cols(nq, n);
    const int64_t S = bc / kSegL;
    return align_up((size_t)nq * bc * 4, 256) + 2 * align_up((size_t)(S + 1) * nq * k * 4, 256) +
           2 * align_up((size_t)nq * k * 4, 256);
}

// Top-k by tiles: `tile(c0, m, buf)` writes the (nq, m) key block of columns [c0, c0 + m)
// (row stride m) into buf; a segmented top-k and a running merge (part 0 = the result so
// far) follow each block.  Keys rank ascending, ties by the smaller id.
hipError_t launch_tiled_topk(int64_t nq, int64_t n, int k, int64_t id_offset, void* ws, float* dists,
                             uint32_t* ids, hipStream_t st, const TileFn& tile) {
    const int64_t bc = flat_tiled_cols(nq, n);
    const int S = (int)(bc / kSegL);
    unsigned char* p = static_cast<unsigned char*>(ws);
    float* buf = reinterpret_cast<float*>(p);
    p += align_up((size_t)nq * bc * 4, 256);
    float* pd = reinterpret_cast<float*>(p);
    p += align_up((size_t)(S + 1) * nq * k * 4, 256);
    uint32_t* pi = reinterpret_cast<uint32_t*>(p);
    p += align_up((size_t)(S + 1) * nq * k * 4, 256);
    float* rd = reinterpret_cast<float*>(p);
    p += align_up((size_t)nq * k * 4, 256);
    uint32_t* ri = reinterpret_cast<uint32_t*>(p);
    hipError_t e = hipSuccess;
    int nparts = 0;  // parts holding data in pd/pi (part 0 = running result once set)
    for (int64_t c0 = 0; c0 < n; c0 += bc) {
        const int64_t m = std::min<int64_t>(bc, n - c0);
        e = tile(c0, m, buf);
        if (e != hipSuccess) return e;
        const int Sc = (int)ceil_div(m, kSegL);
        const int part0 = nparts == 0 ? 0 : 1;
        switch ((k + 63) / 64) {
            case 1: e = launch_topk_seg<1>(buf, nq, m, m, Sc, k, id_offset + c0, part0, pd, pi, st); break;
            case 2: e = launch_topk_seg<2>(buf, nq, m, m, Sc, k, id_offset + c0, part0, pd, pi, st); break;
            case 3: e = launch_topk_seg<3>(buf, nq, m, m, Sc, k, id_offset + c0, part0, pd, pi, st); break;
            default: e = launch_topk_seg<4>(buf, nq, m, m, Sc, k, id_offset + c0, part0, pd, pi, st); break;
        }
        if (e != hipSuccess) return e;
        nparts = part0 + Sc;
        const bool last = c0 + bc >= n;
        e = launch_topk_merge(pd, pi, nparts, nq, k, last ? dists : rd, last ? ids : ri, st);
        if (e != hipSuccess) return e;
        if (!last) {  // the merged list becomes part 0
            e = hipMemcpyAsync(pd, rd, (size_t)nq * k * 4, hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipMemcpyAsync(pi, ri, (size_t)nq * k * 4, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
            nparts = 1;
        }
    }
    return e;
}

// Exact top-k by tiles: pairwise chains for a column chunk, then launch_tiled_topk's
// segmented top-k and running merge.  Same chains and (dist, id) order as flat_scan.
hipError_t launch_flat_tiled(const float* q, int64_t nq, const float* x, int64_t n, int d, int metric, int k,
                             int64_t id_offset, void* ws, float* dists, uint32_t* ids, hipStream_t st) {
    const bool vec = (d % 4) == 0 && ((uintptr_t)q % 16) == 0 && ((uintptr_t)x % 16) == 0;
    const bool ip = metric == MIVQ_METRIC_INNER_PRODUCT;
    return launch_tiled_topk(nq, n, k, id_offset, ws, dists, ids, st, [&](int64_t c0, int64_t m, float* buf) {
        const dim3 grid((unsigned)ceil_div(nq, PBM), (unsigned)ceil_div(m, PBN));
        const float* y = x + c0 * d;
        if (ip) {
            if (vec) hipLaunchKernelGGL((pairwise_kernel<true, true>), grid, dim3(256), 0, st, q, nq, y, m, d, buf);
            else hipLaunchKernelGGL((pairwise_kernel<true, false>), grid, dim3(256), 0, st, q, nq, y, m, d, buf);
        } else {
            if (vec) hipLaunchKernelGGL((pairwise_kernel<false, true>), grid, dim3(256), 0, st, q, nq, y, m, d, buf);
            else hipLaunchKernelGGL((pairwise_kernel<false, false>), grid, dim3(256), 0, st, q, nq, y, m, d, buf);
        }
        return hipGetLastError();
    });
}

namespace {

int ivf_splits(int64_t nq, int nprobe) {
    const int64_t want = ceil_div(512, std::max<int64_t>(nq, 1));
    const int64_t maxs = ceil_div(nprobe, kIvfWaves);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, maxs));
}

template <int R, bool L2>
hipError_t launch_ivf_scan(const float* lut, int64_t nq, int M, int ksub, const float* pdd, const uint32_t* pll,
                           int nprobe, const int64_t* offsets, const uint8_t* codes, const uint32_t* ids,
                           const float* tau, int k, float* pd, uint32_t* pi, hipStream_t st) {
    const int ns = ivf_splits(nq, nprobe);
    const int pps = (int)ceil_div(nprobe, ns);
    const size_t smem = (size_t)M * ksub * sizeof(float);
    auto kern = ivfpq_scan_kernel<R, L2>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)ns, (unsigned)nq), dim3(kIvfWaves * 64), smem, st, lut, M, ksub, pdd, pll,
                       nprobe, pps, offsets, codes, ids, tau, k, nq, pd, pi);
    return hipGetLastError();
}

template <int R>
hipError_t launch_ivf_scan_m(bool l2, const float* lut, int64_t nq, int M, int ksub, const float* pdd,
                             const uint32_t* pll, int nprobe, const int64_t* offsets, const uint8_t* codes,
                             const uint32_t* ids, const float* tau, int k, float* pd, uint32_t* pi, hipStream_t st) {
    return l2 ? launch_ivf_scan<R, true>(lut, nq, M, ksub, pdd, pll, nprobe, offsets, codes, ids, tau, k, pd, pi, st)
              : launch_ivf_scan<R, false>(lut, nq, M, ksub, pdd, pll, nprobe, offsets, codes, ids, tau, k, pd, pi, st);
}

unsigned grid_for(int64_t total) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 65536));
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" int mivq_pairwise_distances(const float* x, int64_t n, const float* y, int64_t m, int32_t d,
                                       int32_t metric, float* out, void* stream) {
    MIVQ_REQUIRE(n >= 0 && m >= 0 && d > 0, MIVQ_ERR_INVALID, "pairwise_distances: bad sizes");
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "pairwise_distances: metric %d", metric);
    MIVQ_REQUIRE(ceil_div(m, PBN) <= 65535, MIVQ_ERR_UNSUPPORTED, "pairwise_distances: m=%lld too large",
                 (long long)m);
    if (n == 0 || m == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && y && out, MIVQ_ERR_INVALID, "pairwise_distances: null pointer");
    const bool vec = (d % 4) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0;
    const dim3 grid((unsigned)ceil_div(n, PBM), (unsigned)ceil_div(m, PBN));
    hipStream_t st = as_stream(stream);
    const bool ip = metric == MIVQ_METRIC_INNER_PRODUCT;
    if (ip) {
        if (vec) hipLaunchKernelGGL((pairwise_kernel<true, true>), grid, dim3(256), 0, st, x, n, y, m, d, out);
        else hipLaunchKernelGGL((pairwise_kernel<true, false>), grid, dim3(256), 0, st, x, n, y, m, d, out);
    } else {
        if (vec) hipLaunchKernelGGL((pairwise_kernel<false, true>), grid, dim3(256), 0, st, x, n, y, m, d, out);
        else hipLaunchKernelGGL((pairwise_kernel<false, false>), grid, dim3(256), 0, st, x, n, y, m, d, out);
    }
    return check_launch("pairwise_distances");
}

extern "C" int mivq_topk_rows(const float* dist, int64_t n, int64_t m, int32_t k, float* out_d, uint32_t* out_i,
                              void* stream) {
    MIVQ_REQUIRE(n >= 0 && m >= 0 && k > 0, MIVQ_ERR_INVALID, "topk_rows: bad sizes");
    MIVQ_REQUIRE(k <= 256, MIVQ_ERR_UNSUPPORTED, "topk_rows: k=%d > 256", k);
    MIVQ_REQUIRE(m < (int64_t)kNoId, MIVQ_ERR_INVALID, "topk_rows: m too large");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE((dist || m == 0) && out_d && out_i, MIVQ_ERR_INVALID, "topk_rows: null pointer");
    const dim3 grid((unsigned)ceil_div(n, 4)), block(256);
    hipStream_t st = as_stream(stream);
    switch (k == 1 ? 0 : (k + 63) / 64) {
        case 0: hipLaunchKernelGGL(topk_rows_kernel<0>, grid, block, 0, st, dist, n, m, k, out_d, out_i); break;
        case 1: hipLaunchKernelGGL(topk_rows_kernel<1>, grid, block, 0, st, dist, n, m, k, out_d, out_i); break;
        case 2: hipLaunchKernelGGL(topk_rows_kernel<2>, grid, block, 0, st, dist, n, m, k, out_d, out_i); break;
        case 3: hipLaunchKernelGGL(topk_rows_kernel<3>, grid, block, 0, st, dist, n, m, k, out_d, out_i); break;
        default: hipLaunchKernelGGL(topk_rows_kernel<4>, grid, block, 0, st, dist, n, m, k, out_d, out_i); break;
    }
    return check_launch("topk_rows");
}

extern "C" size_t mivq_bucket_sort_workspace_bytes(int64_t n, int32_t K) {
    if (n < 0 || K <= 0) return 0;
    const int64_t nb = std::max<int64_t>(1, ceil_div(n, kBucketRows));
    return align_up((size_t)nb * K * sizeof(uint32_t), 256) + align_up((size_t)K * sizeof(int64_t), 256);
}

extern "C" int mivq_bucket_sort(const uint32_t* assign, int64_t n, int32_t K, int64_t* offsets, uint32_t* order,
                                void* workspace, size_t workspace_bytes, void* stream) {
    MIVQ_REQUIRE(n >= 0 && K > 0, MIVQ_ERR_INVALID, "bucket_sort: bad sizes");
    MIVQ_REQUIRE(K <= 16384, MIVQ_ERR_UNSUPPORTED, "bucket_sort: K=%d > 16384", K);
    MIVQ_REQUIRE(n < (int64_t)kNoId, MIVQ_ERR_INVALID, "bucket_sort: n too large for uint32 rows");
    MIVQ_REQUIRE(offsets, MIVQ_ERR_INVALID, "bucket_sort: null offsets");
    const size_t need = mivq_bucket_sort_workspace_bytes(n, K);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "bucket_sort: workspace %zu < %zu",
                 workspace_bytes, need);
    hipStream_t st = as_stream(stream);
    const int64_t nb = std::max<int64_t>(1, ceil_div(n, kBucketRows));
    uint32_t* cnt = static_cast<uint32_t*>(workspace);
    int64_t* tot = reinterpret_cast<int64_t*>(static_cast<unsigned char*>(workspace) +
                                              align_up((size_t)nb * K * sizeof(uint32_t), 256));
    if (n > 0) MIVQ_REQUIRE(assign && order, MIVQ_ERR_INVALID, "bucket_sort: null pointer");
    hipLaunchKernelGGL(bucket_hist_kernel, dim3((unsigned)nb), dim3(256), (size_t)K * 4, st, assign, n, K, cnt);
    hipLaunchKernelGGL(bucket_colscan_kernel, dim3((unsigned)ceil_div(K, 256)), dim3(256), 0, st, cnt, nb, K, tot);
    hipLaunchKernelGGL(bucket_offsets_kernel, dim3(1), dim3(1024), 0, st, tot, K, offsets);
    if (n > 0)
        hipLaunchKernelGGL(bucket_scatter_kernel, dim3((unsigned)nb), dim3(64), (size_t)K * 8, st, assign, n, K, cnt,
                           offsets, order);
    return check_launch("bucket_sort");
}

extern "C" int mivq_centroid_update(const float* x, int64_t n, int32_t d, int32_t K, const int64_t* offsets,
                                    const uint32_t* order, float* centroids, int32_t* counts, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0 && K > 0, MIVQ_ERR_INVALID, "centroid_update: bad sizes");
    MIVQ_REQUIRE(offsets && centroids && counts && (n == 0 || (x && order)), MIVQ_ERR_INVALID,
                 "centroid_update: null pointer");
    hipLaunchKernelGGL(centroid_update_kernel, dim3((unsigned)K), dim3(256), 0, as_stream(stream), x, d, offsets,
                       order, centroids, counts);
    return check_launch("centroid_update");
}

extern "C" int mivq_ivf_residuals(const float* x, int64_t n, int32_t d, const float* coarse, const uint32_t* assign,
                                  float* r, void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "ivf_residuals: bad sizes");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && coarse && assign && r, MIVQ_ERR_INVALID, "ivf_residuals: null pointer");
    hipLaunchKernelGGL(residual_kernel, dim3(grid_for(n * (int64_t)d)), dim3(256), 0, as_stream(stream), x, n, d,
                       coarse, assign, r);
    return check_launch("ivf_residuals");
}

extern "C" int mivq_gather_rows(const void* src, int64_t row_bytes, const uint32_t* order, int64_t n, void* dst,
                                void* stream) {
    MIVQ_REQUIRE(n >= 0 && row_bytes > 0 && row_bytes % 4 == 0, MIVQ_ERR_INVALID,
                 "gather_rows: row_bytes must be a positive multiple of 4");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(src && order && dst && src != dst, MIVQ_ERR_INVALID, "gather_rows: null or aliased pointer");
    const int64_t words = row_bytes / 4;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * words)), dim3(256), 0, as_stream(stream),
                       static_cast<const uint32_t*>(src), words, order, n, static_cast<uint32_t*>(dst));
    return check_launch("gather_rows");
}

extern "C" int mivq_ivfpq_terms(const uint8_t* codes, int64_t n, int32_t d, int32_t M, int32_t nbits,
                                const float* pq_centroids, const float* cn, const float* coarse,
                                const uint32_t* assign, float* tau, void* stream) {
    MIVQ_REQUIRE(n >= 0 && M > 0 && d > 0 && d % M == 0, MIVQ_ERR_INVALID, "ivfpq_terms: bad sizes");
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "ivfpq_terms: nbits=%d", nbits);
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(codes && pq_centroids && cn && coarse && assign && tau, MIVQ_ERR_INVALID,
                 "ivfpq_terms: null pointer");
    hipLaunchKernelGGL(ivfpq_terms_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), codes,
                       n, d, M, 1 << nbits, pq_centroids, cn, coarse, assign, tau);
    return check_launch("ivfpq_terms");
}

extern "C" size_t mivq_ivfpq_search_workspace_bytes(int64_t nq, int32_t nprobe, int32_t k) {
    if (nq <= 0 || nprobe <= 0 || k <= 0) return 0;
    const int64_t parts = (int64_t)ivf_splits(nq, nprobe) * kIvfWaves;
    return align_up((size_t)parts * nq * k * sizeof(float), 256) + align_up((size_t)parts * nq * k * 4, 256);
}

extern "C" int mivq_ivfpq_search(const float* lut, int64_t nq, int32_t M, int32_t nbits, const float* probe_d,
                                 const uint32_t* probe_l, int32_t nprobe, int32_t nlist, const int64_t* offsets,
                                 const uint8_t* list_codes, const uint32_t* list_ids, const float* tau,
                                 int32_t metric, int32_t k, void* workspace, size_t workspace_bytes, float* dists,
                                 uint32_t* ids, void* stream) {
    MIVQ_REQUIRE(nq >= 0 && M > 0 && nprobe > 0 && nlist > 0 && k > 0, MIVQ_ERR_INVALID, "ivfpq_search: bad sizes");
    MIVQ_REQUIRE(nbits >= 1 && nbits <= 8, MIVQ_ERR_UNSUPPORTED, "ivfpq_search: nbits=%d", nbits);
    MIVQ_REQUIRE(k <= 256, MIVQ_ERR_UNSUPPORTED, "ivfpq_search: k=%d > 256", k);
    MIVQ_REQUIRE(metric == MIVQ_METRIC_L2 || metric == MIVQ_METRIC_INNER_PRODUCT, MIVQ_ERR_UNSUPPORTED,
                 "ivfpq_search: metric %d", metric);
    const int ksub = 1 << nbits;
    MIVQ_REQUIRE((int64_t)M * ksub * 4 <= 128 * 1024, MIVQ_ERR_UNSUPPORTED, "ivfpq_search: M*ksub too large for LDS");
    if (nq == 0) return MIVQ_OK;
    const bool l2 = metric == MIVQ_METRIC_L2;
    MIVQ_REQUIRE(lut && probe_d && probe_l && offsets && list_codes && list_ids && dists && ids && (!l2 || tau),
                 MIVQ_ERR_INVALID, "ivfpq_search: null pointer");
    const size_t need = mivq_ivfpq_search_workspace_bytes(nq, nprobe, k);
    MIVQ_REQUIRE(workspace && workspace_bytes >= need, MIVQ_ERR_WORKSPACE, "ivfpq_search: workspace %zu < %zu",
                 workspace_bytes, need);
    hipStream_t st = as_stream(stream);
    const int parts = ivf_splits(nq, nprobe) * kIvfWaves;
    float* pd = static_cast<float*>(workspace);
    uint32_t* pi = reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) +
                                               align_up((size_t)parts * nq * k * sizeof(float), 256));
    hipError_t e;
    switch ((k + 63) / 64) {
        case 1: e = launch_ivf_scan_m<1>(l2, lut, nq, M, ksub, probe_d, probe_l, nprobe, offsets, list_codes, list_ids, tau, k, pd, pi, st); break;
        case 2: e = launch_ivf_scan_m<2>(l2, lut, nq, M, ksub, probe_d, probe_l, nprobe, offsets, list_codes, list_ids, tau, k, pd, pi, st); break;
        case 3: e = launch_ivf_scan_m<3>(l2, lut, nq, M, ksub, probe_d, probe_l, nprobe, offsets, list_codes, list_ids, tau, k, pd, pi, st); break;
        default: e = launch_ivf_scan_m<4>(l2, lut, nq, M, ksub, probe_d, probe_l, nprobe, offsets, list_codes, list_ids, tau, k, pd, pi, st); break;
    }
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "ivfpq_scan: %s", hipGetErrorString(e));
    e = launch_topk_merge(pd, pi, parts, nq, k, dists, ids, st);
    if (e != hipSuccess) return set_error(MIVQ_ERR_HIP, "ivfpq merge: %s", hipGetErrorString(e));
    return MIVQ_OK;
}
