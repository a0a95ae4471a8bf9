// topk.h — the wave-resident exact top-k shared by the search kernels (adc.hip, ivf.hip).
// Elements are (dist, id) pairs ranked ascending by dist, then id; NaN is mapped to +inf by
// the callers, the sentinel is (+inf, kNoId).
#pragma once

#include "mivq_common.h"

#include <functional>

namespace mivq {

constexpr uint32_t kNoId = 0xFFFFFFFFu;

__device__ __forceinline__ bool pair_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && ia < ib);
}

// Sorted list of k <= 64*R elements: element e in lane e%64, register e/64.
template <int R>
struct WaveTopK {
    float d[R];
    uint32_t id[R];

    __device__ void init() {
#pragma unroll
        for (int r = 0; r < R; ++r) { d[r] = INFINITY; id[r] = kNoId; }
    }
    // element k-1 (the current threshold); wave-uniform
    __device__ void kth(int k, float& kd, uint32_t& ki) const {
        const int r = (k - 1) >> 6, ln = (k - 1) & 63;
        float vd = d[0];
        uint32_t vi = id[0];
#pragma unroll
        for (int q = 1; q < R; ++q) if (q == r) { vd = d[q]; vi = id[q]; }
        kd = __shfl(vd, ln);
        ki = __shfl(vi, ln);
    }
    // insert (cd, ci) known to be < element k-1; wave-uniform call
    __device__ void insert(float cd, uint32_t ci, int k, int lane) {
        int p = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = r * 64 + lane;
            p += __popcll(__ballot(e < k && pair_less(d[r], id[r], cd, ci)));
        }
        float nd[R];
        uint32_t ni[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // element e-1: lane-1 of the same register, or lane 63 of register r-1
            float pd = __shfl_up(d[r], 1);
            uint32_t pi = __shfl_up(id[r], 1);
            float td = INFINITY;
            uint32_t ti = kNoId;
            if (r > 0) {  // compile-time r: wave-uniform shuffle
                td = __shfl(d[r > 0 ? r - 1 : 0], 63);
                ti = __shfl(id[r > 0 ? r - 1 : 0], 63);
            }
            if (lane == 0) { pd = td; pi = ti; }
            const int e = r * 64 + lane;
            nd[r] = e > p ? pd : (e == p ? cd : d[r]);
            ni[r] = e > p ? pi : (e == p ? ci : id[r]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) { d[r] = nd[r]; id[r] = ni[r]; }
    }
    // offer one candidate per lane (valid lanes only); wave-uniform call
    __device__ void offer(bool valid, float dv, uint32_t gid, int k, int lane, float& thr_d, uint32_t& thr_i) {
        unsigned long long mask = __ballot(valid && pair_less(dv, gid, thr_d, thr_i));
        while (mask) {
            const int src = __builtin_ctzll(mask);
            mask &= mask - 1;
            const float cd = __shfl(dv, src);
            const uint32_t ci = __shfl(gid, src);
            if (!pair_less(cd, ci, thr_d, thr_i)) continue;
            insert(cd, ci, k, lane);
            kth(k, thr_d, thr_i);
        }
    }
};

// Merges per-part sorted lists laid out (parts, nq, k) into (nq, k); parts == 0 writes the
// sentinel everywhere.  Defined in adc.hip.
hipError_t launch_topk_merge(const float* pd, const uint32_t* pi, int parts, int64_t nq, int k, float* od,
                             uint32_t* oi, hipStream_t st, const int* qlist = nullptr, const int* qcount = nullptr);

// Tiled top-k (ivf.hip): a key-block producer + segmented top-k + running merge.  The
// workspace of flat_tiled_workspace_bytes serves both launchers.
using TileFn = std::function<hipError_t(int64_t c0, int64_t m, float* buf)>;
hipError_t launch_tiled_topk(int64_t nq, int64_t n, int k, int64_t id_offset, void* ws, float* dists,
                             uint32_t* ids, hipStream_t st, const TileFn& tile);
// Columns per key block of launch_tiled_topk (a multiple of its 4096-column segment; the key
// block is nq x that many floats at the start of its workspace).
int64_t tiled_topk_cols(int64_t nq, int64_t n);
// Tiled exact brute force (ivf.hip): pairwise chains + segmented top-k + running merge.
size_t flat_tiled_workspace_bytes(int64_t nq, int64_t n, int k);
hipError_t launch_flat_tiled(const float* q, int64_t nq, const float* x, int64_t n, int d, int metric, int k,
                             int64_t id_offset, void* ws, float* dists, uint32_t* ids, hipStream_t st);

}  // namespace mivq
