// pq_encode_cs.hip — codebook-stationary fp16-MFMA PQ encode with exact re-check (gfx950).
//
// The hot kernel of ProductQuantizer.compress (/root/reference/src/haag_vq/methods/
// product_quantization.py:76-80 -> faiss ProductQuantizer::compute_codes).  Codes equal the
// canonical encode of include/mivq.h bit for bit; the filter window W is derived in pq.hip
// (pq_prep_mfma_kernel / the comment above pq_encode_mfma_kernel).
//
// Work decomposition.  Workgroup (chunk, m) owns subspace m for rows [r0, r1) of one chunk
// (blockIdx = chunk*M + m).  The number of chunks is chosen so that the grid is a whole
// number of rounds of workgroups over the CUs (one workgroup per CU: the LDS below).
//
// Launch 1, the filter (streaming).  LDS holds, for the workgroup's life,
//   cimg : the fp16 operand image of C_m in fragment order (8*KS KiB; ds_read_b128)
//   stg  : one fp16 x tile per wave, 32 rows x 16*KS halves, row pitch 32*KS+16 bytes
//   hb   : the scaled accumulator init -|c|^2 * sigma * tau / 2;  cnl : |c|^2
// 12 waves (3 per SIMD) each stream 32-row blocks ("vb").  x is read with buffer loads
// whose wave-instruction covers whole row segments (floor(64/(dsub/4)) rows, e.g. 2 rows =
// 768 bytes for dsub = 96; a lane-per-row fragment load touches 64 cache lines per
// instruction and streams at less than half the rate), scaled by sigma, converted to fp16
// and written to the wave's tile (tile rows past the range keep stale values: an MFMA
// column depends on its own row only); the MFMA B fragments are read back from it.  The next
// vb's loads are in flight while the current one is filtered: 8*KS v_mfma_f32_32x32x16_f16,
// a grouped top-2 / lane top-3 per lane, the partner-lane merge, then
//   1 candidate in the window -> the code is written;
//   2 candidates              -> the pair is held for one step while the 8-B load of its
//                                pair spreads is in flight; if the score gap exceeds the
//                                pair's own window, k1 is the code, else (row, k1, k2) goes
//                                to the workgroup's pair list;
//   >= 3 candidates, or a row the window cannot bound (fp16 overflow, NaN) -> full list.
// Launch 2, pq_resolve_merged_kernel: one workgroup per filter workgroup settles both lists
// with the canonical fp32 chains (fp32 codebook in LDS), re-running the filter for full
// items to list the centroids inside the window.  Launch 3 transposes the codes.
// Codes go to a transposed (M, n) scratch (32 contiguous bytes per vb); lists live in a
// workspace of n*M uint2 (workgroup (c, m) owns entries m*n + [r0, r1): pairs from the
// front, full items from the back).
// (Measured and dropped: a consumer wave inside the filter workgroup settling the items while
// the other 11 waves stream -- the filter lost 13 % and the consumer could not keep up.)
#include "pq_internal.h"

#include <math.h>

#include <type_traits>

namespace mivq {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 12;  // 768 threads, 3 waves per SIMD
constexpr int kGcListNc = 4;  // wide-subspace resolve: pieces of a centroid row in the list chains (dsub > 128)

// Wide subspaces (dsub 97..192, KS 7..12): the f16 image alone takes up to 96 KiB of LDS, so
// the filter runs 4 waves (one per SIMD, up to 512 registers) with two blocks in flight each.
constexpr int kWideWaves = 4;
constexpr int cs_waves(int KS) { return KS <= 6 ? kWaves : kWideWaves; }
constexpr int kRsrcWord3 = 0x00020000;  // gfx9 buffer resource: 32-bit data format
// x stream cache policy: nt (read once).  Rounds 4-5 measured the others.  The
// dsub-48 filter, whose odd subspaces share a 128-B line with their neighbour, reads with sc0
// instead: 8.12 -> 7.54 GB per PQ32 1M x 1536 launch (PMC FETCH_SIZE) and 1.753 -> 1.738 ms per
// call back to back, codes identical (profiles/r05_s35; policy 0: 7.56 GB, 1.742 ms).  For the
// other shapes sc0 is slower (r05_s36: dsub 96 1.35 -> 1.45 ms, dsub 64 -3 %, dsub 192 -11 %).
constexpr int kXAux = 2;
constexpr int kXAux48 = 1;
// Byte of (row, subspace m) in the (M, n) code scratch (transposed once at the end).  Round 5
// measured the codes stored in the (n, M) output directly (1-B stores 16 B apart, no transpose
// launch): no faster per call.
__device__ __forceinline__ int64_t code_at(int64_t row, int m, int64_t n, int M) {
    (void)M;
    return (int64_t)m * n + row;
}

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

// Two values at once: the largest of {t1, t2, a, b} is max3(t1, a, b) and the second is
// max(med3(t1, a, b), t2) (t2 <= t1 <= the top of {t1, a, b}): 3 ops for 2 values.
__device__ __forceinline__ void top2_insert2(float& t1, float& t2, float a, float b) {
    float n1, md, n2;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(n1) : "v"(t1), "v"(a), "v"(b));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(md) : "v"(t1), "v"(a), "v"(b));
    asm("v_max_f32 %0, %1, %2" : "=v"(n2) : "v"(md), "v"(t2));
    t1 = n1; t2 = n2;
}

// Merges a group's sorted (g1 >= g2) into the lane state (t1 >= t2 >= t3, t3 holding
// max(third, every group's second)): t1' = max(t1, g1), t2' = med3(t1, g1, max(t2, g2))
// (second of the union), t3' = max3(t3, min(t2, g1), g2) (third of the union, min(t1, g2) <=
// g2 folded into the g2 term).  5 ops.
__device__ __forceinline__ void merge_group(float& t1, float& t2, float& t3, float g1, float g2) {
    float a, b, n1, n2, n3;
    asm("v_max_f32 %0, %1, %2" : "=v"(a) : "v"(t2), "v"(g2));
    asm("v_min_f32 %0, %1, %2" : "=v"(b) : "v"(t2), "v"(g1));
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(n2) : "v"(t1), "v"(g1), "v"(a));
    asm("v_max_f32 %0, %1, %2" : "=v"(n1) : "v"(t1), "v"(g1));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(n3) : "v"(t3), "v"(b), "v"(g2));
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
    const half2v hv = __builtin_convertvector((float2v){a, b}, half2v);
    return __builtin_bit_cast(uint32_t, hv);
}

// s * (8 floats read from LDS) -> 8 halves, with SCALAR multiplies: a packed fp32 instruction
// must never consume a register written by an LDS read (beside another kernel's
// LDS DMA + MFMAs such results lose lanes 48..63; tools/isa_audit.py checks the built library)
__device__ __forceinline__ u32x4 cvt8_scaled(const f32x4 a0, const f32x4 a1, float s) {
    return (u32x4){cvt2(__fmul_rn(a0.x, s), __fmul_rn(a0.y, s)), cvt2(__fmul_rn(a0.z, s), __fmul_rn(a0.w, s)),
                   cvt2(__fmul_rn(a1.x, s), __fmul_rn(a1.y, s)), cvt2(__fmul_rn(a1.z, s), __fmul_rn(a1.w, s))};
}

__device__ __forceinline__ float dot2_self(uint32_t u, float acc) {
    const half2v hv = __builtin_bit_cast(half2v, u);
    return __builtin_amdgcn_fdot2(hv, hv, acc, false);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }

// Lanes 0..31 receive lane l + 32's value.  The filter's lane pair (l, l + 32) holds one row;
// only the h = 0 lanes use the merged result.  (v_permlane32_swap measured the same.)
__device__ __forceinline__ float upper_half(float v) { return __shfl_xor(v, 32); }

// 8 x reads (stride XS bytes) and the 4 reads of two centroid-pair rows (CS bytes apart),
// all issued back to back, then one lgkmcnt(0).
template <int G, int XS, int CS>
__device__ __forceinline__ void lds_burst(uint32_t xa, uint32_t ca, f32x4 (&xq)[G], f32x4& p0, f32x4& p1, f32x4& q0,
                                          f32x4& q1) {
    static_assert(G == 8, "burst shape");
    asm volatile(
        "ds_read_b128 %0, %12\n\t"
        "ds_read_b128 %1, %12 offset:%14\n\t"
        "ds_read_b128 %2, %12 offset:%15\n\t"
        "ds_read_b128 %3, %12 offset:%16\n\t"
        "ds_read_b128 %4, %12 offset:%17\n\t"
        "ds_read_b128 %5, %12 offset:%18\n\t"
        "ds_read_b128 %6, %12 offset:%19\n\t"
        "ds_read_b128 %7, %12 offset:%20\n\t"
        "ds_read_b128 %8, %13\n\t"
        "ds_read_b128 %9, %13 offset:16\n\t"
        "ds_read_b128 %10, %13 offset:%21\n\t"
        "ds_read_b128 %11, %13 offset:%22\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(xq[0]), "=v"(xq[1]), "=v"(xq[2]), "=v"(xq[3]), "=v"(xq[4]), "=v"(xq[5]), "=v"(xq[6]), "=v"(xq[7]),
          "=v"(p0), "=v"(p1), "=v"(q0), "=v"(q1)
        : "v"(xa), "v"(ca), "i"(XS), "i"(2 * XS), "i"(3 * XS), "i"(4 * XS), "i"(5 * XS), "i"(6 * XS), "i"(7 * XS),
          "i"(CS), "i"(CS + 16)
        : "memory");
}

// Workgroup -> (subspace m, row chunk).  Workgroups are dealt to the 8 XCDs round-robin; when
// the grid allows, each XCD gets all M subspaces of a chunk in consecutive slots, so the M
// workgroups reading one row range run side by side on one XCD and sweep the same DRAM pages
// together.  Both kernels of the encode use the same mapping (the lists are per workgroup).
__device__ __forceinline__ void wg_coords_of(unsigned b, unsigned g, int M, int& m, int64_t& chunk) {
    if (g % (8u * (unsigned)M) == 0) {
        const unsigned j = b >> 3;
        m = (int)(j % (unsigned)M);
        chunk = (int64_t)(j / (unsigned)M) * 8 + (b & 7u);
    } else {
        m = (int)(b % (unsigned)M);
        chunk = b / (unsigned)M;
    }
}

__device__ __forceinline__ void wg_coords(int M, int& m, int64_t& chunk) {
    wg_coords_of(blockIdx.x, gridDim.x, M, m, chunk);
}

// Load instructions per vb: ceil(32 / RPI), RPI = floor(64 / (dsub/4)) >= floor(16 / KS).
template <int KS>
constexpr int max_loads() {
    return (32 + (16 / KS) - 1) / (16 / KS);
}


// DS > 0: the kernel for sub-rows of exactly DS floats (the addresses and load counts fold
// to constants); DS = 0 reads dsub at run time.
// KH = 2 (wide subspaces with dsub == 16 KS, KS even): the wave's tile holds half of the
// block's K at a time (the image's K-steps 0..KS/2-1, then the rest), so the tile is half as
// wide and 8 waves fit next to the image; the B fragments of both halves stay in registers.
// Image K-step g gives lane half h the dims 8 KS h + 8 g + [0, 8), so tile half hh holds the
// dims hh 8 KT + [0, 8 KT) and 8 KS + hh 8 KT + [0, 8 KT) (KT = KS / 2): two 32 KT-byte
// segments of each row.
template <int KS, int LAYOUT, int DS = 0, int NW = kWaves, int KH = 1>
__global__ __launch_bounds__(NW * 64) void pq_encode_cs_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub_in, int64_t rows_per_wg,
    const float* __restrict__ C, const float* __restrict__ cn, const half8* __restrict__ img,
    const float* __restrict__ hinit, const float4* __restrict__ bnd, uint8_t* __restrict__ codesT,
    uint2* __restrict__ items, int2* __restrict__ counts, const float2* __restrict__ pdw,
    const float4* __restrict__ bnd2) {
    static_assert(KH == 1 || (KH == 2 && KS % 2 == 0), "K halves");
    constexpr int FR = 8 * KS * 64;
    constexpr int KT = KS / KH;          // K-steps per tile fill
    constexpr int PITCH = 32 * KT + 16;  // bytes per fp16 tile row (16 B pad: conflict-free reads)
    constexpr int NIMAX = LAYOUT == 0 ? max_loads<KT>() : 2 * KT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    half8* cimg = reinterpret_cast<half8*>(smem);
    unsigned char* stg_all = smem + FR * 16;
    constexpr int NT = NW * 64;
    constexpr int kDep = (NW >= kWaves || KH > 1) ? 1 : 2;  // x blocks in flight per wave
    float* hb = reinterpret_cast<float*>(stg_all + NW * 32 * PITCH);
    float* cnl = hb + 256;
    int* ctr = reinterpret_cast<int*>(cnl + 256);  // [0] pairs, [1] full, [2] resolve batches
    constexpr int kProd = NW;  // streaming waves

    const int dsub = DS > 0 ? DS : dsub_in;
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;  // w: wave-uniform (SGPR)
    const int r = l & 31, h = l >> 5;
    int m;
    int64_t chunk;
    wg_coords(M, m, chunk);
    const int64_t r0 = chunk * rows_per_wg;
    const int64_t r1 = min(n, r0 + rows_per_wg);
    if (r0 >= r1) return;
    const int nrows = (int)(r1 - r0);

    {  // stage the subspace's fp16 codebook image, norms; zero the tiles (pad columns stay 0)
        const half8* src = img + (int64_t)m * FR;
        for (int f = tid; f < FR; f += NT) cimg[f] = src[f];
        uint4* z = reinterpret_cast<uint4*>(stg_all);
        for (int f = tid; f < NW * 32 * PITCH / 16; f += NT) z[f] = make_uint4(0u, 0u, 0u, 0u);
        if (tid < 256) {
            hb[tid] = hinit[(int64_t)m * 256 + tid];
            cnl[tid] = cn[(int64_t)m * 256 + tid];
        }
        if (tid < 4) ctr[tid] = 0;
    }
    __syncthreads();
    {

    // ------------------------------------------------------------------ phase 1: stream
    // Load geometry.  LAYOUT 0: instruction i reads rows rpi*i + [0, rpi), lanes past
    // rpi*q idle.  LAYOUT P in {1, 3}: the vb's 32*q chunks are read in order, 64 per
    // instruction, all lanes busy; the lane pattern repeats every P instructions (RP rows),
    // so P per-lane offsets suffice.
    const int dsub_h = dsub / KH;            // floats per tile fill (KH = 2: dsub == 16 KS)
    const int q = dsub_h >> 2;               // 16-B chunks per row and tile fill
    const int XS = d;                        // row stride of the loads
    constexpr int PER = LAYOUT == 0 ? 1 : LAYOUT;
    const int rpi = LAYOUT == 0 ? min(32, 64 / q) : 64 * PER / q;  // rows per instruction / period
    const int ni = LAYOUT == 0 ? (32 + rpi - 1) / rpi : q / 2;
    int prow[PER], voff[PER], toff[PER];
    bool lactive = true;
#pragma unroll
    for (int sidx = 0; sidx < PER; ++sidx) {
        const int c = LAYOUT == 0 ? l : 64 * sidx + l;
        prow[sidx] = c / q;
        const int col = c - prow[sidx] * q;
        const int gcol = 4 * col;
        voff[sidx] = (prow[sidx] * XS + gcol) * 4;
        toff[sidx] = prow[sidx] * PITCH + 8 * col;
    }
    if (LAYOUT == 0) lactive = l < rpi * q;
    // Buffer over this workgroup's rows of subspace m.  voffset + soffset is range-checked, so
    // rows past the range read as zeros without a branch; idle lanes of LAYOUT 0 get a
    // voffset >= 2^31, past any range.
    const __amdgpu_buffer_rsrc_t xr_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + r0 * d + (int64_t)m * dsub), 0,
        (int)(((int64_t)(nrows - 1) * XS + dsub) * 4), kRsrcWord3);
#pragma unroll
    for (int sidx = 0; sidx < PER; ++sidx)
        if (!lactive) voff[sidx] = (int)0x80000000u;

    const float4 bm = bnd[m];
    const float sigma = bm.x;
    const float2v sig2 = {sigma, sigma};
    const float xs_eta = 5.9604645e-8f * sqrtf((float)dsub);  // 2^-24 * sqrt(dsub) (pq.hip kEta)
    const uint32_t vmask = opaque_mask();
    unsigned char* stg = stg_all + w * 32 * PITCH;
    const int nvb = (nrows + 31) >> 5;

    // first tile row of instruction i (uniform part) and this lane's row within it
    auto ibase = [&](int i) { return LAYOUT == 0 ? rpi * i : rpi * (i / PER); };
    // One code path for every vb (no branches around the loads: divergent paths would make the
    // compiler join the prefetch registers with moves that wait for the loads right away).
    auto load = [&](int vb, int hh, float4* dst) {
#pragma unroll
        for (int i = 0; i < NIMAX; ++i) {
            if (i < ni) {  // uniform
                // the block's uniform offset goes in soffset (SALU; gfx950 range-checks
                // voffset + soffset, tools/probes/soffset_range.hip), the lane's in voffset
                const int so = (vb * 32 + ibase(i)) * XS * 4 + hh * (16 * KT * 4);
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr_rsrc, voff[i % PER], so,
                                                                      DS == 48 ? kXAux48 : kXAux);
                dst[i] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                                     __uint_as_float(v[3]));
            }
        }
    };

    // Pair window inside the filter (pdw != null): a row with exactly two candidates is held
    // for one step while the 8-B load of its pair spreads {||c~_k1 - c~_k2||, ||dc_k1 - dc_k2||}
    // (pq_prep_spread_kernel) is in flight; if the score gap exceeds the pair's own f16
    // rounding bound, k1 is the code and the row never reaches the resolve kernel.
    int pend_row = -1, pend_k = 0;
    float pend_gap = 0.0f, pend_xs = 0.0f;
    float2 pend_pd = make_float2(0.0f, 0.0f);
    // The pair's load is issued and consumed inside one step (before the refill, settled at the
    // tail): as a loop-carried load result, the compiler copied it at the loop latch, i.e. waited
    // vmcnt(0) -- for the next x block's refill too -- at the end of every step.  M > 64 (no
    // per-pair spreads prepared): every pair goes to the list.
    const bool pd_on = pdw != nullptr;
    const float2* pdsrc = pd_on ? pdw : reinterpret_cast<const float2*>(bnd2);
    const float4 b2 = pd_on ? bnd2[m] : make_float4(0.f, 0.f, 0.f, 0.f);
    // The pending pair's spreads: every lane loads (a pair-less lane, or M > 64, reads a valid
    // 8 B that is never used), so no branch surrounds the load.
    // dsub 64 at 16 waves: the round-4 loop with both accumulators spills (20-140 B per lane,
    // 3 % slower), so that kernel runs it with ONE accumulator (kNoPipe: the next centroid
    // block's MFMAs wait for this block's ranking; the other three waves of the SIMD overlap
    // them): 122 VGPRs, 6.52 -> 6.47 ms per 6.65M x 1024 call (profiles/r04_s19).  The generic
    // shapes (DS == 0) keep round 3's structure (refill under its branch, the pair load at the
    // tail, the sigma test per block): their register budgets differ per KS.  (Measured and
    // dropped, round 4: a fixed count of range-checked stores per step, profiles/r04_s9, r04_s28.)
    constexpr bool kR3Loop = DS == 0;
    constexpr bool kNoPipe = DS == 64 && NW == 16;
    constexpr bool kPdEarly = !kR3Loop;
    constexpr bool kRefillCond = kR3Loop;
    constexpr bool kPin = !kR3Loop;
    auto load_pending_pd = [&]() __attribute__((always_inline)) {
        const bool on = pd_on && pend_row >= 0;
        pend_pd = pdsrc[((int64_t)(pd_on ? m : 0) * 256 + (on ? (pend_k & 0xFF) : 0)) * 256 + (on ? (pend_k >> 8) : 0)];
    };
    auto settle_pending = [&]() __attribute__((always_inline)) {
        if (pend_row < 0) return false;
        if (!pd_on) return true;
        const float w12 = 1.0625f * (fmaf(4.8828125e-4f, pend_xs, b2.z) * pend_pd.x + pend_xs * pend_pd.y +
                                     b2.x * pend_xs + b2.y);
        if (pend_gap > w12) {
            codesT[code_at(r0 + pend_row, m, n, M)] = (uint8_t)(pend_k & 0xFF);
            return false;
        }
        return true;
    };
    // Appends this wave's pair items (row prow, candidates pk) and full items (row frow) to the
    // workgroup's lists: pairs from the front, full items from the back.
    auto append = [&](bool isp, int prow, int pk, bool isf, int frow) __attribute__((always_inline)) {
        const uint64_t bp = __ballot(isp);
        const uint64_t bfull = __ballot(isf);
        if (bp | bfull) {
            int basep = 0, basef = 0;
            if (l == 0) {
                if (bp) basep = atomicAdd(&ctr[0], __popcll(bp));
                if (bfull) basef = atomicAdd(&ctr[1], __popcll(bfull));
            }
            basep = __shfl(basep, 0);
            basef = __shfl(basef, 0);
            const uint64_t below = (1ull << l) - 1ull;
            uint2* list = items + (int64_t)m * n + r0;
            if (isp) list[basep + __popcll(bp & below)] = make_uint2((uint32_t)prow, (uint32_t)pk);
            if (isf) list[nrows - 1 - (basef + __popcll(bfull & below))] = make_uint2((uint32_t)frow, 0u);
        }
    };

    // One step encodes block vb from registers xr and refills xr with block vb + kDep*NW
    // right after staging it, so kDep blocks per wave are in flight.
    auto step = [&](auto kScaled, const int vb, float4 (&xrh)[KH][NIMAX]) __attribute__((always_inline)) {
        half8 bf[KS];
        float xx = 0.0f;
#pragma unroll
        for (int hh = 0; hh < KH; ++hh) {
        float4 (&xr)[NIMAX] = xrh[hh];
        // sigma * x -> fp16 -> this wave's tile (LAYOUT 0: lanes past the block's rows skip).
        // sigma == 1 (ordinary codebook magnitudes) runs a loop without the multiply; the choice
        // is made once per workgroup, outside the loop (a uniform branch here made the register
        // allocator join the x registers of two paths with copies that wait for every load;
        // kScaled == 2: the round-3 per-block test, kept for dsub 64).
        auto stage = [&](bool scaled) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < NIMAX; ++i) {
                if (i < ni && (LAYOUT != 0 || (lactive && ibase(i) + prow[0] < 32))) {
                    if (scaled) {
                        const float2v lo = (float2v){xr[i].x, xr[i].y} * sig2;
                        const float2v hi = (float2v){xr[i].z, xr[i].w} * sig2;
                        *reinterpret_cast<uint2*>(stg + ibase(i) * PITCH + toff[i % PER]) =
                            make_uint2(cvt2(lo.x, lo.y), cvt2(hi.x, hi.y));
                    } else {
                        *reinterpret_cast<uint2*>(stg + ibase(i) * PITCH + toff[i % PER]) =
                            make_uint2(cvt2(xr[i].x, xr[i].y), cvt2(xr[i].z, xr[i].w));
                    }
                }
            }
        };
        if constexpr (decltype(kScaled)::value == 2) {  // one branch around the whole block
            if (sigma == 1.0f)
                stage(false);
            else
                stage(true);
        } else {
            stage(decltype(kScaled)::value == 1);
        }
        lds_fence();
        if constexpr (KH > 1) {
            // contiguous halves: tile half hh holds dims [hh dsub/2, (hh+1) dsub/2), which are
            // exactly the dims of lane half h == hh for every image K-step (8 KS h + 8 g + j),
            // so those lanes read all KS fragments from it (exec-masked, no VALU) and the row
            // segment is read as two whole-line halves
            if (h == hh) {
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    bf[ks] = *reinterpret_cast<const half8*>(stg + r * PITCH + 16 * ks);
                    const u32x4 u = __builtin_bit_cast(u32x4, bf[ks]);
                    xx = dot2_self(u[0], xx); xx = dot2_self(u[1], xx);
                    xx = dot2_self(u[2], xx); xx = dot2_self(u[3], xx);
                }
            }
        } else {
#pragma unroll
        for (int ks = 0; ks < KT; ++ks) {
            bf[hh * KT + ks] = *reinterpret_cast<const half8*>(stg + r * PITCH + h * (16 * KT) + 16 * ks);
            const u32x4 u = __builtin_bit_cast(u32x4, bf[hh * KT + ks]);
            xx = dot2_self(u[0], xx); xx = dot2_self(u[1], xx);
            xx = dot2_self(u[2], xx); xx = dot2_self(u[3], xx);
        }
        }
        // The refill is unconditional: past the workgroup's last block the range-checked buffer
        // returns zeros without a memory access.  (Under a branch, the join made the compiler
        // wait vmcnt(0) at the step's tail for the pair-spread load -- i.e. for this refill too,
        // so the next block's loads had only one step's compute to land in.)
        // issued before the refill, so its wait at the tail leaves the refill in flight
        if (kPdEarly && hh == 0) load_pending_pd();
        if (!kRefillCond || vb + kDep * kProd < nvb) load(vb + kDep * kProd, hh, xr);
        // keeps the loads here: the scheduler otherwise sinks them below the MFMAs (shorter
        // register live ranges), leaving them only the step's tail to land in
        if (kPin) __builtin_amdgcn_sched_barrier(0);
        }
        xx += upper_half(xx);  // lanes 0..31: the row norm over both halves

        // Candidates: the 16 packed scores of centroid block cb in this lane form a group; each
        // group keeps its top-2 (g1, g2: pack, then max3 + med3 + max per two scores), and (t1, t2, t3) is the
        // top-3 of all groups' top-2s.  t1, t2 are then the lane's true first and second; a
        // value that no group's top-2 holds lies below its group's g2, so with R = max g2:
        //   t2 < thr                        -> one candidate,
        //   t2 >= thr, t3 < thr, R < thr    -> exactly two (t1, t2),
        //   t3 >= thr or R >= thr           -> possibly more: full item.
        // R is folded into the third slot (t3 := max(t3, R) after each group): R <= t2 always,
        // so the inserts keep t1, t2 exact and t3 = max(third, R), also across the lane-pair
        // merge.  (A pair inside one group becomes a full item: about 1/16 of the pairs.)
        float t1 = -INFINITY, t2 = -INFINITY, t3 = -INFINITY;
        constexpr int NCB = 8;
        // MFMAs of centroid block cb+1 go into the other accumulator before the top-3 of cb
        // reads this one, so a wave's matrix and vector work overlap
        // KH = 2: the A fragments in two halves (a scheduling barrier between them), so at most
        // KS/2 of them are live next to the block's x registers
        auto scores = [&](int cb) __attribute__((always_inline)) {
            floatx16 acc;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const float4 hv = *reinterpret_cast<const float4*>(hb + cb * 32 + 8 * qq + 4 * h);
                acc[4 * qq + 0] = hv.x; acc[4 * qq + 1] = hv.y;
                acc[4 * qq + 2] = hv.z; acc[4 * qq + 3] = hv.w;
            }
            constexpr int NP = KH > 1 ? 2 : 1;
#pragma unroll
            for (int part = 0; part < NP; ++part) {
                half8 a[KS / NP];
#pragma unroll
                for (int ks = 0; ks < KS / NP; ++ks)
                    a[ks] = cimg[(cb * KS + part * (KS / NP) + ks) * 64 + l];
#pragma unroll
                for (int ks = 0; ks < KS / NP; ++ks)
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks], bf[part * (KS / NP) + ks], acc, 0, 0, 0);
                if (NP > 1 && part == 0) __builtin_amdgcn_sched_barrier(0);
            }
            return acc;
        };
        {
            floatx16 acc_cur = scores(0);
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                floatx16 acc_next;
                if (!kNoPipe && cb + 1 < NCB) acc_next = scores(cb + 1);
                {
                    // a group's first two scores: their max and min (2 ops), then 3 per pair
                    const float a0 = pack_idx(acc_cur[0], vmask, (uint32_t)(cb * 32));
                    const float a1 = pack_idx(acc_cur[1], vmask, (uint32_t)(cb * 32 + 1));
                    float g1, g2;
                    asm("v_max_f32 %0, %1, %2" : "=v"(g1) : "v"(a0), "v"(a1));
                    asm("v_min_f32 %0, %1, %2" : "=v"(g2) : "v"(a0), "v"(a1));
#pragma unroll
                    for (int i = 2; i < 16; i += 2)
                        top2_insert2(g1, g2, pack_idx(acc_cur[i], vmask, (uint32_t)(cb * 32 + (i & 3) + 8 * (i >> 2))),
                                     pack_idx(acc_cur[i + 1], vmask,
                                              (uint32_t)(cb * 32 + ((i + 1) & 3) + 8 * ((i + 1) >> 2))));
                    merge_group(t1, t2, t3, g1, g2);
                }
                if (cb + 1 < NCB) acc_cur = kNoPipe ? scores(cb + 1) : acc_next;
            }
        }
        const uint32_t hbit = (uint32_t)h << 2;
        t1 = __uint_as_float(__float_as_uint(t1) | hbit);
        t2 = __uint_as_float(__float_as_uint(t2) | hbit);
        t3 = __uint_as_float(__float_as_uint(t3) | hbit);
        {
            const float p1 = upper_half(t1), p2 = upper_half(t2), p3 = upper_half(t3);
            top3_insert(t1, t2, t3, p1);
            top3_insert(t1, t2, t3, p2);
            top3_insert(t1, t2, t3, p3);
        }
        // Xs >= ||sigma x||: |sigma x - x~| <= 2^-11 |sigma x| + 2^-24 per component
        // (v_sqrt_f32: 1 ulp, inside the 1e-5 margin; a flushed denormal xx still leaves Xs >= xs_eta)
        const float Xs = (__builtin_amdgcn_sqrtf(xx) * (1.0f + 1e-5f) + xs_eta) * (1.0f + 9.765625e-4f);
        const float W = bm.y * Xs + bm.z;
        const float thr = t1 - W;
        const bool bad = !(Xs < 65000.0f) || !isfinite(t1) || !isfinite(W);
        const int ncand = bad ? 3 : 1 + (t2 >= thr) + (t3 >= thr);
        const int k1 = (int)(__float_as_uint(t1) & 0xFFu);
        const int k2 = (int)(__float_as_uint(t2) & 0xFFu);
        const int rowl = vb * 32 + r;
        const bool mine = (h == 0) && rowl < nrows;
        if (mine && ncand == 1) codesT[code_at(r0 + rowl, m, n, M)] = (uint8_t)k1;
        const float gap = __fmul_rn(__fsub_rn(t1, t2), 0.99999988f);  // rounded down
        if (kR3Loop && pdw != nullptr) {
            // round-3 tail (dsub 64, generic shapes): settle the previous block's pair, then
            // load this block's pair spreads (a runtime branch: M > 64 appends pairs directly)
            const bool listp = settle_pending();
            append(listp, pend_row, pend_k, mine && ncand >= 3, rowl);
            const bool np = mine && ncand == 2;
            pend_pd = pdw[((int64_t)m * 256 + (np ? k1 : 0)) * 256 + (np ? k2 : 0)];
            pend_row = np ? rowl : -1;
            pend_k = k1 | (k2 << 8);
            pend_gap = gap;
            pend_xs = Xs;
        } else if (!kR3Loop) {
            // The previous block's pair (its pd load went out before this block's refill): k1
            // is the code when the gap exceeds the pair's own window, else it goes to the list.
            const bool listp = settle_pending();
            append(listp, pend_row, pend_k, mine && ncand >= 3, rowl);
            pend_row = mine && ncand == 2 ? rowl : -1;
            pend_k = k1 | (k2 << 8);
            pend_gap = gap;
            pend_xs = Xs;
            if (!kPdEarly) load_pending_pd();
        } else {
            append(mine && ncand == 2, rowl, k1 | (k2 << 8), mine && ncand >= 3, rowl);  // M > 64: no pair window
        }
    };
    auto run = [&](auto kScaled) __attribute__((always_inline)) {
        float4 xa[KH][NIMAX], xb[KH][NIMAX];
        int vb = w;
#pragma unroll
        for (int hh = 0; hh < KH; ++hh) {
            if (vb < nvb) load(vb, hh, xa[hh]);
            if (kDep == 2 && vb + kProd < nvb) load(vb + kProd, hh, xb[hh]);
        }
        for (; vb < nvb; vb += kDep * kProd) {
            step(kScaled, vb, xa);
            if (kDep == 1) continue;
            if (vb + kProd >= nvb) break;
            step(kScaled, vb + kProd, xb);
        }
    };
    if constexpr (kR3Loop) {
        run(std::integral_constant<int, 2>{});  // sigma tested per block
    } else {
        if (sigma == 1.0f)
            run(std::integral_constant<int, 0>{});
        else
            run(std::integral_constant<int, 1>{});
    }
    if (!kR3Loop || pdw != nullptr) {  // the last block's pending pair
        if (kPdEarly) load_pending_pd();
        const bool listp = settle_pending();
        append(listp, pend_row, pend_k, false, 0);
    }
    }  // producers
    __syncthreads();
    if (tid == 0) counts[blockIdx.x] = make_int2(ctr[0], ctr[1]);
}

// Merged resolve (the library default): one launch settles a workgroup's full items and the
// pairs its filter could not settle with the pair window.  One workgroup (4 waves, one per
// SIMD: up to 512 registers per lane) per encode workgroup; LDS holds the exact fp32 codebook
// C_m (the canonical chains of both kinds read it), the norms, the accumulator init, and per
// wave a 32-row fp32 staging tile.  A full batch loads the filter's f16 A operands of all 8
// centroid blocks (192 registers at KS = 6, from the L2-resident prepared image) together with
// its row gather.
//   full batch (32 rows): gather the rows, build the B operand exactly as the filter does, one
//     MFMA sweep with all 8 accumulators kept, t1 = max; each lane marks its centroids inside
//     the window (score >= t1 - W) in a 128-bit mask (registers only) and runs their canonical
//     chains in increasing k, one loop for all of them; the two lanes of a row merge (s, k).
//     Every minimiser of the canonical score lies inside the window, so the smallest (s, k) is
//     the canonical code.  Rows the window cannot vouch for (non-finite, out of range) take all
//     256 centroids.  (Round 1 appended the candidates to per-lane LDS lists: 128 conflicted
//     stores per lane per batch.)
//   pair batch (32 rows): lane (r, 0) runs the chain of k1, lane (r, 1) that of k2; merge.
// (Tried and dropped: claiming batches one ahead so the next pair batch's rows load during the
// current one: no gain (+10 % per launch in that build).  With every chain and MFMA skipped the
// launch still takes ~85 us: the row gathers run at ~4 TB/s of random 384-B segments.)
constexpr int kMWaves = 4;

// The LDS codebook keeps rows 16*KS floats apart (no room for padding) with the 16-B chunks of
// row k permuted by j -> j ^ (k & 7) (k & 3 when a row has 4 (mod 8) chunks): random-k chain
// reads then spread over the bank row (unswizzled, a 96-float pitch maps every row to the same
// two bank offsets: 22 M conflict cycles per 1M-row call, PMC).
template <int KS>
__device__ __forceinline__ int cswz(int k) { return (4 * KS) % 8 == 0 ? (k & 7) : (k & 3); }

// Wide subspaces (KS > 6): the fp32 codebook (up to 192 KiB) does not fit in LDS; the
// canonical chains read the centroid rows from C itself (L2-resident) and the full batches
// load the A operands one centroid block at a time.
template <int KS>
constexpr bool merged_gc() { return KS > 6; }

// GC full batches: the (row, centroid) candidates of a batch go to a per-wave LDS list of up
// to kGcCap entries and are chained 64 at a time, one per lane (a lane-per-row loop would run
// as many steps as the busiest lane has candidates, each an L2 round trip plus a dsub-long
// chain); per-row (s, k) minima through 64-bit LDS atomics.
constexpr int kGcCap = 4096;

template <int KS>
constexpr int merged_smem_bytes() {
    return (merged_gc<KS>() ? 0 : 256 * 16 * KS * 4) + 2 * 256 * 4 + 16 + kMWaves * (32 * (16 * KS + 4) * 4) +
           (merged_gc<KS>() ? kMWaves * (32 * 8 + kGcCap * 2) : 0);
}

// float -> uint32 whose unsigned order is the float order (-0 == +0; NaN above everything)
__device__ __forceinline__ uint32_t ord_key(float s) {
    const uint32_t u = s == 0.0f ? 0u : __float_as_uint(s);
    return s != s ? 0xFFFFFFFFu : (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <int KS, int DS>
__global__ __launch_bounds__(kMWaves * 64) __attribute__((amdgpu_waves_per_eu(1, 1))) void pq_resolve_merged_kernel(
    const float* __restrict__ x, int64_t n, int d, int M, int dsub_in, int64_t rows_per_wg,
    const float* __restrict__ C, const float* __restrict__ cn, const half8* __restrict__ img,
    const float* __restrict__ hinit, const float4* __restrict__ bnd, uint8_t* __restrict__ codesT,
    const uint2* __restrict__ items, const int2* __restrict__ counts) {
    constexpr int DP = 16 * KS;  // padded dsub
    constexpr int XP = DP + 4;   // floats per staged x row
    constexpr int NL = 2 * KS;   // 16-B loads per lane per 32-row gather
    constexpr int FR = 8 * KS * 64;
    const int dsub = DS > 0 ? DS : dsub_in;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int CP = DP;
    constexpr bool GC = merged_gc<KS>();
    float* cl = reinterpret_cast<float*>(smem);  // [256][DP], chunks swizzled (cswz); GC: none
    float* cnl = cl + (GC ? 0 : 256 * CP);
    float* hb = cnl + 256;
    int* ctr = reinterpret_cast<int*>(hb + 256);
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    const int r = l & 31, h = l >> 5;
    float* xf = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(ctr + 4) +
                                         w * (32 * XP * 4));
    // GC candidate lists (after the staging tiles): per wave 32 row keys, then kGcCap entries
    unsigned long long* gkeys = reinterpret_cast<unsigned long long*>(
                                    reinterpret_cast<unsigned char*>(ctr + 4) + kMWaves * (32 * XP * 4)) + w * 32;
    unsigned short* glist = reinterpret_cast<unsigned short*>(
                                reinterpret_cast<unsigned char*>(ctr + 4) + kMWaves * (32 * XP * 4) + kMWaves * 32 * 8) +
                            w * kGcCap;

    int m;
    int64_t chunk;
    wg_coords(M, m, chunk);
    const int64_t r0 = chunk * rows_per_wg;
    const int64_t r1 = min(n, r0 + rows_per_wg);
    if (r0 >= r1) return;
    const int nrows = (int)(r1 - r0);
    const int2 cnt = counts[blockIdx.x];
    const int np = cnt.x, nf = cnt.y;
    if (np + nf == 0) return;
    const float* Cm = C + (int64_t)m * 256 * dsub;
    {  // the fp32 codebook, zero-padded to DP; 16-B copies, 8 in flight per thread
        const int q4 = DP >> 2, tot = GC ? 0 : 256 * q4;
        for (int e0 = tid; e0 < tot; e0 += 8 * kMWaves * 64) {
            f32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * kMWaves * 64;
                const int k = e / q4, j = e - k * q4;
                v[u] = (e < tot && 4 * j < dsub) ? *reinterpret_cast<const f32x4*>(Cm + (int64_t)k * dsub + 4 * j)
                                                 : (f32x4){0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * kMWaves * 64;
                const int k = e / q4, j = e - k * q4;
                if (e < tot) *reinterpret_cast<f32x4*>(cl + k * CP + 4 * (j ^ cswz<KS>(k))) = v[u];
            }
        }
        cnl[tid] = cn[(int64_t)m * 256 + tid];
        hb[tid] = hinit[(int64_t)m * 256 + tid];
        if (tid == 0) {
            ctr[0] = 0;
            ctr[1] = kMWaves;  // pair batches 0..kMWaves-1 are the waves' first (static)
        }
    }
    __syncthreads();
    const half8* im = img + (int64_t)m * FR;

    const float4 bm = bnd[m];
    const float xs_eta = 5.9604645e-8f * sqrtf((float)dsub);
    const int q = dsub >> 2;
    const int nld = (32 * q + 63) >> 6;
    const uint2* list = items + (int64_t)m * n + r0;
    const float* xsub = x + r0 * d + (int64_t)m * dsub;
    const int nbf = (nf + 31) >> 5, nbp = (np + 31) >> 5;

    // canonical score of centroid k for the row xv held in registers (DS > 0: the whole
    // centroid row is read first, then the sequential fmaf chain runs without waits)
    constexpr int NQ = DS > 0 ? DS / 4 : 1;
    // GC (wide subspaces): the centroid row comes from C (L2) with all of its loads in flight
    // at once (or half of them), so a chain waits for one or two L2 round trips instead of
    // one per 16-B step
    auto exact_reg = [&](const f32x4 (&xv)[NQ], int k) __attribute__((always_inline)) {
        const float* c = GC ? Cm + (int64_t)k * dsub : cl + k * CP;
        const int sw = GC ? 0 : cswz<KS>(k);
        // the centroid row in two halves (register budget: the pair loop holds a prefetched
        // gather next to the row)
        constexpr int NH = (NQ + 1) / 2;
        float dot = 0.0f;
#pragma unroll
        for (int t0 = 0; t0 < NQ; t0 += NH) {
            f32x4 cv[NH];
#pragma unroll
            for (int t = 0; t < NH; ++t)
                if (t0 + t < NQ) cv[t] = *reinterpret_cast<const f32x4*>(c + 4 * ((t0 + t) ^ sw));
#pragma unroll
            for (int t = 0; t < NH; ++t) {
                if (t0 + t < NQ) {
                    dot = __builtin_fmaf(xv[t0 + t].x, cv[t].x, dot);
                    dot = __builtin_fmaf(xv[t0 + t].y, cv[t].y, dot);
                    dot = __builtin_fmaf(xv[t0 + t].z, cv[t].z, dot);
                    dot = __builtin_fmaf(xv[t0 + t].w, cv[t].w, dot);
                }
            }
        }
        return __builtin_fmaf(-2.0f, dot, cnl[k]);
    };
    auto load_row = [&](const float* xr, f32x4 (&xv)[NQ]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < NQ; ++t) xv[t] = *reinterpret_cast<const f32x4*>(xr + 4 * t);
    };
    // GC, DS > 0: canonical score of centroid k for the staged row xrr (LDS); the centroid row
    // comes from C in NC pieces, each with all of its loads in flight (one L2 round trip per
    // piece instead of one per 16-B step)
    auto chain_gc = [&](auto nc_tag, const float* xrr, int k) __attribute__((always_inline)) {
        constexpr int NC = decltype(nc_tag)::value;
        constexpr int NP = (NQ + NC - 1) / NC;
        const float* c = Cm + (int64_t)k * dsub;
        float dot = 0.0f;
#pragma unroll
        for (int t0 = 0; t0 < NQ; t0 += NP) {
            f32x4 cv[NP];
#pragma unroll
            for (int t = 0; t < NP; ++t)
                if (t0 + t < NQ) cv[t] = *reinterpret_cast<const f32x4*>(c + 4 * (t0 + t));
#pragma unroll
            for (int t = 0; t < NP; ++t) {
                if (t0 + t < NQ) {
                    const f32x4 xq = *reinterpret_cast<const f32x4*>(xrr + 4 * (t0 + t));
                    dot = __builtin_fmaf(xq.x, cv[t].x, dot);
                    dot = __builtin_fmaf(xq.y, cv[t].y, dot);
                    dot = __builtin_fmaf(xq.z, cv[t].z, dot);
                    dot = __builtin_fmaf(xq.w, cv[t].w, dot);
                }
            }
        }
        return __builtin_fmaf(-2.0f, dot, cnl[k]);
    };
    // canonical score of centroid k for the staged row xr (sequential fmaf chain over t), any
    // dsub; GC: the centroid row straight from C (unswizzled)
    auto exact = [&](const float* xr, int k) __attribute__((always_inline)) {
        const float* c = GC ? Cm + (int64_t)k * dsub : cl + k * CP;
        const int sw = GC ? 0 : cswz<KS>(k);
        float dot = 0.0f;
#pragma unroll 2
        for (int t = 0; t < (DS > 0 ? DS : dsub); t += 4) {
            const f32x4 cv = *reinterpret_cast<const f32x4*>(c + 4 * ((t >> 2) ^ sw));
            const f32x4 xv = *reinterpret_cast<const f32x4*>(xr + t);
            dot = __builtin_fmaf(xv.x, cv.x, dot);
            dot = __builtin_fmaf(xv.y, cv.y, dot);
            dot = __builtin_fmaf(xv.z, cv.z, dot);
            dot = __builtin_fmaf(xv.w, cv.w, dot);
        }
        return __builtin_fmaf(-2.0f, dot, cnl[k]);
    };
    // The rows of a batch (row offsets in rowl of lanes 0..cntb-1) are gathered in two halves:
    // gather_issue puts the 16-B loads in flight into registers, gather_commit writes them to
    // the wave's staging tile.  The loop issues batch b+1's gather before it computes batch b
    // (after a full batch's A-operand loads, so waiting for those never waits for the prefetch):
    // each wave keeps one batch of row gathers in flight while it computes.
    auto gather_issue = [&](int cntb, int rowl, f32x4 (&v)[NL]) __attribute__((always_inline)) {
        // the lane index through an opaque move: the per-j offsets are recomputed per gather
        // (a few VALU) instead of being hoisted out of the batch loop (2 NL registers)
        int lv;
        asm volatile("v_mov_b32 %0, %1" : "=v"(lv) : "v"(l));
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int c = j * 64 + lv;
            const int row = c / q, col = c - row * q;
            const int src = __shfl(rowl, min(row, 31));
            const bool ok = j < nld && row < cntb;
            v[j] = *reinterpret_cast<const f32x4*>(xsub + (ok ? (int64_t)src * d + 4 * col : 0));
        }
    };
    auto gather_commit = [&](const f32x4 (&v)[NL]) __attribute__((always_inline)) {
        int lv;
        asm volatile("v_mov_b32 %0, %1" : "=v"(lv) : "v"(l));
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int c = j * 64 + lv;
            const int row = c / q, col = c - row * q;
            if (j < nld && row < 32) *reinterpret_cast<f32x4*>(xf + row * XP + 4 * col) = v[j];
        }
        if (DS == 0 || DS != DP)
            for (int e = l; e < 32 * (DP - dsub); e += 64) {
                const int row = e / (DP - dsub);
                xf[row * XP + dsub + (e - row * (DP - dsub))] = 0.0f;
            }
        lds_fence();
    };
    // batch b's items: lanes with r < cntb hold (row, k1 | k2 << 8) (full items: (row, 0))
    auto batch_info = [&](int b, uint2& it, int& cntb) __attribute__((always_inline)) {
        const bool full = b < nbf;
        const int first = (full ? b : b - nbf) * 32;
        cntb = min(32, (full ? nf : np) - first);
        // unconditional (clamped) load: no load sits on a divergent path, so the compiler's
        // wait-count bookkeeping stays exact around the prefetched gathers
        const int e = full ? nrows - 1 - (first + r) : first + r;
        const uint2 v = list[r < cntb ? e : 0];
        it = r < cntb ? v : make_uint2(0u, 0u);
    };

    // full batch (rows staged): one MFMA sweep with the A operands aa, window mask, chains
    auto full_batch = [&](const half8 (&aa)[GC ? 1 : 8][KS], int cntb, int rowl) __attribute__((always_inline)) {
        const float* xr = xf + r * XP;
        half8 bf[KS];
        float xx = 0.0f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const float* src = xr + h * 8 * KS + 8 * ks;
            const u32x4 u = cvt8_scaled(*reinterpret_cast<const f32x4*>(src), *reinterpret_cast<const f32x4*>(src + 4),
                                        bm.x);
            bf[ks] = __builtin_bit_cast(half8, u);
            xx = dot2_self(u[0], xx); xx = dot2_self(u[1], xx);
            xx = dot2_self(u[2], xx); xx = dot2_self(u[3], xx);
        }
        xx += __shfl_xor(xx, 32);
        floatx16 acc[8];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const float4 hv = *reinterpret_cast<const float4*>(hb + cb * 32 + 8 * qq + 4 * h);
                acc[cb][4 * qq + 0] = hv.x; acc[cb][4 * qq + 1] = hv.y;
                acc[cb][4 * qq + 2] = hv.z; acc[cb][4 * qq + 3] = hv.w;
            }
        }
        if constexpr (GC) {
            // the lane index through an opaque move: the 8 KS fragment addresses are formed
            // here, per batch, not hoisted out of the batch loop (2 registers each)
            int lv;
            asm volatile("v_mov_b32 %0, %1" : "=v"(lv) : "v"(l));
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {
                half8 a1[KS];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) a1[ks] = im[(cb * KS + ks) * 64 + lv];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[ks], bf[ks], acc[cb], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int cb = 0; cb < 8; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aa[cb][ks], bf[ks], acc[cb], 0, 0, 0);
        }
        float t1 = -INFINITY;
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
#pragma unroll
            for (int i = 0; i < 16; ++i) t1 = fmaxf(t1, acc[cb][i]);
        t1 = fmaxf(t1, __shfl_xor(t1, 32));
        const float Xs = (__builtin_amdgcn_sqrtf(xx) * (1.0f + 1e-5f) + xs_eta) * (1.0f + 9.765625e-4f);
        const float W = bm.y * Xs + bm.z;
        const float thr = t1 - W;
        const bool bad = !(Xs < 65000.0f) || !isfinite(t1) || !isfinite(W);
        // this lane's centroids inside the window as a 128-bit mask (4 words of two centroid
        // blocks; register-only, no per-value LDS stores), then their canonical chains in
        // increasing k, one loop for all of them; a row the window cannot vouch for takes
        // all 128 of the lane's centroids
        uint32_t wm[4];
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
            uint32_t mm = 0u;
#pragma unroll
            for (int i = 0; i < 32; ++i) mm |= acc[2 * q2 + (i >> 4)][i & 15] >= thr ? (1u << i) : 0u;
            wm[q2] = bad ? 0xFFFFFFFFu : mm;
        }
        if constexpr (GC && DS > 0) {
            // candidate list: lane prefix of the candidate counts, entries (row << 8) | k
            const int cnt = r < cntb ? __popc(wm[0]) + __popc(wm[1]) + __popc(wm[2]) + __popc(wm[3]) : 0;
            int inc = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(inc, o);
                if (l >= o) inc += t;
            }
            const int T = __builtin_amdgcn_readfirstlane(__shfl(inc, 63));
            if (T <= kGcCap) {
                if (l < 32) gkeys[l] = ~0ull;
                int at = inc - cnt;
                if (r < cntb) {
#pragma unroll
                    for (int q2 = 0; q2 < 4; ++q2) {
                        uint32_t mm = wm[q2];
                        while (mm) {
                            const int bit = __builtin_ctz(mm);
                            mm &= mm - 1u;
                            const int cb = 2 * q2 + (bit >> 4), i = bit & 15;
                            glist[at++] = (unsigned short)((r << 8) | (cb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h));
                        }
                    }
                }
                lds_fence();
                for (int base = 0; base < T; base += 64) {
                    if (base + l < T) {
                        const int e = glist[base + l];
                        const int rr = e >> 8, k = e & 0xFF;
                        const float sc = chain_gc(std::integral_constant<int, (DS > 128 ? kGcListNc : 1)>{}, xf + rr * XP, k);
                        atomicMin(&gkeys[rr], ((unsigned long long)ord_key(sc) << 32) | (unsigned)k);
                    }
                }
                lds_fence();
                if (h == 0 && r < cntb) {
                    const unsigned long long key = gkeys[r];
                    // (s, k) minimum; no finite-or--inf candidate (all NaN / +inf) -> 0, as below
                    codesT[code_at(r0 + rowl, m, n, M)] = (uint8_t)((uint32_t)(key >> 32) < 0xFF800000u ? (key & 0xFF) : 0);
                }
                return;
            }
        }
        float bs = INFINITY;
        int bk = 256;
        auto take = [&](float sc, int k) __attribute__((always_inline)) {
            if (sc < bs || (sc == bs && k < bk)) { bs = sc; bk = k; }
        };
        if (r < cntb) {
            f32x4 xv[GC ? 1 : NQ];
            if constexpr (DS > 0 && !GC) load_row(xr, xv);
            while ((wm[0] | wm[1] | wm[2] | wm[3]) != 0u) {
                const int wi = wm[0] ? 0 : wm[1] ? 1 : wm[2] ? 2 : 3;
                const uint32_t wsel = wm[0] ? wm[0] : wm[1] ? wm[1] : wm[2] ? wm[2] : wm[3];
                const int bit = __builtin_ctz(wsel);
                const uint32_t rest = wsel & (wsel - 1u);
                wm[0] = wi == 0 ? rest : wm[0];
                wm[1] = wi == 1 ? rest : wm[1];
                wm[2] = wi == 2 ? rest : wm[2];
                wm[3] = wi == 3 ? rest : wm[3];
                const int cb = 2 * wi + (bit >> 4), i = bit & 15;
                const int k = cb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                if constexpr (GC && DS > 0) take(chain_gc(std::integral_constant<int, (DS > 128 ? 2 : 1)>{}, xr, k), k);
                else if constexpr (DS > 0) take(exact_reg(xv, k), k);
                else take(exact(xr, k), k);
            }
        }
        const float os = __shfl_xor(bs, 32);
        const int ok = __shfl_xor(bk, 32);
        if (os < bs || (os == bs && ok < bk)) { bs = os; bk = ok; }
        if (h == 0 && r < cntb) codesT[code_at(r0 + rowl, m, n, M)] = (uint8_t)((bs < INFINITY) ? bk : 0);
    };
    // pair batch (rows staged): lane (r, 0) runs the chain of k1, lane (r, 1) that of k2
    auto pair_batch = [&](int cntb, uint2 it) __attribute__((always_inline)) {
        const float* xr = xf + r * XP;
        const int rowl = (int)it.x;
        const int k1 = (int)(it.y & 0xFFu), k2 = (int)((it.y >> 8) & 0xFFu);
        const int kk = h ? k2 : k1;
        float sc = 0.0f;
        if (r < cntb) {
            if constexpr (GC && DS > 0) {
                // the next batch's gather is in flight (2 KS registers): the centroid row in
                // two pieces when a whole one would not fit next to it
                sc = chain_gc(std::integral_constant<int, (DS + 8 * KS > 200 ? 2 : 1)>{}, xr, kk);
            } else if constexpr (DS > 0) {
                f32x4 xv[NQ];
                load_row(xr, xv);
                sc = exact_reg(xv, kk);
            } else {
                sc = exact(xr, kk);
            }
        }
        const float os = __shfl_xor(sc, 32);
        if (h == 0 && r < cntb) {
            // (s1, k1) here, (s2, k2) from the partner: smallest (s, k), NaN never wins
            const bool two = os < sc || (os == sc && k2 < k1) || (sc != sc && os == os);
            codesT[code_at(r0 + rowl, m, n, M)] = (uint8_t)(two ? k2 : k1);
        }
    };

    // Full batches first (claimed from ctr[0]; their A operands take 192 registers, so their
    // gathers are not prefetched), then pair batches (claimed from ctr[1]) with the next pair
    // batch's gather in flight while the current one is computed.
    // (Round 5 measured the A operands loaded once per wave, with and without the next full
    // batch's gather in flight: no faster)
    for (;;) {
        int bb = 0;
        if (l == 0) bb = atomicAdd(&ctr[0], 1);
        bb = __builtin_amdgcn_readfirstlane(__shfl(bb, 0));
        if (bb >= nbf) break;
        uint2 it;
        int cntb;
        batch_info(bb, it, cntb);
        f32x4 v[NL];
        gather_issue(cntb, (int)it.x, v);
        half8 aa[GC ? 1 : 8][KS];
        if constexpr (!GC) {
#pragma unroll
            for (int cb = 0; cb < 8; ++cb)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) aa[cb][ks] = im[(cb * KS + ks) * 64 + l];
        }
        gather_commit(v);
        full_batch(aa, cntb, (int)it.x);
        lds_fence();  // the tile is rewritten by the next commit
    }
    // pair batches: the first one per wave is static (b = w), the rest are claimed from ctr[1]
    int b = w, cntb = 0;
    uint2 it = make_uint2(0u, 0u);
    f32x4 va[NL], vb2[NL];
    batch_info(nbf + b, it, cntb);
    gather_issue(cntb, (int)it.x, va);
    // one batch: stage vc (batch b), claim the next and put its gather into vn, compute b
    auto iter = [&](const f32x4 (&vc)[NL], f32x4 (&vn)[NL]) __attribute__((always_inline)) {
        int bn = 0;
        if (l == 0) bn = atomicAdd(&ctr[1], 1);
        bn = __builtin_amdgcn_readfirstlane(__shfl(bn, 0));
        uint2 itn;
        int cntn;
        batch_info(nbf + bn, itn, cntn);  // past the end: cntn <= 0, no rows
        // vc's gather and the list entries of bn: everything in flight is needed now
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        gather_commit(vc);
        gather_issue(cntn, (int)itn.x, vn);  // cntn <= 0: every lane reads row 0 (discarded)
        pair_batch(cntb, it);
        lds_fence();  // the tile is rewritten by the next commit
        b = bn;
        it = itn;
        cntb = cntn;
    };
    while (b < nbp) {
        iter(va, vb2);
        if (b >= nbp) break;
        iter(vb2, va);
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

// Same transpose with 16-B memory operations (n % 16 == 0 and 16-B aligned buffers): the
// subspace rows come in as uint4 (16 codes), each thread assembles 16 output bytes from the
// LDS tile ([M][256 + 16], padded) and stores them as one uint4.
template <int MC>  // MC > 0: compile-time M (shifts instead of divisions)
__global__ __launch_bounds__(256) void pq_transpose_codes16_kernel(const uint8_t* __restrict__ codesT, int64_t n,
                                                                   int M_in, uint8_t* __restrict__ codes) {
    const int M = MC > 0 ? MC : M_in;
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];  // [M][272]
    constexpr int TP = 256 + 16;
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    const int rows = (int)min<int64_t>(256, n - r0);  // a multiple of 16
    const int q = rows >> 4;                           // uint4 per subspace row
    for (int e = threadIdx.x; e < M * q; e += 256) {
        const int mm = e / q, c = e - mm * q;
        *reinterpret_cast<uint4*>(tile + mm * TP + 16 * c) =
            *reinterpret_cast<const uint4*>(codesT + (int64_t)mm * n + r0 + 16 * c);
    }
    __syncthreads();
    const int nout = (rows * M) >> 4;  // uint4 of output
    for (int e = threadIdx.x; e < nout; e += 256) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int o = 16 * e + 4 * j + b;  // output byte: row o / M, subspace o % M
                v |= (uint32_t)tile[(o % M) * TP + o / M] << (8 * b);
            }
            w[j] = v;
        }
        *reinterpret_cast<uint4*>(codes + r0 * M + 16 * (int64_t)e) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

}  // namespace

// CU count of the current device, cached per (thread, device): no shared mutable state.
int device_cus() {
    constexpr int kMaxDev = 64;
    static thread_local int cache[kMaxDev] = {};
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev >= 0 && dev < kMaxDev && cache[dev] > 0) return cache[dev];
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    if (dev >= 0 && dev < kMaxDev) cache[dev] = cus;
    return cus;
}

namespace {

// Chunk count for one workgroup per CU at a time: minimise the rounds of workgroups per row
// (ceil(chunks*M / CUs) / chunks), preferring fewer chunks, with at least 32 nw rows each
// and few enough rows that a chunk's buffer offsets fit 31 bits.
int64_t pick_chunks(int64_t n, int d, int M, int cus, int nw) {
    const int64_t rmax = std::max<int64_t>(32, ((int64_t)1 << 31) / ((int64_t)d * 4) - 64);
    const int64_t cmin = ceil_div(n, rmax);
    const int64_t cmax = std::max<int64_t>(cmin, std::min<int64_t>(ceil_div(n, 32 * nw), 4 * (int64_t)cus));
    int64_t best = cmin;
    double best_cost = 1e300;
    for (int64_t c = cmin; c <= cmax; ++c) {
        const double cost = (double)ceil_div(c * M, (int64_t)cus) / (double)c;
        if (cost < best_cost * (1.0 - 1e-9)) { best_cost = cost; best = c; }
    }
    return best;
}

}  // namespace

int cs_smem_bytes(int KS, int dsub) {
    (void)dsub;
    return 8 * KS * 64 * 16 + cs_waves(KS) * 32 * (32 * KS + 16) + 2 * 256 * 4 + 16;
}

// Load layout for dsub (see the kernel): period-P flat layouts where all lanes stay busy.
int cs_layout(int dsub) {
    switch (dsub >> 2) {
        case 2: case 4: case 8: case 16: return 1;
        case 6: case 12: case 24: return 3;
        default: return 0;
    }
}

template <int KS>
hipError_t launch_pq_encode_cs_v(const float* x, int64_t n, int d, int M, int dsub, const float* C, const float* cn,
                                 const void* img, const float* hinit, const void* bnd, const void* pd, const void* bnd2,
                                 uint8_t* codesT, void* items, void* counts, hipStream_t st) {
    const int smem = cs_smem_bytes(KS, dsub);
    const int layout = cs_layout(dsub);
    constexpr int NW = cs_waves(KS);
    auto kern = layout == 1 ? pq_encode_cs_kernel<KS, 1, 0, NW>
              : layout == 3 ? pq_encode_cs_kernel<KS, 3, 0, NW> : pq_encode_cs_kernel<KS, 0, 0, NW>;
    int nw_launch = NW, smem_launch = smem;
    // specialised shapes (addresses and load counts folded; waves per shape measured)
    if constexpr (KS == 6) {  // D = 1536, M = 16: the headline
        // (round 5: 16 waves, one accumulator and the x / centroid fragments read per centroid
        // block to fit 128 VGPRs: 0.3-3 % slower than these 12, profiles/r05_s26)
        if (dsub == 96) kern = pq_encode_cs_kernel<6, 3, 96, 12>;
    }
    if constexpr (KS == 3) {  // D = 1536, M = 32 (the OPQ32 / PQ32 shape of BASELINE config #3)
        if (dsub == 48) {
            constexpr int NW48 = 16;
            kern = pq_encode_cs_kernel<3, 3, 48, NW48>;
            nw_launch = NW48;
            smem_launch = smem + (NW48 - NW) * 32 * (32 * KS + 16);
        }
    }
    if constexpr (KS == 4) {  // D = 1024, M = 16 (BASELINE config #5)
        if (dsub == 64) {
            // (round 5: 12 waves with two pipelined accumulators, 12 with one and 8 waves measured
            // 0.5-4 % slower, profiles/r05_s20)
            constexpr int NW64 = 16;
            kern = pq_encode_cs_kernel<4, 1, 64, NW64>;
            nw_launch = NW64;
            smem_launch = smem + (NW64 - NW) * 32 * (32 * KS + 16);
        }
    }
    // wide subspaces with dsub == 16 KS (128, 160, 192): the tile filled in two K halves, so 8
    // waves fit next to the image instead of 4 (KH = 2 above)
    if constexpr (KS >= 8 && KS % 2 == 0) {
        if (dsub == 16 * KS) {
            constexpr int KT = KS / 2, NWW = 8;
            constexpr int LH = (4 * KT == 24 || 4 * KT == 12) ? 3 : (4 * KT == 16 || 4 * KT == 32) ? 1 : 0;
            kern = pq_encode_cs_kernel<KS, LH, 16 * KS, NWW, 2>;
            nw_launch = NWW;
            smem_launch = 8 * KS * 64 * 16 + NWW * 32 * (32 * KT + 16) + 2 * 256 * 4 + 16;
        }
    }
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem_launch);
    if (e != hipSuccess) return e;
    const int cus = device_cus();
    const int64_t chunks = pick_chunks(n, d, M, cus, nw_launch);
    const int64_t R = align_up(ceil_div(n, chunks), (int64_t)32);
    const int64_t grid = ceil_div(n, R) * M;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(nw_launch * 64), smem_launch, st, x, n, d, M, dsub, R, C, cn,
                       static_cast<const half8*>(img), hinit, static_cast<const float4*>(bnd), codesT,
                       static_cast<uint2*>(items), static_cast<int2*>(counts), static_cast<const float2*>(pd),
                       static_cast<const float4*>(bnd2));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    constexpr int msmem = merged_smem_bytes<KS>();
    static_assert(msmem <= 160 * 1024, "merged resolve LDS");
    // DS specialisations: the row held in registers for the chains (exact_reg); wide
    // subspaces with dsub == 16 KS as well (their chains read C from L2)
    constexpr bool wide_ds = KS >= 8 && KS % 2 == 0;
    auto mkern = (KS == 6 && dsub == 96)   ? pq_resolve_merged_kernel<KS, (KS == 6 ? 96 : 0)>
                 : (KS == 4 && dsub == 64) ? pq_resolve_merged_kernel<KS, (KS == 4 ? 64 : 0)>
                 : (KS == 3 && dsub == 48) ? pq_resolve_merged_kernel<KS, (KS == 3 ? 48 : 0)>
                 : (wide_ds && dsub == 16 * KS) ? pq_resolve_merged_kernel<KS, (wide_ds ? 16 * KS : 0)>
                                           : pq_resolve_merged_kernel<KS, 0>;
    e = hipFuncSetAttribute((const void*)mkern, hipFuncAttributeMaxDynamicSharedMemorySize, msmem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mkern, dim3((unsigned)grid), dim3(kMWaves * 64), msmem, st, x, n, d, M, dsub, R, C, cn,
                       static_cast<const half8*>(img), hinit, static_cast<const float4*>(bnd), codesT,
                       static_cast<const uint2*>(items), static_cast<const int2*>(counts));
    return hipGetLastError();
}

// (at most ceil(n / (32 nw)) row chunks per subspace; nw >= kWideWaves)
size_t cs_counts_bytes(int64_t n, int M) { return (size_t)ceil_div(n, 32 * kWideWaves) * M * sizeof(int2); }

hipError_t launch_pq_encode_cs(int KS, const float* x, int64_t n, int d, int M, int dsub, const float* C,
                               const float* cn, const void* img, const float* hinit, const void* bnd, const void* pd,
                               const void* bnd2, uint8_t* codesT, void* items, void* counts, uint8_t* codes,
                               hipStream_t st) {
    hipError_t e = hipErrorInvalidValue;
    switch (KS) {
#define MIVQ_CS_CASE(k)                                                                                        \
    case k:                                                                                                    \
        e = launch_pq_encode_cs_v<k>(x, n, d, M, dsub, C, cn, img, hinit, bnd, pd, bnd2, codesT,            \
                                     items, counts, st);                                                       \
        break;
        MIVQ_CS_CASE(1) MIVQ_CS_CASE(2) MIVQ_CS_CASE(3) MIVQ_CS_CASE(4) MIVQ_CS_CASE(5) MIVQ_CS_CASE(6)
        MIVQ_CS_CASE(7) MIVQ_CS_CASE(8) MIVQ_CS_CASE(9) MIVQ_CS_CASE(10) MIVQ_CS_CASE(11) MIVQ_CS_CASE(12)
#undef MIVQ_CS_CASE
        default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    const bool v16 = n % 16 == 0 && (reinterpret_cast<uintptr_t>(codesT) % 16) == 0 &&
                     (reinterpret_cast<uintptr_t>(codes) % 16) == 0 && M <= 256;
    if (v16 && M == 16)
        hipLaunchKernelGGL(pq_transpose_codes16_kernel<16>, dim3((unsigned)ceil_div(n, 256)), dim3(256),
                           (size_t)(256 + 16) * M, st, codesT, n, M, codes);
    else if (v16)
        hipLaunchKernelGGL(pq_transpose_codes16_kernel<0>, dim3((unsigned)ceil_div(n, 256)), dim3(256),
                           (size_t)(256 + 16) * M, st, codesT, n, M, codes);
    else
        hipLaunchKernelGGL(pq_transpose_codes_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), (size_t)256 * M,
                           st, codesT, n, M, codes);
    return hipGetLastError();
}

}  // namespace mivq
