// lut_stress.hip — root-cause probe for the two-stream adc_lut mismatch.
//
// Runs an ADC-LUT kernel variant on stream A many times while a partner kernel runs on
// stream B, and compares every LUT with the serial result.  Variants:
//   v4f   : round 2's 16-B centroid loads (the form that failed 1-5 of 8 trials)
//   dword : the dword loads that replaced it
//   lib   : mivq_adc_lut from libmivq.so (whatever HEAD ships)
//   v4f_scalar : 16-B loads, math kept off the packed fp32 instructions
//   dword_pk   : dword loads, math forced onto v_pk_add_f32 / v_pk_fma_f32
// Partners (stream B): none, lut (the same variant), opq_glds (mivq_opq_rotate_prepared at
// d = 768: round 2 ran split_x + the LDS-DMA GEMM there; HEAD runs the register-staged GEMM),
// opq_split (d = 776: the register-staged GEMM),
// pq_encode, adc_search, and synthetic LDS streamers: dma16 (global_load_lds_dwordx4), dma4
// (global_load_lds_dword), regstage (global_load_dwordx4 + ds_write_b128), dma_mfma (LDS DMA
// overlapped with MFMAs: the minimal trigger).  Round-2 results (glds GEMM alone vs split_x
// alone) are in profiles/r03_s1_lut_stress3_*.log.
// Extra victim: regpk (a packed-fp32 chain on registers only).
// Prints, per (variant, partner), the number of LUT launches checked, the number with a
// mismatch, and a histogram of the mismatching runs by (k mod 64) start and length.
//
// Build:  hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/probes/lut_stress.hip \
//           -Ivector-quantization_amd/csrc -Iinclude -Lvector-quantization_amd/lib -lmivq \
//           -Wl,-rpath,'$ORIGIN/../../vector-quantization_amd/lib' -o tools/probes/lut_stress
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "mivq.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)
#define CM(x)                                                                          \
    do {                                                                               \
        int r_ = (x);                                                                  \
        if (r_ != 0) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, mivq_last_error()); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int kLutQ = 32;

// mode 0: v4f loads (round-2 form), 1: dword loads
template <int MODE>
__global__ __launch_bounds__(256) void lut_kernel(const float* __restrict__ q, int64_t nq, int d, int M, int ksub,
                                                  int dsub, const float* __restrict__ C, float* __restrict__ lut) {
    extern __shared__ __attribute__((aligned(16))) float qs[];
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
    auto step = [&](float c0, float c1, float c2, float c3, int t0, int nt) __attribute__((always_inline)) {
#pragma unroll
        for (int qq = 0; qq < kLutQ; ++qq) {
            const float* qr = qs + qq * dsub + t0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float cj = j == 0 ? c0 : j == 1 ? c1 : j == 2 ? c2 : c3;
                if (j < nt) {
                    const float df = __fsub_rn(qr[j], cj);
                    acc[qq] = __builtin_fmaf(df, df, acc[qq]);
                }
            }
        }
    };
    if constexpr (MODE == 3) {
        // dword loads, math forced onto packed fp32 ops (two queries per v_pk_* instruction)
        typedef float v2f __attribute__((ext_vector_type(2)));
        v2f acc2[kLutQ / 2];
#pragma unroll
        for (int i = 0; i < kLutQ / 2; ++i) acc2[i] = v2f{0.0f, 0.0f};
        for (int t0 = 0; t0 < dsub; t0 += 4) {
            const float cc[4] = {c[t0], c[t0 + 1], c[t0 + 2], c[t0 + 3]};
#pragma unroll
            for (int i = 0; i < kLutQ / 2; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const v2f qv = v2f{qs[(2 * i) * dsub + t0 + j], qs[(2 * i + 1) * dsub + t0 + j]};
                    const v2f df = qv - v2f{cc[j], cc[j]};
                    acc2[i] = __builtin_elementwise_fma(df, df, acc2[i]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kLutQ / 2; ++i) { acc[2 * i] = acc2[i].x; acc[2 * i + 1] = acc2[i].y; }
    } else if constexpr (MODE == 2) {
        // v4f loads, scalar math (an empty asm per chain step keeps the SLP vectorizer from
        // pairing two queries into one packed instruction)
        v4f cur = *reinterpret_cast<const v4f*>(c);
        for (int t0 = 0; t0 < dsub; t0 += 4) {
            const v4f nxt = (t0 + 4 < dsub) ? *reinterpret_cast<const v4f*>(c + t0 + 4) : cur;
#pragma unroll
            for (int qq = 0; qq < kLutQ; ++qq) {
                const float* qr = qs + qq * dsub + t0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float df = __fsub_rn(qr[j], cur[j]);
                    acc[qq] = __builtin_fmaf(df, df, acc[qq]);
                    asm volatile("" : "+v"(acc[qq]));
                }
            }
            cur = nxt;
        }
    } else if constexpr (MODE == 0) {
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
        if (qq < nqb) lut[((q0 + qq) * M + m) * ksub + k] = acc[qq];
}

// Register-only packed-fp32 victim: no LDS reads and no loads in the chain; each lane of
// block (m, qb) writes the same output layout as the LUT kernel.
__global__ __launch_bounds__(256) void regpk_kernel(int M, float* __restrict__ out) {
    typedef float v2f __attribute__((ext_vector_type(2)));
    const int m = blockIdx.x, k = threadIdx.x;
    v2f acc[kLutQ / 2];
#pragma unroll
    for (int i = 0; i < kLutQ / 2; ++i) acc[i] = v2f{1e-3f * (float)(k + i), 1e-3f * (float)(m + i + 1)};
    for (int t = 0; t < 96; ++t) {
        const v2f b = v2f{0.999f - 1e-5f * (float)t, 0.998f + 1e-6f * (float)k};
#pragma unroll
        for (int i = 0; i < kLutQ / 2; ++i) acc[i] = __builtin_elementwise_fma(acc[i], b, v2f{1e-4f, 2e-4f});
    }
#pragma unroll
    for (int i = 0; i < kLutQ / 2; ++i) {
        const int64_t q0 = (int64_t)blockIdx.y * kLutQ;
        out[((q0 + 2 * i) * M + m) * 256 + k] = acc[i].x;
        out[((q0 + 2 * i + 1) * M + m) * 256 + k] = acc[i].y;
    }
}

// Synthetic partners: 256-thread workgroups streaming a buffer into 64 KiB of LDS, either by
// LDS DMA (SIZE 16: global_load_lds_dwordx4, SIZE 4: global_load_lds_dword) or through
// registers (SIZE 0: global_load_dwordx4 + ds_write_b128).
template <int SIZE>
__global__ __launch_bounds__(256) void dma_partner_kernel(const float* __restrict__ src, int64_t nsrc, int iters,
                                                          float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef __attribute__((address_space(3))) void lds_void;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    float s = 0.0f;
    for (int it = 0; it < iters; ++it) {
        const int64_t base = (((int64_t)blockIdx.x * iters + it) * 16384) % (nsrc - 16384);
        if constexpr (SIZE == 16) {
#pragma unroll
            for (int i = 0; i < 16; ++i)  // 4 waves x 16 x 1 KiB = 64 KiB
                __builtin_amdgcn_global_load_lds((const void*)(src + base + (w * 16 + i) * 256 + l * 4),
                                                 (lds_void*)(lds + (w * 16 + i) * 1024), 16, 0, 0);
        } else if constexpr (SIZE == 4) {
#pragma unroll 8
            for (int i = 0; i < 64; ++i)  // 4 waves x 64 x 256 B = 64 KiB
                __builtin_amdgcn_global_load_lds((const void*)(src + base + (w * 64 + i) * 64 + l),
                                                 (lds_void*)(lds + (w * 64 + i) * 256), 4, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const v4f v = *reinterpret_cast<const v4f*>(src + base + (w * 16 + i) * 256 + l * 4);
                *reinterpret_cast<v4f*>(lds + (w * 16 + i) * 1024 + l * 16) = v;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        s += reinterpret_cast<const float*>(lds)[(tid * 67 + it) & 16383];
        __syncthreads();
    }
    sink[(int64_t)blockIdx.x * 256 + tid] = s;
}

// DMA + MFMA: each wave streams 16 KiB into LDS by global_load_lds_dwordx4 while it runs a
// chain of v_mfma_f32_32x32x16_f16 on register operands.
__global__ __launch_bounds__(256) void dma_mfma_partner_kernel(const float* __restrict__ src, int64_t nsrc, int iters,
                                                               float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef __attribute__((address_space(3))) void lds_void;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    typedef float floatx16 __attribute__((ext_vector_type(16)));
    half8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.001f * (l + i)); b[i] = (_Float16)(0.002f * (l - i)); }
    floatx16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;
    for (int it = 0; it < iters; ++it) {
        const int64_t base = (((int64_t)blockIdx.x * iters + it) * 16384) % (nsrc - 16384);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src + base + (w * 16 + i) * 256 + l * 4),
                                             (lds_void*)(lds + (w * 16 + i) * 1024), 16, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[j], 0, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        a[0] += (_Float16)reinterpret_cast<const float*>(lds)[(tid * 67 + it) & 16383];
        __syncthreads();
    }
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) s += acc[j][e];
    sink[(int64_t)blockIdx.x * 256 + tid] = s;
}

static void launch_partner_dma(int size, const float* src, int64_t nsrc, float* sink, hipStream_t s) {
    const dim3 grid(1024), block(256);
    if (size == 16) hipLaunchKernelGGL(dma_partner_kernel<16>, grid, block, 65536, s, src, nsrc, 64, sink);
    else if (size == 4) hipLaunchKernelGGL(dma_partner_kernel<4>, grid, block, 65536, s, src, nsrc, 64, sink);
    else if (size == 0) hipLaunchKernelGGL(dma_partner_kernel<0>, grid, block, 65536, s, src, nsrc, 64, sink);
    else hipLaunchKernelGGL(dma_mfma_partner_kernel, grid, block, 65536, s, src, nsrc, 64, sink);
    CK(hipGetLastError());
}

__global__ void fill_kernel(float* p, int64_t n, uint32_t seed, float scale) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * scale;
}

struct Data {
    int n, d, M, dsub, nq;
    float *X, *C, *A, *Y, *lutp;
    void *oprep, *owork, *pprep, *pwork, *swork;
    size_t owb, pwb, swb;
    uint8_t* codes;
    float* sd;
    uint32_t* si;
};

static Data make(int n, int d, int M, uint32_t seed) {
    Data D{};
    D.n = n; D.d = d; D.M = M; D.dsub = d / M; D.nq = 64;
    CK(hipMalloc(&D.X, (size_t)n * d * 4));
    CK(hipMalloc(&D.C, (size_t)d * 256 * 4));
    CK(hipMalloc(&D.A, (size_t)d * d * 4));
    CK(hipMalloc(&D.Y, (size_t)n * d * 4));
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)(((int64_t)n * d + 255) / 256)), dim3(256), 0, 0, D.X, (int64_t)n * d, seed, 0.07f);
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((d * 256 + 255) / 256)), dim3(256), 0, 0, D.C, (int64_t)d * 256, seed + 1, 0.07f);
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)(((int64_t)d * d + 255) / 256)), dim3(256), 0, 0, D.A, (int64_t)d * d, seed + 2, 0.1f);
    CK(hipDeviceSynchronize());
    if (d % 8 == 0) {
        CK(hipMalloc(&D.oprep, mivq_opq_prep_bytes(d)));
        CM(mivq_opq_prepare(D.A, d, 0, D.oprep, nullptr));
        D.owb = mivq_opq_rotate_workspace_bytes(n, d);
        CK(hipMalloc(&D.owork, D.owb));
    }
    if (d % M == 0) {
        CK(hipMalloc(&D.pprep, mivq_pq_prep_bytes(d, M, 8)));
        CM(mivq_pq_prepare(D.C, d, M, 8, D.pprep, nullptr));
        D.pwb = mivq_pq_encode_workspace_bytes(n, d, M, 8);
        CK(hipMalloc(&D.pwork, D.pwb));
        CK(hipMalloc(&D.codes, (size_t)n * M));
        CM(mivq_pq_encode(D.X, n, d, M, 8, D.C, D.pprep, D.pwork, D.pwb, D.codes, 0, nullptr));
        CK(hipMalloc(&D.lutp, (size_t)D.nq * M * 256 * 4));
        CM(mivq_adc_lut(D.X, D.nq, d, M, 8, D.C, 0, D.lutp, nullptr));
        D.swb = mivq_adc_search_workspace_bytes(D.nq, n, M, 8, 10);
        CK(hipMalloc(&D.swork, D.swb));
        CK(hipMalloc(&D.sd, D.nq * 10 * 4));
        CK(hipMalloc(&D.si, D.nq * 10 * 4));
    }
    CK(hipDeviceSynchronize());
    return D;
}

static void launch_lut(int variant, const Data& D, float* out, hipStream_t s) {
    const size_t smem = (size_t)kLutQ * D.dsub * 4;
    const dim3 grid((unsigned)D.M, (unsigned)((D.nq + kLutQ - 1) / kLutQ));
    if (variant == 3)
        hipLaunchKernelGGL(lut_kernel<2>, grid, dim3(256), smem, s, D.X, (int64_t)D.nq, D.d, D.M, 256, D.dsub, D.C, out);
    else if (variant == 4)
        hipLaunchKernelGGL(lut_kernel<3>, grid, dim3(256), smem, s, D.X, (int64_t)D.nq, D.d, D.M, 256, D.dsub, D.C, out);
    else if (variant == 5)
        hipLaunchKernelGGL(regpk_kernel, grid, dim3(256), 0, s, D.M, out);
    else if (variant == 0)
        hipLaunchKernelGGL(lut_kernel<0>, grid, dim3(256), smem, s, D.X, (int64_t)D.nq, D.d, D.M, 256, D.dsub, D.C, out);
    else if (variant == 1)
        hipLaunchKernelGGL(lut_kernel<1>, grid, dim3(256), smem, s, D.X, (int64_t)D.nq, D.d, D.M, 256, D.dsub, D.C, out);
    else
        CM(mivq_adc_lut(D.X, D.nq, D.d, D.M, 8, D.C, 0, out, s));
    CK(hipGetLastError());
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const int reps = 16;  // LUT launches per iteration, each into its own buffer
    // main data set (d = 768, M = 8, dsub = 96: the concurrency test's shape)
    Data D = make(60000, 768, 8, 11u);
    Data E = make(60000, 776, 8, 21u);  // d % 32 != 0: register-staged OPQ GEMM
    const size_t lut_elems = (size_t)D.nq * D.M * 256;
    std::vector<float*> outs(reps);
    for (auto& o : outs) CK(hipMalloc(&o, lut_elems * 4));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    std::vector<float> ref(lut_elems), got(lut_elems);
    const char* vnames[6] = {"v4f", "dword", "lib", "v4f_scalar", "dword_pk", "regpk"};
    const char* pnames[12] = {"none", "lut", "opq_glds", "opq_split", "pq_encode", "adc_search", "dma16", "dma4", "regstage", "-", "-", "dma_mfma"};
    float* sink;
    CK(hipMalloc(&sink, 1024 * 256 * 4));
    CK(hipFuncSetAttribute((const void*)dma_mfma_partner_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    for (int sz : {16, 4, 0}) CK(hipFuncSetAttribute(sz == 16 ? (const void*)dma_partner_kernel<16> : sz == 4 ? (const void*)dma_partner_kernel<4> : (const void*)dma_partner_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    int only_v = -1, only_p = -1;
    if (argc > 2) only_v = atoi(argv[2]);
    if (argc > 3) only_p = atoi(argv[3]);
    for (int v = 0; v < 6; ++v) {
        if (only_v >= 0 && v != only_v) continue;
        launch_lut(v, D, outs[0], sa);
        CK(hipStreamSynchronize(sa));
        CK(hipMemcpy(ref.data(), outs[0], lut_elems * 4, hipMemcpyDeviceToHost));
        for (int p = 0; p < 12; ++p) {
            if ((only_p >= 0 && p != only_p) || pnames[p][0] == '-') continue;
            long checked = 0, bad = 0, badel = 0;
            std::map<std::string, long> hist;
            for (int it = 0; it < iters; ++it) {
                for (auto& o : outs) CK(hipMemsetAsync(o, 0xFF, lut_elems * 4, sa));
                CK(hipStreamSynchronize(sa));
                // partner first (it runs long), then the LUT launches on the other stream
                switch (p) {
                    case 0: break;
                    case 1: for (int r = 0; r < 8; ++r) launch_lut(v, D, D.lutp, sb); break;
                    case 2: CM(mivq_opq_rotate_prepared(D.X, D.n, D.d, D.oprep, D.owork, D.owb, D.Y, sb)); break;
                    case 3: CM(mivq_opq_rotate_prepared(E.X, E.n, E.d, E.oprep, E.owork, E.owb, E.Y, sb)); break;
                    case 4: CM(mivq_pq_encode(D.X, D.n, D.d, D.M, 8, D.C, D.pprep, D.pwork, D.pwb, D.codes, 0, sb)); break;
                    case 5:
                        for (int r = 0; r < 4; ++r)
                            CM(mivq_adc_search(D.lutp, D.nq, D.codes, D.n, D.M, 8, 10, 0, D.swork, D.swb, D.sd, D.si, sb));
                        break;
                    case 6: launch_partner_dma(16, E.Y, (int64_t)E.n * E.d, sink, sb); break;
                    case 7: launch_partner_dma(4, E.Y, (int64_t)E.n * E.d, sink, sb); break;
                    case 8: launch_partner_dma(0, E.Y, (int64_t)E.n * E.d, sink, sb); break;
                    case 11: launch_partner_dma(1, E.Y, (int64_t)E.n * E.d, sink, sb); break;
                }
                for (int r = 0; r < reps; ++r) launch_lut(v, D, outs[r], sa);
                CK(hipStreamSynchronize(sa));
                CK(hipStreamSynchronize(sb));
                for (int r = 0; r < reps; ++r) {
                    CK(hipMemcpy(got.data(), outs[r], lut_elems * 4, hipMemcpyDeviceToHost));
                    ++checked;
                    bool any = false;
                    for (size_t i = 0; i < lut_elems;) {
                        if (memcmp(&got[i], &ref[i], 4) == 0) { ++i; continue; }
                        size_t j = i;
                        while (j < lut_elems && memcmp(&got[j], &ref[j], 4) != 0) ++j;
                        any = true;
                        badel += (long)(j - i);
                        const int k0 = (int)(i % 256), q = (int)(i / (256 * D.M)), m = (int)((i / 256) % D.M);
                        char key[96];
                        snprintf(key, sizeof key, "kmod64=%d len=%zu", k0 % 64, j - i);
                        hist[key]++;
                        if (bad < 4 && hist.size() < 8)
                            fprintf(stdout, "  span q=%d m=%d k=%d..%zu got %.6g want %.6g\n", q, m, k0, k0 + (j - i) - 1,
                                    got[i], ref[i]);
                        i = j;
                    }
                    if (any) ++bad;
                }
            }
            printf("variant=%s partner=%s checked=%ld bad=%ld bad_elems=%ld\n", vnames[v], pnames[p], checked, bad, badel);
            for (auto& kv : hist) printf("    %s : %ld\n", kv.first.c_str(), kv.second);
            fflush(stdout);
        }
    }
    return 0;
}
