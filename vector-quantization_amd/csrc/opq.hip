// opq.hip — OPQ rotation as an fp32 MFMA GEMM on gfx950.
//
// Replaces faiss.OPQMatrix.apply / reverse_transform used by OptimizedProductQuantizer
// (/root/reference/src/haag_vq/methods/optimized_product_quantization.py:26,31,34):
//   transpose == 0 : y = x . A^T   (LinearTransform::apply, A is d_out x d_in row-major)
//   transpose == 1 : y = x . A     (reverse_transform of an orthonormal A)
// The rotation is a genuine dense contraction, so it runs on the matrix cores in exact
// f32 (v_mfma_f32_32x32x2_f32: each instruction is a k-ordered fmaf chain, no reduced
// precision).  128x128 output tile per 256-thread workgroup, 2x2 32x32 tiles per wave,
// BK = 16 slices of x and A staged through LDS (k-major so every fragment read is a
// contiguous, conflict-free 128-B row).
//
// mivq_opq_rotate itself runs the library fp32 GEMM (rocBLAS sgemm on the caller's stream,
// 147 TFLOP/s at 1M x 1536 against 56 for opq_gemm_kernel — tools/dbg/gemm_probe.py): the
// rotation is a plain GEMM with nothing to fuse.  MIVQ_OPQ_NATIVE_GEMM=1 selects the kernel
// below instead; it also serves when rocBLAS reports an error.
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "mivq_common.h"

namespace mivq {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

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
        // x tile: 128 rows x 16 k = 2048 floats, 8 per thread
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + q * 256;
            const int i = e >> 4, kk = e & 15;
            const int64_t row = r0 + i;
            xs[kk][i] = (row < n && k0 + kk < d) ? x[row * d + k0 + kk] : 0.0f;
        }
        // B tile: 16 k x 128 cols
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

}  // namespace
}  // namespace mivq

namespace mivq {
namespace {

// One rocBLAS handle per device, created on first use and kept for the process.
rocblas_handle blas_handle() {
    static std::mutex mu;
    static std::map<int, rocblas_handle> handles;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto it = handles.find(dev);
    if (it != handles.end()) return it->second;
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) return nullptr;
    handles[dev] = h;
    return h;
}

// y (n x d, row-major) = x . A^T (transpose 0) or x . A (transpose 1).  Column-major view:
// Y^T = op(A_cm) . X^T with A_cm = A^T as stored, so op = T for x . A^T and N for x . A.
bool rotate_blas(const float* x, int64_t n, int d, const float* A, int transpose, float* y, hipStream_t st) {
    static const bool native = [] {
        const char* e = std::getenv("MIVQ_OPQ_NATIVE_GEMM");
        return e && e[0] == '1';
    }();
    if (native) return false;
    rocblas_handle h = blas_handle();
    if (!h || rocblas_set_stream(h, st) != rocblas_status_success) return false;
    const float one = 1.0f, zero = 0.0f;
    const int64_t step = (int64_t)1 << 30;  // rocblas_int columns per call
    for (int64_t r = 0; r < n; r += step) {
        const int cols = (int)std::min<int64_t>(step, n - r);
        if (rocblas_sgemm(h, transpose ? rocblas_operation_none : rocblas_operation_transpose, rocblas_operation_none,
                          d, cols, d, &one, A, d, x + r * d, d, &zero, y + r * d, d) != rocblas_status_success)
            return false;
    }
    return true;
}

}  // namespace
}  // namespace mivq

using namespace mivq;

extern "C" int mivq_opq_rotate(const float* x, int64_t n, int32_t d, const float* A, int32_t transpose, float* y,
                               void* stream) {
    MIVQ_REQUIRE(n >= 0 && d > 0, MIVQ_ERR_INVALID, "opq_rotate: bad sizes n=%lld d=%d", (long long)n, d);
    MIVQ_REQUIRE(transpose == 0 || transpose == 1, MIVQ_ERR_INVALID, "opq_rotate: transpose must be 0 or 1");
    if (n == 0) return MIVQ_OK;
    MIVQ_REQUIRE(x && A && y && x != y, MIVQ_ERR_INVALID, "opq_rotate: null or aliased pointer");
    if (mivq::rotate_blas(x, n, d, A, transpose, y, as_stream(stream))) return check_launch("opq_rotate (rocBLAS)");
    const dim3 grid((unsigned)ceil_div(n, BM), (unsigned)ceil_div(d, BN));
    hipLaunchKernelGGL(opq_gemm_kernel, grid, dim3(256), 0, as_stream(stream), x, n, d, A, transpose, y);
    return check_launch("opq_rotate");
}
