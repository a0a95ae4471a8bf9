// mivq_common.h — shared helpers for the libmivq HIP sources (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

#include "../../include/mivq.h"

namespace mivq {

// ---------------------------------------------------------------- errors
// Per-thread error string behind mivq_last_error() (declared in mivq.h).
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Returns MIVQ_ERR_HIP with the launch error if the last launch failed.
int check_launch(const char* what);

// CU count of the current device, cached per (thread, device) (pq_encode_cs.hip).
int device_cus();

#define MIVQ_REQUIRE(cond, code, ...)                          \
    do {                                                       \
        if (!(cond)) return ::mivq::set_error((code), __VA_ARGS__); \
    } while (0)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---------------------------------------------------------------- PQ prep layout
// The derived codebook data built by mivq_pq_prepare, as byte offsets into one buffer:
//   cn    : (M, ksub)           f32  canonical ||c||^2 (sequential fmaf chain)
//   ct    : (M, dsub, ksub)     f32  transposed codebook for the exact / LUT kernels
//   img   : (M, 8 cb, KS, 64 lanes, 8 halves) f16 MFMA A-operand image (ksub == 256,
//           dsub padded to KS*16), see pq_encode.hip
//   hinit : (M, ksub)           f32  -||c||^2 / 2 * scale^2 (MFMA accumulator init)
//   bnd   : (M, 4)              f32  {sigma, a, b, tau}: scales and the filter window W = a Xs + b
//   spread: (M, 2)              u32  bits of Dmax, DDmax (pairwise spreads of the image)
//   pd    : (M, 256, 256)       f32x2 per centroid pair {||c~_i - c~_j||, ||dc_i - dc_j||} (rounded
//           up) for the pair window of the resolve kernel; only when M <= kPdMaxM
//   bnd2  : (M, 4)              f32  {a_rest, b_rest, eta', 0}: the pair window's other terms
constexpr int kPdMaxM = 64;  // pair-distance tables are kept for up to 64 subspaces (32 MiB)

struct PqPrepLayout {
    size_t cn, ct, img, hinit, bnd, spread, pd, bnd2, total;
    int32_t dsub, ksub, ks;  // ks = padded dsub / 16 (k-steps of the f16 MFMA)
    bool mfma;               // filter path available for this shape
};

inline PqPrepLayout pq_prep_layout(int32_t d, int32_t M, int32_t nbits) {
    PqPrepLayout L{};
    L.dsub = d / M;
    L.ksub = 1 << nbits;
    L.ks = (L.dsub + 15) / 16;
    L.mfma = (L.ksub == 256) && (L.ks <= 16);
    size_t off = 0;
    L.cn = off;    off = align_up(off + sizeof(float) * (size_t)M * L.ksub, 256);
    L.ct = off;    off = align_up(off + sizeof(float) * (size_t)M * L.dsub * L.ksub, 256);
    L.img = off;   off = align_up(off + (L.mfma ? (size_t)M * 8 * L.ks * 64 * 8 * 2 : 0), 256);
    L.hinit = off; off = align_up(off + sizeof(float) * (size_t)M * L.ksub, 256);
    L.bnd = off;   off = align_up(off + sizeof(float) * (size_t)M * 4, 256);
    L.spread = off; off = align_up(off + sizeof(uint32_t) * (size_t)M * 2, 256);
    L.pd = off;     off = align_up(off + ((L.mfma && M <= kPdMaxM) ? (size_t)M * 256 * 256 * 8 : 0), 256);
    L.bnd2 = off;   off = align_up(off + sizeof(float) * (size_t)M * 4, 256);
    L.total = off;
    return L;
}

inline int pq_code_size(int32_t M, int32_t nbits) { return (M * nbits + 7) / 8; }

}  // namespace mivq
