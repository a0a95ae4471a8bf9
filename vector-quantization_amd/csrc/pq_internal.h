// pq_internal.h — kernels of pq_encode_cs.hip dispatched from pq.hip.
#pragma once

#include "mivq_common.h"

namespace mivq {

// Dynamic LDS bytes of the codebook-stationary encode for KS k-steps and dsub.
int cs_smem_bytes(int KS, int dsub);

// Bytes of the per-workgroup list counts of launch_pq_encode_cs.
size_t cs_counts_bytes(int64_t n, int M);

// Codebook-stationary fp16-MFMA encode with exact re-check (KS in 1..12).  Writes the
// transposed codes into codesT (M, n) and then the (n, M) byte codes into `codes`; `items`
// is scratch for n*M uint2 (the rows the filter could not settle alone), `counts` for
// cs_counts_bytes(n, M).  pd / bnd2: the prep buffer's pair spreads and pair-window terms (pd
// may be null: no pair window).
hipError_t launch_pq_encode_cs(int KS, const float* x, int64_t n, int d, int M, int dsub, const float* C,
                               const float* cn, const void* img, const float* hinit, const void* bnd, const void* pd,
                               const void* bnd2, uint8_t* codesT, void* items, void* counts, uint8_t* codes,
                               hipStream_t st);

}  // namespace mivq
