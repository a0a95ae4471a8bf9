#!/bin/bash
# round-4 session 9: (a) fixed per-step store count in the filter tail (tools/build/fixst.so,
# MIVQ_CS_FIXED_STORES=1); (b) conflict-free staging-store order in the OPQ GEMM
# (tools/build/opq_wswz.so, MIVQ_OPQ_WSWZ=1) -- each variant's parity tests first (MIVQ_LIB),
# then interleaved A/Bs against the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/fixst.so python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10 --M 32" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10 --M 8" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 4 --n 10000000" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/d64w12f.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/xcdm.so --reps 10" \
  "python tools/ab_lib.py tools/build/xcdm.so --reps 6 --n 6650000 --d 1024" \
  "MIVQ_LIB=$PWD/tools/build/opq_wswz.so python -u -m pytest tests/test_opq_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_wswz.so --reps 6"
