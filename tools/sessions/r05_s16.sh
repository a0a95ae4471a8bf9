#!/bin/bash
# round-5 session 16: OPQ split GEMM with the SIMD-partner stagger (waves 4..7 run a half-step of
# MFMAs before staging) -- tests + interleaved A/B against the same build without it and the
# session-14 build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_opq_gpu.py tests/test_concurrency_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/ab_opq.py $L/libmivq.so $L/ab/libmivq_opq_nostag.so $L/ab/libmivq_opq_base.so --reps 10" \
  "python -u tools/ab_opq.py $L/ab/libmivq_opq_base.so $L/ab/libmivq_opq_nostag.so $L/libmivq.so --reps 10"
