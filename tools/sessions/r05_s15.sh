#!/bin/bash
# round-5 session 15: OPQ split GEMM, d % 32 == 0 path with scalar k offsets and packed split
# (tests + interleaved A/B against the session-14 build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_opq_gpu.py tests/test_concurrency_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/ab_opq.py vector-quantization_amd/lib/libmivq.so vector-quantization_amd/lib/ab/libmivq_opq_base.so --reps 10" \
  "python -u tools/ab_opq.py vector-quantization_amd/lib/ab/libmivq_opq_base.so vector-quantization_amd/lib/libmivq.so --reps 10"
