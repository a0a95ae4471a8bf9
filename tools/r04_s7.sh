#!/bin/bash
# round-4 session 7: dsub 64 back on the exact round-3 tail; OPQ GEMM non-temporal x / B loads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_xnt.so tools/build/opq_bnt.so --reps 6"
