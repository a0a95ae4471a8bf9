#!/bin/bash
# round-4 session 8: dsub 64 round-3 loop with the per-block sigma branch restored
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10"
