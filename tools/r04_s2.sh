#!/bin/bash
# round-4 session 2: fixed tests, filter variants, PC sampling and counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_golden_wide.py tests/test_opq_gpu.py tests/test_concurrency_gpu.py tests/test_kernels_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_g8.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_prio.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_xaux0.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_r03.so --what adc --reps 6" \
  "bash tools/pcsample.sh r04s2" \
  "bash tools/pmc.sh r04s2"
