#!/bin/bash
# round-4 session 25: stage-first loop in erq_rotate_fast_kernel (tools/build/erq_sf.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/erq_sf.so python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py tests/test_golden_wide.py -m gpu -q -x -k extrabitq --timeout 120 --timeout-method thread" \
  "python tools/ab_erq.py tools/build/erq_sf.so --reps 6" \
  "python tools/ab_erq.py tools/build/erq_sf.so --reps 6 --n 100000 --d 1024"
