#!/bin/bash
# round-4 session 20: dsub 64 single-accumulator round-4 loop in-tree -- parity, A/B against the
# session-8 build (libmivq_r04b.so), then the PMC traffic passes of the final sources
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_r04b.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/libmivq_r04b.so --reps 10" || exit $?
bash tools/pmc_traffic.sh
