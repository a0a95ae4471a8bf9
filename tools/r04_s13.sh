#!/bin/bash
# round-4 session 13: erq_rotate_fast_kernel (16-B range-checked loads two slices ahead) vs the
# generic kernel with the same tile order (erq_slow.so) and the round-3 build (erq_r3.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py tests/test_golden_wide.py tests/test_opq_gpu.py -m gpu -q -x -k 'extrabitq or polar or opq_train' --timeout 120 --timeout-method thread" \
  "python tools/ab_erq.py tools/build/erq_slow.so --reps 6" \
  "python tools/ab_erq.py tools/build/erq_r3.so --reps 6" \
  "python tools/ab_erq.py tools/build/erq_slow.so --reps 6 --n 100000 --d 1024"
