#!/bin/bash
# round-4 session 28: fixed per-step store count with dsub 64 on the round-4 loop (fixst2.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/fixst2.so python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k pq_encode --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/fixst2.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/fixst2.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/fixst2.so --reps 10"
