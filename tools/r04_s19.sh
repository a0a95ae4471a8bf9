#!/bin/bash
# round-4 session 19: dsub 64 (config #5 shape) on the round-4 loop with one accumulator
# (MIVQ_CS_NOPIPE: fits 16 waves' 128 VGPRs without spills) vs the in-tree round-3 loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/d64np.so python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k 'pq_encode' --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/d64np.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/d64np.so --reps 6 --n 6650000 --d 1024"
