#!/bin/bash
# round-4 session 9: fixed per-step store count in the filter tail (tools/build/fixst.so,
# MIVQ_CS_FIXED_STORES=1) -- its parity tests first (MIVQ_LIB), then A/Bs against the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/fixst.so python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10 --M 32" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 10 --M 8" \
  "python tools/ab_lib.py tools/build/fixst.so --reps 4 --n 10000000"
