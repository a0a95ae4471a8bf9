#!/bin/bash
# round-4 session 5: filter loop without the vmcnt(0) stalls (pair load inside the step,
# unconditional pinned refill, no sigma branch) -- parity first, then interleaved A/Bs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10 --M 32" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10 --M 8" \
  "python tools/ab_lib.py tools/build/pf128.so --reps 10" \
  "python tools/ab_lib.py tools/build/pdlate.so --reps 10" \
  "python tools/ab_lib.py tools/build/d64w12.so --reps 6 --n 6650000 --d 1024"
