#!/bin/bash
# round-4 session 6: filter loop (pinned refill, in-step pair load, per-workgroup sigma loops;
# dsub 64 on the round-3 loop) -- parity, A/Bs against the session-4 build, 10M line, PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_pinning_gpu.py tests/test_golden_wide.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10 --M 32" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10 --M 8" \
  "python tools/ab_lib.py tools/build/libmivq_r04a.so --reps 10 --data clustered" \
  bench10m
