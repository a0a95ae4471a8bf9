#!/bin/bash
# round-4 session 3: x-stream cache-policy variants, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python tools/ab_lib.py tools/build/libmivq_xaux3.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_xaux18.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_xaux19.so --reps 10" \
  "python bench.py"
