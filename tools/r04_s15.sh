#!/bin/bash
# round-4 session 15: RaBitQ-1 encode with batched loads (in-tree) vs the generic loop (rq_old.so);
# SQ-8 with 8 rows of loads in flight per wave (sqd8.so) vs 4 (in-tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_sweep_gpu.py -m gpu -q -x -k 'rabitq or sq' --timeout 120 --timeout-method thread" \
  "MIVQ_LIB=$PWD/tools/build/sqd8.so python -u -m pytest tests/test_kernels_gpu.py tests/test_golden_wide.py -m gpu -q -x -k 'sq' --timeout 120 --timeout-method thread" \
  "python tools/ab_stream.py tools/build/rq_old.so --kind rabitq1 --reps 10" \
  "python tools/ab_stream.py tools/build/rq_old.so --kind rabitq1 --reps 10" \
  "python tools/ab_stream.py tools/build/sqd8.so --kind sq8 --reps 10" \
  "python tools/ab_stream.py tools/build/sqd8.so --kind sq8 --reps 10"
