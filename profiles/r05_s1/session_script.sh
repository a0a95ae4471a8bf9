#!/bin/bash
# round-5 session 1: slice pipeline (filter on two streams, resolve on a high-priority stream)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k 'pq_encode' --timeout 120 --timeout-method thread" \
  "python -u tools/probe_pipe.py --n 1000000 --cfg base:PIPE=0 --cfg s2:SLICES=2 --cfg s3:SLICES=3 --cfg s4:SLICES=4 --cfg s8:SLICES=8" \
  "python -u tools/probe_pipe.py --n 10000000 --reps 5 --cfg base:PIPE=0 --cfg p2m:SLICE_ROWS=2097152 --cfg p1m:SLICE_ROWS=1048576 --cfg p512k:SLICE_ROWS=524288"
