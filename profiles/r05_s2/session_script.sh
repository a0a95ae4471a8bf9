#!/bin/bash
# round-5 session 2: slice pipeline variants (2: filters on one stream, resolve high priority;
# 3: filters on one stream, resolve on a normal-priority stream)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u tools/probe_pipe.py --n 1000000 --cfg base:PIPE=0 --cfg m2s2:PIPE=2,SLICES=2 --cfg m3s2:PIPE=3,SLICES=2 --cfg m2s4:PIPE=2,SLICES=4" \
  "python -u tools/probe_pipe.py --n 10000000 --reps 5 --cfg base:PIPE=0 --cfg m2:PIPE=2 --cfg m3:PIPE=3 --cfg m2r1m:PIPE=2,SLICE_ROWS=1048576"
