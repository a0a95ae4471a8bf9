#!/bin/bash
# round 6 session 28: estimator query staging with both halves loaded at the step's start and
# stored at its end (full) -- A/B against the default (half-step staging)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/probe_rq.py $A/libmivq_full.so --reps 7" \
  "python tools/probe_rq.py $A/libmivq_full.so --nq 10000 --n 1000000 --d 1024 --reps 3" \
  "python tools/probe_rq.py $A/libmivq_full.so --nq 200 --n 1000000 --d 3072 --reps 5"
