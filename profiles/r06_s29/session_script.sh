#!/bin/bash
# round 6 session 29: estimator dense first block of 4096 / 16384 codes vs 8192 (default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/probe_rq.py $A/libmivq_f4096.so --reps 9" \
  "python tools/probe_rq.py $A/libmivq_f16384.so --reps 9" \
  "python tools/probe_rq.py $A/libmivq_f4096.so --nq 10000 --n 1000000 --d 1024 --reps 3" \
  "python tools/probe_rq.py $A/libmivq_f4096.so --nq 100 --n 1000000 --d 3072 --reps 7"
