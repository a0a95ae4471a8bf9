#!/bin/bash
# round 6 session 34: M = 32 scan with the code rows from buffer loads (pinned kernel) -- A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/ab_lib.py $A/libmivq_m32buf.so --what adc --M 32 --reps 10" \
  "python tools/ab_lib.py $A/libmivq_m32buf.so --what adc --M 32 --nq 4000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_m32buf.so --what adc --M 32 --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python tools/ab_lib.py $A/libmivq_m32buf.so --what adc --reps 5"
