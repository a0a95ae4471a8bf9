#!/bin/bash
# round 6 session 26: ADC scan at twice the row chunks (nch2: two+ rounds of workgroups, pinned
# prefetch) vs the cost model's chunks -- more shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/ab_lib.py $A/libmivq_nch2.so --what adc --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python tools/ab_lib.py $A/libmivq_nch2.so --what adc --nq 2000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_nch2.so --what adc --n 2000000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_nch2.so --what adc --n 4000000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_nch2.so --what adc --n 6650000 --d 1024 --nq 3000 --reps 3"
