#!/bin/bash
# round 6 session 24: qscan pinned prefetch chosen by shape (default) vs never (pin0) / always
# (pin1), several shapes; ids and distances compared
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/ab_lib.py $A/libmivq_pin0.so --what adc --reps 10" \
  "python tools/ab_lib.py $A/libmivq_pin1.so --what adc --reps 10" \
  "python tools/ab_lib.py $A/libmivq_pin0.so --what adc --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python tools/ab_lib.py $A/libmivq_pin1.so --what adc --n 6650000 --d 1024 --nq 1000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_pin0.so --what adc --n 6650000 --d 1024 --nq 1000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_pin0.so --what adc --nq 4000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_pin1.so --what adc --nq 4000 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_pin0.so --what adc --M 32 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_pin1.so --what adc --M 32 --reps 5"
