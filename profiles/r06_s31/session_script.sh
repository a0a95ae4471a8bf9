#!/bin/bash
# round 6 session 31: filtered-scan chunk rule (one-round grids: >= 4 chunks, <= 1024 steps per
# chunk) against the previous build (head); ADC GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_abi.py tests/test_kernels_gpu.py -k 'adc or abi or filtered' -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 5 --nq 2000" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 5 --nq 4000" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 3 --n 6650000 --d 1024 --nq 1000" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 5 --nq 1000" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 5 --nq 2000 --M 32"
