#!/bin/bash
# round 6 session 35: even-query unpack as an SGPR-mask v_and (32-bit) instead of a v_perm -- A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python tools/ab_lib.py $A/libmivq_andlo0.so --what adc --reps 10" \
  "python tools/ab_lib.py $A/libmivq_andlo0.so --what adc --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python tools/ab_lib.py $A/libmivq_andlo0.so --what adc --M 32 --reps 10" \
  "python tools/ab_lib.py $A/libmivq_andlo0.so --what adc --M 32 --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python tools/ab_lib.py $A/libmivq_keys2.so --what adc --reps 10" \
  "python tools/ab_lib.py $A/libmivq_keys2.so --what adc --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py -k 'adc or qscan' -q -x --timeout 120 --timeout-method thread"
