#!/bin/bash
# round-5 session 21: integer ADC scan addressing by SDWA byte-select shifts (one op per lookup):
# ADC tests, then interleaved A/B against the unrolled build of session 20
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py -m gpu -q -x -rf -k 'adc or filtered' --timeout 300 --timeout-method thread" \
  "python -u tools/ab_lib.py $L/libmivq_qsunroll.so --what adc --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_qsunroll.so --what adc --M 32 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_qsunroll.so --what adc --n 6650000 --d 1024 --reps 4"
