#!/bin/bash
# round 6 session 4: ADC (packed LUT, pipelined rerank, short qscan epilogue, buffer code fetch)
# vs HEAD's ADC source (lib/ab/libmivq_head.so); ADC tests; kernel split; default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py tests/test_abi.py tests/test_concurrency_gpu.py tests/test_pinning_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_head.so --what adc --reps 10" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_head.so --what adc --reps 10 --M 32" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_head.so --what adc --reps 5 --n 6650000 --d 1024 --nq 10000" \
  "bash tools/adc_split.sh 1m" \
  "bash tools/adc_split.sh c5 --n 6650000 --d 1024 --nq 10000" \
  "python -u bench.py"
