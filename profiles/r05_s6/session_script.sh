#!/bin/bash
# round-5 session 6: filtered ADC tests (NaN hook), u8-entry table A/B, then session 5's items
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "MIVQ_LIB=$PWD/vector-quantization_amd/lib/ab/libmivq_adce8.so python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_adce8.so --what adc --reps 8" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_adce8.so --what adc --reps 8 --M 32" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_adce8.so --what adc --reps 3 --n 6650000 --d 1024 --nq 10000" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_res2.so --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_0.so --M 32 --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_1.so --M 32 --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_16.so --M 32 --reps 6" \
  "python -u -m pytest tests/test_sharded_gpu.py tests/test_opq_gpu.py tests/test_sweep_gpu.py tests/test_quantizers_gpu.py tests/test_export_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread"
