#!/bin/bash
# round-5 session 4: filtered ADC (tests + timing), the pruned encode file (bit-exact tests and
# interleaved A/Bs: pre-prune build, resolve A operands per wave, direct (n, M) code stores)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/probe_adc.py" \
  "python -u tools/probe_adc.py --M 32" \
  "python -u tools/probe_adc.py --n 6650000 --d 1024 --nq 10000 --reps 4" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_pre_prune.so --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_res1.so --reps 8" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_direct.so --reps 8" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_direct_res1.so --reps 8" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_direct_res1.so --reps 3 --n 10000000"
