#!/bin/bash
# round-5 session 5: dsub-48 cache-policy A/Bs, resolve variant 2, multi-rank / caller tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_res2.so --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_0.so --M 32 --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_1.so --M 32 --reps 6" \
  "python -u tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_xaux48_16.so --M 32 --reps 6" \
  "python -u -m pytest tests/test_sharded_gpu.py tests/test_opq_gpu.py tests/test_sweep_gpu.py tests/test_quantizers_gpu.py tests/test_export_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread"
