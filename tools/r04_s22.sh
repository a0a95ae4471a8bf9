#!/bin/bash
# round-4 session 22: OPQ GEMM loop order variants (split-and-store first / no last-step branches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/opq_sfirst.so python -u -m pytest tests/test_opq_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "MIVQ_LIB=$PWD/tools/build/opq_uncond.so python -u -m pytest tests/test_opq_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_sfirst.so tools/build/opq_uncond.so --reps 6" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_sfirst.so tools/build/opq_uncond.so --reps 6"
