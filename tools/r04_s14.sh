#!/bin/bash
# round-4 session 14: OPQ split GEMM with range-checked buffer loads (tools/build/opq_buf.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "MIVQ_LIB=$PWD/tools/build/opq_buf.so python -u -m pytest tests/test_opq_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_buf.so --reps 6" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/opq_buf.so --reps 6"
