#!/bin/bash
# round-5 session 27: OPQ split GEMM with 128 x 128 tiles everywhere (two independent
# workgroups per CU: their barriers do not sync each other) vs the 256 x 256 default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib
bash tools/gpu_session.sh \
  "python -u tools/ab_opq.py $L/libmivq.so $L/ab/libmivq_opqs.so --reps 10" \
  "python -u tools/ab_opq.py $L/ab/libmivq_opqs.so $L/libmivq.so --reps 10"
