#!/bin/bash
# round-5 session 36: x-stream policy sc0 (and 0) for the other filter shapes, interleaved A/Bs
# against the in-tree build (codes compared bit for bit): dsub 96 (headline), 64 (config #5), 192 (PQ8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_d96a1.so --reps 20" \
  "python -u tools/ab_lib.py $L/libmivq_d96a0.so --reps 20" \
  "python -u tools/ab_lib.py $L/libmivq_d64a1.so --d 1024 --M 16 --n 2000000 --reps 20" \
  "python -u tools/ab_lib.py $L/libmivq_d192a1.so --M 8 --reps 20" \
  "python -u tools/ab_lib.py $L/libmivq_d96a1.so --reps 20 --n 4000000"
