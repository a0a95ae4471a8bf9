#!/bin/bash
# round-5 session 28: slice size of large encode calls (2^21 rows default) at 10M x 1536:
# 2^19 / 2^20 / 2^22-row slices, interleaved A/Bs, codes compared
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_sl20.so --n 10000000 --reps 3" \
  "python -u tools/ab_lib.py $L/libmivq_sl22.so --n 10000000 --reps 3" \
  "python -u tools/ab_lib.py $L/libmivq_sl19.so --n 10000000 --reps 3" \
  "python -u tools/ab_lib.py $L/libmivq_sl20.so --n 10000000 --reps 3"
