#!/bin/bash
# round-5 session 29: 2^20-row slices (better at 10M x 1536, session 28) on the config #5 shape and
# on a 1.5M-row call (one full slice + a half one)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_sl20.so --n 6650000 --d 1024 --reps 4" \
  "python -u tools/ab_lib.py $L/libmivq_sl20.so --n 1500000 --reps 6" \
  "python -u tools/ab_lib.py $L/libmivq_sl20.so --n 6650000 --d 1024 --reps 4"
