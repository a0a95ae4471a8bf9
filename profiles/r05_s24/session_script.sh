#!/bin/bash
# round-5 session 24: ADC LUT kernel, 32 (default) vs 16 / 8 queries per workgroup
# (interleaved A/B, LUTs compared bit for bit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_lutq16.so --what lut --n 100000 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_lutq8.so --what lut --n 100000 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_lutq16.so --what lut --n 100000 --M 32 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_lutq16.so --what lut --n 100000 --d 1024 --nq 10000 --reps 4"
