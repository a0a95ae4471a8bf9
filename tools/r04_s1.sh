#!/bin/bash
# round-4 session 1: GPU tests and A/Bs of this round's changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh pytest \
  "python tools/ab_lib.py tools/build/libmivq_oldpd.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_nopl.so --reps 10" \
  "python tools/ab_lib.py tools/build/libmivq_r03.so --reps 10" \
  "python tools/ab_opq.py vector-quantization_amd/lib/libmivq.so tools/build/libmivq_opq8w.so tools/build/libmivq_r03.so --reps 6"
