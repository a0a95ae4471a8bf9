#!/bin/bash
# round-5 session 13: the full GPU suite on the pruned sources (OPQ online row scales, fixed ADC
# filter constants, encode A/B knobs removed); OPQ A/B against the build with the row-scale
# pass; PMC traffic passes and kernel-trace splits (by kernel instance and launch size)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/ab_opq.py vector-quantization_amd/lib/libmivq.so vector-quantization_amd/lib/ab/libmivq_opq_rowpass.so --reps 8" \
  "bash tools/pmc_traffic.sh" \
  "bash tools/prof_split.sh r05_1m --steps 5 --warmup 2" \
  "bash tools/prof_split.sh r05_10m --n 10000000 --no-adc --steps 3 --warmup 1"
