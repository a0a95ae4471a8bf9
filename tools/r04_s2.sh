#!/bin/bash
# round-4 session 2: ADC A/B, PC sampling and counters of the filter
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh "python tools/ab_lib.py tools/build/libmivq_r03.so --what adc --reps 6" \
  "bash tools/pcsample.sh r04s2" "bash tools/pmc.sh r04s2"
