#!/bin/bash
# round 6 session 32: filtered ADC grid-shape tests (pinned kernel, chunk rule)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py -q -x --timeout 120 --timeout-method thread"
