#!/bin/bash
# round-5 session 8: per-lane top-2 integer-LUT scan (tests, timing, PMC) and the callers' tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u -m pytest tests/test_kernels_gpu.py -k 'adc or flat or topk' tests/test_sharded_gpu.py tests/test_export_gpu.py tests/test_quantizers_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/probe_adc.py" \
  "python -u tools/probe_adc.py --M 32" \
  "python -u tools/probe_adc.py --n 6650000 --d 1024 --nq 10000 --reps 4" \
  "python -u tools/probe_adc.py --data clustered" \
  "bash tools/pmc_qscan.sh top2"
