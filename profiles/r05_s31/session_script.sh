#!/bin/bash
# round-5 session 31: two-rank streaming sweep for PQ / OPQ / SQ on one GPU; the bench's ADC leg
# on clustered rows (alt_data.adc)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_sharded_gpu.py -m gpu -v -x -rf --timeout 600 --timeout-method thread" \
  "python -u bench.py --no-configs --no-north-star --no-config5 --no-cpu-baseline --steps 3 --warmup 1"
