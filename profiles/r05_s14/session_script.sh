#!/bin/bash
# round-5 session 14: the final encode / OPQ / ADC sources after the prune: full GPU suite,
# smoke, PMC traffic passes (profiles/traffic.json), kernel-trace splits by call size, and the
# default bench (the driver's command)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh pytest smoke \
  "bash tools/pmc_traffic.sh" \
  "bash tools/prof_split.sh r05_1m --steps 5 --warmup 2" \
  "bash tools/prof_split.sh r05_10m --n 10000000 --no-adc --steps 3 --warmup 1" \
  "python -u bench.py"
