#!/bin/bash
# round-5 session 25: checkpoint of the current sources -- full GPU suite, smoke, PMC traffic
# passes (profiles/traffic.json), kernel-trace splits by call size, the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh pytest smoke \
  "bash tools/pmc_traffic.sh" \
  "bash tools/prof_split.sh r05_1m --steps 5 --warmup 2" \
  "python -u bench.py"
