#!/bin/bash
# round-4 session 24 (final): default bench line (driver's command) and the kernel trace of the
# driver-equivalent command, on the final sources with their traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh \
  "python bench.py" \
  "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3"
