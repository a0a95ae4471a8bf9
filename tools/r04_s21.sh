#!/bin/bash
# round-4 session 21 (final): round-end checks on the final tree and a kernel trace of the
# driver-equivalent bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh pytest smoke \
  "python bench.py" \
  "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3"
