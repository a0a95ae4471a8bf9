#!/bin/bash
# round-4 session 4: kernel traces (driver-equivalent bench run; the OPQ fit alone)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 10 --warmup 3" \
  "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_opqfit -o run --output-format csv -- python tools/opq_fit_probe.py"
