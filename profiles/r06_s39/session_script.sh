#!/bin/bash
# round 6 session 39: rerank cost split by kernel trace (profiling builds: no inserts / no
# gathers + lookups; their timings in ab_lib include the fp32 re-run their wrong bounds cause)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "rocprofv3 --kernel-trace -d gpurun_out/rrp1 -o run --output-format csv -- python tools/ab_lib.py $A/libmivq_rrp1.so --what adc --reps 5" \
  "rocprofv3 --kernel-trace -d gpurun_out/rrp2 -o run --output-format csv -- python tools/ab_lib.py $A/libmivq_rrp2.so --what adc --reps 5"
