#!/bin/bash
# round 6 session 21: query chains on a 64-query LDS-staged kernel; B operands read two k-steps
# ahead (bq2 variant) -- A/B against the previous build (scr4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k rabitq tests/test_rabitq_index_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_scr4.so --reps 7" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_bq2.so --reps 7" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_bq2.so --nq 10000 --n 1000000 --d 1024 --reps 3" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_scr4.so --nq 100 --n 1000000 --d 3072 --reps 5" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py none --reps 3"
