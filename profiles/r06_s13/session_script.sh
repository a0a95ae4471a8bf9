#!/bin/bash
# round 6 session 13: screened RaBitQ estimator blocks (dense first block, then keys appended only
# when they beat the running k-th element, merged in place)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k rabitq tests/test_rabitq_index_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqbase.so" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqbase.so --nq 10000 --n 1000000 --d 1024 --reps 3" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqbase.so --reps 3"
