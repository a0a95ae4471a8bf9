#!/bin/bash
# round 6 session 8: persistent pipelined multi-query RaBitQ estimator
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k rabitq tests/test_rabitq_index_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqold.so" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqold.so --reps 3" \
  "bash tools/pmc_rq.sh est vector-quantization_amd/lib/ab/libmivq_rqold.so"
