#!/bin/bash
# round 6 session 15: estimator epilogue at 7 VALU per (query, code) term, one compare per key
# before the exact test; query staging through range-checked buffer loads (no spills)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k rabitq tests/test_rabitq_index_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_scr2.so --reps 7" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_scr2.so --nq 10000 --n 1000000 --d 1024 --reps 3" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_scr2.so --nq 100 --n 1000000 --d 3072 --reps 5" \
  "bash tools/pmc_rq.sh est"
