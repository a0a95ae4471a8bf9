#!/bin/bash
# round-5 session 38: `vq-benchmark ivf-bench` runners on the GPU (tests/test_ivf_bench_gpu.py);
# run inline (profiles/ does not travel to the box):
bash tools/gpu_session.sh \
  "python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ivf_bench_gpu.py -m gpu"
