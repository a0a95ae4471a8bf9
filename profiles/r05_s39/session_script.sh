#!/bin/bash
# round-5 session 39: the search-index benchmark driver (run_benchmarks) and ivf-bench on the GPU
bash tools/gpu_session.sh \
  "python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_run_benchmarks_gpu.py tests/test_ivf_bench_gpu.py -m gpu"
