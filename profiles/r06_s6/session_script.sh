#!/bin/bash
# round 6 session 6: RaBitQ estimator search (qprep chains staged, multi-query MFMA) vs round 5
# (rqold); tiled top-k segment length 4096 (this) vs 16384 / 1024; tests; ADC A/B; bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py tests/test_rabitq_index_gpu.py tests/test_ivf_gpu.py tests/test_adc_filtered_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqold.so" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_seg16k.so" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_seg1k.so" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_seg16k.so --reps 3" \
  "python -u bench.py --no-north-star --no-config5 --no-alt-data"
