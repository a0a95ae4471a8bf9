#!/bin/bash
# round 6 session 43: qstats with the wave's rows loaded first and |v| max from min / max -- A/B against HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py tests/test_pinning_gpu.py -k 'adc or lut or filtered' -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 20" \
  "python tools/ab_lib.py $A/libmivq_head.so --what adc --n 6650000 --d 1024 --nq 10000 --reps 3" \
  "rocprofv3 --kernel-trace -d gpurun_out/qstats -o run --output-format csv -- python tools/ab_lib.py $A/libmivq_head.so --what adc --reps 5"
