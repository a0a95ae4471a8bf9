#!/bin/bash
# round 6 session 27: merged resolve -- two pair-batch gathers in flight (list entries three
# ahead, unconditional range-checked code stores): encode A/B against the previous build (head)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k pq_encode -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py $A/libmivq_head.so --reps 10" \
  "python tools/ab_lib.py $A/libmivq_head.so --M 8 --reps 10" \
  "python tools/ab_lib.py $A/libmivq_head.so --n 6650000 --d 1024 --reps 5" \
  "python tools/ab_lib.py $A/libmivq_head.so --M 32 --reps 10" \
  "bash tools/prof_split.sh r06_s27 --steps 5 --warmup 2 --no-adc --no-north-star --no-config5 --no-configs --no-alt-data --no-cpu-baseline"
