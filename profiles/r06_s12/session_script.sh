#!/bin/bash
# round 6 session 12: merged resolve split over two workgroups per list (this) vs one (split1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k 'pq or slice' tests/test_pinning_gpu.py tests/test_opq_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_split1.so --reps 20" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_split1.so --reps 10 --M 8" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_split1.so --reps 10 --M 32" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_split1.so --reps 6 --n 6650000 --d 1024" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_split1.so --reps 4 --n 10000000"
