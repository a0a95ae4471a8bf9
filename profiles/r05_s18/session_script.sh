#!/bin/bash
# round-5 session 18: bench.py --gpus 2 on one card over gloo (the multi-rank bench path on real
# device memory), the other multi-rank GPU tests, and the D = 3072 Extended RaBitQ fixture
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_sharded_gpu.py tests/test_golden_wide.py -m gpu -v -rf --timeout 600 --timeout-method thread"
