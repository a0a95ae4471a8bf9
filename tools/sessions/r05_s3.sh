#!/bin/bash
# round-5 session 3: multi-rank callers on one GPU, polar-factor fix, search / index paths
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_sharded_gpu.py tests/test_opq_gpu.py tests/test_sweep_gpu.py tests/test_quantizers_gpu.py tests/test_export_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread"
