#!/bin/bash
# round-5 session 34: the RCCL world-1 collective test (new), and library GEMM yardsticks for the
# OPQ rotation's shape (torch.matmul f16 / bf16 / fp32 vs the split-f16 kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_sharded_gpu.py -m gpu" \
  "python -u tools/opq_probe.py --lib-gemm --reps 10"
