#!/bin/bash
# round-5 session 17: stall counters of the OPQ split GEMM (what bounds it at ~50 % MFMA busy:
# VALU halving and a SIMD-partner stagger both measured neutral in sessions 15-16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "bash tools/pmc_opq.sh r05 && for k in opq_split_gemm opq_row_scale; do echo == \$k; python tools/pmc_summary.py gpurun_out/pmc_opq_r05 \$k 3; done > gpurun_out/pmc_opq_r05/summary.txt 2>&1"
