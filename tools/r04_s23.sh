#!/bin/bash
# round-4 session 23 / 26: GPU tests + smoke on the final sources, then their PMC traffic passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh pytest smoke || exit $?
bash tools/pmc_traffic.sh
