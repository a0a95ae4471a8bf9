#!/bin/bash
# round-5 session 12: full GPU suite, smoke and the default bench on the session-11 sources
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh pytest smoke "python -u bench.py"
