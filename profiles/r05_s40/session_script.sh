#!/bin/bash
# round-5 session 40: the whole GPU suite and smoke on the final tree (after the ivf-bench /
# run_benchmarks callers and the RCCL test)
bash tools/gpu_session.sh pytest smoke
