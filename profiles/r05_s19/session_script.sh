#!/bin/bash
# round-5 session 19: kernel splits by call size for the config #5 shape (6.65M x 1024, dsub 64)
# and for the other bench legs (PQ8, OPQ32, SQ-8, RaBitQ-1, Extended RaBitQ)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/prof_r05_cfg
mkdir -p $OUT
bash tools/gpu_session.sh \
  "bash tools/prof_split.sh r05_c5 --n 6650000 --d 1024 --no-adc --steps 3 --warmup 1" \
  "timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --n 200000 --no-adc --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --steps 2 --warmup 1 > $OUT/bench.log 2>&1 && f=\$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1) && python tools/ktrace_calls.py \$f > $OUT/split_by_call.txt && for k in pq_ opq_ sq_ rabitq_ erq_; do python tools/ktrace_v.py \$f \$k; done > $OUT/split_by_grid.txt"
