#!/bin/bash
# Stochastic PC sampling (rocprofv3, beta) over the encode-only bench: where the filter's waves
# are and why they stall.  usage: tools/pcsample.sh <tag>  -> gpurun_out/pcs_<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pcs_$1
mkdir -p $OUT
BENCH="python -u bench.py --no-adc --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --no-configs --steps 10 --warmup 2"
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval 262144 --kernel-include-regex "pq_encode_cs_kernel|pq_resolve_merged" \
    -d $OUT/raw -o run --output-format csv -- $BENCH > $OUT/run.log 2>&1
rc=$?
echo "pc sampling exit $rc"
ls -R $OUT/raw | head -20
exit 0
