#!/bin/bash
# Kernel split of one mivq_adc_search configuration: rocprofv3 --kernel-trace over
# tools/probe_adc.py (filtered and fp32-scan searches interleaved), then tools/ktrace.py.
# usage: tools/adc_split.sh <tag> [probe_adc.py args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
OUT=gpurun_out/adcsplit_$tag
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python tools/probe_adc.py --reps 5 "$@" > $OUT/probe.log 2>&1
rc=$?
echo "rocprofv3 exit $rc"
[ $rc -ne 0 ] && exit $rc
tr=$(find $OUT -name "*kernel_trace.csv" | head -1)
python tools/ktrace.py "$tr" adc_lut_pk adc_lut_kernel adc_qstats adc_qtab adc_qscan adc_rerank "adc_scan_kernel<1, 8, 1>" topk_merge | tee $OUT/split.txt
