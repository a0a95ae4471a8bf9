#!/bin/bash
# Kernel split of one encode configuration: rocprofv3 --kernel-trace --stats over a short
# bench run, then tools/ktrace.py on the trace.  usage: tools/prof_split.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
OUT=gpurun_out/prof_$tag
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --no-configs "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprofv3 exit $rc"
[ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $OUT/run_kernel_trace.csv)
python tools/ktrace.py $f pq_encode_cs_kernel pq_resolve transpose_codes adc_lut adc_scan topk_merge | tee $OUT/split.txt
s=$(ls $OUT/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$s" ] && s=$(ls $OUT/run_kernel_stats.csv)
cp $s $OUT/kernel_stats.csv
# every kernel instance (template arguments) by launch size: the 2^21-row slices, the tail, the
# small calls of the fit and the sweep, each on its own line
for k in pq_ adc_ topk_ opq_ sq_ rabitq_; do python tools/ktrace_v.py $f $k; done > $OUT/split_by_grid.txt
python tools/ktrace_calls.py $f > $OUT/split_by_call.txt
