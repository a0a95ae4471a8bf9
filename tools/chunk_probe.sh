#!/bin/bash
# Filter / resolve durations per library variant (rocprofv3 kernel traces of the headline leg).
# usage: tools/chunk_probe.sh name=path.so ...   (name "default" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="--steps 40 --warmup 10 --no-adc --no-cpu-baseline --no-alt-data --no-config5 --no-configs --no-north-star"
for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$name" != default ]; then export MIVQ_LIB=$PWD/$lib; else unset MIVQ_LIB; fi
    timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/kt_$name -o run --output-format csv -- \
        python3 bench.py $B > gpurun_out/kt_$name.log 2>&1 || exit $?
    f=$(find gpurun_out/kt_$name -name '*kernel_trace.csv' | head -n 1)
    echo "== $name: $(grep -h 'encode:' gpurun_out/kt_$name.log)"
    python3 tools/ktrace.py "$f" pq_encode_cs_kernel pq_resolve transpose_codes
done
