#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, no tracing) over a bench run covering the headline
# encode and the OPQ32 / SQ-8 / RaBitQ-1 legs; then tools/traffic.py writes profiles/traffic.json
# and tools/pmc_summary.py the per-kernel counter summaries.  usage: tools/pmc_traffic.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
KRE="pq_encode_cs_kernel|pq_resolve_merged|pq_transpose_codes|opq_row_scale|opq_split_gemm|sq_encode_f32_vec|rabitq_encode_wide_kernel|erq_rotate_fast_kernel"
BENCH="python -u bench.py --no-adc --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --steps 3 --warmup 1"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    echo "== pass $i: $group"
    # counters only for the benched kernels: every other dispatch (k-means / OPQ fit, torch ops)
    # runs unserialised, so a pass takes about as long as the bench itself
    timeout -k 10 -s KILL 400 rocprofv3 --pmc $group --kernel-include-regex "$KRE" -d $OUT/p$i -o run --output-format csv -- $BENCH > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python tools/traffic.py $OUT 3 > $OUT/traffic.log 2>&1
for k in pq_encode_cs_kernelILi6ELi3ELi96 pq_resolve_merged_kernelILi6ELi96 pq_encode_cs_kernelILi12ELi3ELi192 pq_encode_cs_kernelILi3ELi3ELi48 opq_split_gemm_kernel sq_encode_f32_vec_kernel rabitq_encode_wide_kernel erq_rotate_fast_kernel; do
    echo "== $k"; python tools/pmc_summary.py $OUT $k 3
done > $OUT/summary.txt 2>&1
cp profiles/traffic.json $OUT/traffic.json
