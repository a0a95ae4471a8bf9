#!/bin/bash
# PMC passes over one bench encode run (rocprofv3 --pmc, no tracing domains mixed in).
# usage: tools/pmc.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
OUT=gpurun_out/pmc_$tag
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
BENCH="python bench.py --no-adc --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --no-configs --steps 3 --warmup 1 $*"
i=0
for group in \
    "FETCH_SIZE" \
    "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
    "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
    "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum" ; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 300 rocprofv3 --pmc $group -d $OUT/p$i -o run --output-format csv -- $BENCH > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
