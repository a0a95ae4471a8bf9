#!/bin/bash
# LDS counters of the ADC scan at 1000 queries x 1M codes (one rocprofv3 --pmc pass each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_adc
mkdir -p $OUT
BENCH="python bench.py --no-cpu-baseline --no-alt-data --no-north-star --no-config5 --no-configs --steps 2 --warmup 1"
i=0
for group in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $group -d $OUT/p$i -o run --output-format csv -- $BENCH > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
