#!/bin/bash
# LDS / VALU / stall counters of the filtered ADC scan (adc_qscan_kernel), one rocprofv3 --pmc
# pass per group over tools/probe_adc.py (filtered and fp32-scan searches interleaved).
# usage: tools/pmc_qscan.sh TAG [probe_adc.py args, e.g. --n 6650000 --d 1024 --nq 10000]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
OUT=gpurun_out/pmc_$tag
mkdir -p $OUT
i=0
for group in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $group --kernel-include-regex "adc_qscan|adc_scan_kernel" -d $OUT/p$i -o run --output-format csv -- python tools/probe_adc.py --reps 2 "$@" > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python tools/pmc_summary.py $OUT adc_qscan | tee $OUT/summary_qscan.txt
python tools/pmc_summary.py $OUT adc_scan_kernel > $OUT/summary_scan.txt
