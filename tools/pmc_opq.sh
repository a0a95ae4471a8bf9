#!/bin/bash
# PMC passes over tools/opq_probe.py (one counter group per rocprofv3 run, no tracing mixed in).
# usage: tools/pmc_opq.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_opq_$1
mkdir -p $OUT
i=0
for group in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
    "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
    "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum" \
    "FETCH_SIZE" ; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 120 rocprofv3 --pmc $group -d $OUT/p$i -o run --output-format csv -- python tools/opq_probe.py --reps 3 > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
