#!/bin/bash
# PMC passes of the RaBitQ estimator kernel (rabitq_est_mq_kernel) and the tiled top-k segment
# kernel over tools/probe_rq.py (1000 queries x 1M x 3072 codes, qb 4), one pass per group.
# usage: tools/pmc_rq.sh TAG [ignored] (this build alone)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
OUT=gpurun_out/pmc_$tag
mkdir -p $OUT
i=0
for group in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
             "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $group --kernel-include-regex "rabitq_est_mq|topk_seg|rq_screen" -d $OUT/p$i -o run --output-format csv -- python tools/probe_rq.py none --reps 2 > $OUT/p$i.log 2>&1
    rc=$?
    echo "   exit $rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python tools/pmc_summary.py $OUT "rabitq_est_mq_kernel<4, true>" | tee $OUT/summary_est.txt
python tools/pmc_summary.py $OUT topk_seg > $OUT/summary_seg.txt
python tools/pmc_summary.py $OUT rq_screen > $OUT/summary_merge.txt
