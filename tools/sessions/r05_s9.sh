#!/bin/bash
# round-5 session 9: kernel trace of the filtered ADC (where the 1M x 1000 call's time goes) and
# the sharded-index test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/adcprof -o run --output-format csv -- python -u tools/probe_adc.py --reps 4 > gpurun_out/adcprof.log 2>&1
rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls gpurun_out/adcprof/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/adcprof/run_kernel_trace.csv)
python tools/ktrace.py $f adc_qstats adc_qtab adc_qscan adc_rerank adc_scan_kernel topk_merge adc_lut | tee gpurun_out/adc_split.txt
timeout -k 10 300 python -u -m pytest tests/test_sharded_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/sharded.log 2>&1
echo "sharded exit $?"; tail -3 gpurun_out/sharded.log
