# round-5 session 43: PMC counters and a kernel trace of the RaBitQ estimator search
# (tools/bench_configs.py --workload rabitq1 --n 200000: 1000 queries over 200k x 3072 codes)
P="python3 -u tools/bench_configs.py --workload rabitq1 --n 200000 --steps 2 --warmup 1 --cpu-seconds 1"
bash tools/gpu_session.sh \
  "timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex rabitq_est_mfma -d gpurun_out/pmc_rq/p1 -o run --output-format csv -- $P > gpurun_out/pmc_rq.log 2>&1 && python tools/pmc_summary.py gpurun_out/pmc_rq rabitq_est_mfma" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_rq -o run --output-format csv -- $P > gpurun_out/kt_rq.log 2>&1 && f=\$(ls gpurun_out/kt_rq/*/run_kernel_stats.csv gpurun_out/kt_rq/run_kernel_stats.csv 2>/dev/null | head -1) && head -12 \$f | cut -c1-220"
