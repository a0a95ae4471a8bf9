#!/bin/bash
# Round-end evidence session (round 6): full GPU suite, smoke, PMC traffic passes
# (profiles/traffic.json), kernel-trace splits by call size at 1M and 10M rows, ADC and RaBitQ
# estimator splits and PMC (the estimator search's PMC and kernel trace too), the VALU issue-rate probe (the ADC roofline's peak), the
# streaming-sweep device rate, the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh pytest smoke \
  "bash tools/pmc_traffic.sh" \
  "bash tools/prof_split.sh r06_1m --steps 5 --warmup 2" \
  "bash tools/prof_split.sh r06_10m --n 10000000 --no-adc --steps 3 --warmup 1" \
  "timeout -k 5 60 ./tools/probes/valu_rate" \
  "bash tools/adc_split.sh 1m" \
  "bash tools/adc_split.sh c5 --n 6650000 --d 1024 --nq 10000" \
  "bash tools/pmc_qscan.sh fin_1m" \
  "bash tools/pmc_qscan.sh fin_c5 --n 6650000 --d 1024 --nq 10000" \
  "bash tools/pmc_rq.sh fin" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py none --reps 3" \
  "python -u tools/stream_rate.py" \
  "python -u bench.py"
