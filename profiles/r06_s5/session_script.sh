#!/bin/bash
# round 6 session 5: fused qstats+qtab (this build) vs the two kernels (lib/ab/libmivq_qp2.so);
# multi-query RaBitQ estimator vs the round-5 kernel (lib/ab/libmivq_rqold.so); VALU issue-rate
# probe (the ADC roofline's peak); tests; qscan PMC at both shapes; bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "timeout -k 5 60 ./tools/probes/valu_rate" \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_kernels_gpu.py tests/test_abi.py tests/test_pinning_gpu.py tests/test_rabitq_index_gpu.py tests/test_ivf_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_qp2.so --what adc --reps 10" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_qp2.so --what adc --reps 5 --n 6650000 --d 1024 --nq 10000" \
  "python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqold.so" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rqsplit -o run --output-format csv -- python tools/probe_rq.py vector-quantization_amd/lib/ab/libmivq_rqold.so --reps 3" \
  "bash tools/adc_split.sh 1m" \
  "bash tools/pmc_qscan.sh fin_1m" \
  "bash tools/pmc_qscan.sh fin_c5 --n 6650000 --d 1024 --nq 10000" \
  "python -u bench.py"
