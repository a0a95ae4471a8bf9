#!/bin/bash
# round-5 session 10: certification rate and time of the filtered ADC vs the integer grid span
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "MIVQ_LIB=$PWD/vector-quantization_amd/lib/ab/libmivq_span1.0.so MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "MIVQ_LIB=$PWD/vector-quantization_amd/lib/ab/libmivq_span4.0.so MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "python -u tools/probe_adc.py" \
  "python -u tools/probe_adc.py --M 32" \
  "python -u tools/probe_adc.py --n 6650000 --d 1024 --nq 10000 --reps 4" \
  "MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --data clustered --reps 3 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "python -u -m pytest tests/test_adc_filtered_gpu.py tests/test_sharded_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread"
