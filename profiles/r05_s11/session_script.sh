#!/bin/bash
# round-5 session 11: per-lane top-3 (certification rate, time) and entry widths 8 / 7 / 6 bits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
AB=$PWD/vector-quantization_amd/lib/ab
stats() { python -u tools/probe_adc.py --reps 3 "$@" 2>&1 | sort | uniq -c | sort -rn | head -8; }
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "MIVQ_ADC_STATS=1 MIVQ_LIB=$AB/libmivq_k3b7.so python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "MIVQ_ADC_STATS=1 MIVQ_LIB=$AB/libmivq_k3b6.so python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "MIVQ_ADC_STATS=1 MIVQ_LIB=$AB/libmivq_k2b8.so python -u tools/probe_adc.py --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "python -u tools/probe_adc.py" \
  "MIVQ_LIB=$AB/libmivq_k3b7.so python -u tools/probe_adc.py" \
  "MIVQ_LIB=$AB/libmivq_k3b6.so python -u tools/probe_adc.py" \
  "MIVQ_ADC_STATS=1 python -u tools/probe_adc.py --data clustered --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "MIVQ_ADC_STATS=1 MIVQ_LIB=$AB/libmivq_k3b6.so python -u tools/probe_adc.py --data clustered --reps 3 2>&1 | sort | uniq -c | sort -rn | head -8" \
  "MIVQ_LIB=$AB/libmivq_k3b6.so python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread"
