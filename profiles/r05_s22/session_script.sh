#!/bin/bash
# round-5 session 22: 5-bit integer ADC entries (eight lookups per byte unpack) vs 6-bit:
# interleaved A/B on Gaussian and clustered rows at M = 16 / 32 and the config #5 shape, then
# the uncertified-query counts of both (MIVQ_ADC_STATS=1, timing ignored)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --M 32 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --data clustered --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --n 6650000 --d 1024 --reps 4" \
  "MIVQ_ADC_STATS=1 python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --reps 1 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "MIVQ_ADC_STATS=1 python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --data clustered --reps 1 2>&1 | sort | uniq -c | sort -rn | head -20" \
  "MIVQ_ADC_STATS=1 python -u tools/ab_lib.py $L/libmivq_bits5.so --what adc --M 32 --reps 1 2>&1 | sort | uniq -c | sort -rn | head -20"
