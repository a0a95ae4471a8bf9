#!/bin/bash
# round-5 session 20: the dsub-64 filter (config #5 shape): 12 waves with two pipelined
# accumulators, 12 waves with one, 8 waves, against the 16-wave single-accumulator default;
# the integer ADC scan with its code-word loop unrolled vs not (interleaved A/Bs, outputs compared)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_nw12.so --n 6650000 --d 1024 --reps 6" \
  "python -u tools/ab_lib.py $L/libmivq_nw12np.so --n 6650000 --d 1024 --reps 6" \
  "python -u tools/ab_lib.py $L/libmivq_nw8.so --n 6650000 --d 1024 --reps 6" \
  "python -u tools/ab_lib.py $L/libmivq_qs0.so --what adc --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_qs0.so --what adc --M 32 --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_nw12.so --n 6650000 --d 1024 --reps 6"
