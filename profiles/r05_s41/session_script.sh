#!/bin/bash
# round-5 session 41: non-temporal row gathers in the merged resolve (build: tools/build_ab.sh rnt -DMIVQ_AB_RNT=1,
# a one-line knob removed after the measurement), interleaved A/Bs, codes compared
L=vector-quantization_amd/lib/ab/libmivq_rnt.so
bash tools/gpu_session.sh "python -u tools/ab_lib.py $L --reps 20" "python -u tools/ab_lib.py $L --reps 20 --n 4000000" \
  "python -u tools/ab_lib.py $L --d 1024 --M 16 --n 2000000 --reps 20" "python -u tools/ab_lib.py $L --M 8 --reps 20"
