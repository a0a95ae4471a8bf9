#!/bin/bash
# round 6 session 1: GPU suite on the flags ABI; A/B of the conflict-free integer-scan layout
# (this build) vs the round-5 layout (lib/ab/libmivq_qold.so) at the headline, config #5 and
# M = 32 shapes; qscan PMC of both layouts at both shapes; the streaming-sweep device rate;
# the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cp vector-quantization_amd/lib/libmivq.so vector-quantization_amd/lib/ab/libmivq_new.so
bash tools/gpu_session.sh pytest smoke \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_qold.so --what adc --reps 10" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_qold.so --what adc --reps 10 --M 32" \
  "python tools/ab_lib.py vector-quantization_amd/lib/ab/libmivq_qold.so --what adc --reps 5 --n 6650000 --d 1024 --nq 10000" \
  "bash tools/pmc_qscan.sh new_1m" \
  "bash tools/pmc_qscan.sh new_c5 --n 6650000 --d 1024 --nq 10000" \
  "cp vector-quantization_amd/lib/ab/libmivq_qold.so vector-quantization_amd/lib/libmivq.so && bash tools/pmc_qscan.sh old_1m && bash tools/pmc_qscan.sh old_c5 --n 6650000 --d 1024 --nq 10000; rc=\$?; cp vector-quantization_amd/lib/ab/libmivq_new.so vector-quantization_amd/lib/libmivq.so; exit \$rc" \
  "python -u tools/stream_rate.py" \
  "python -u bench.py"
