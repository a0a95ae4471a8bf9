#!/bin/bash
# round-5 session 26: the dsub-96 (headline) filter at 16 waves / 4 per SIMD (one accumulator,
# x and centroid fragments read per centroid block to fit 128 VGPRs) vs the 12-wave default;
# codes compared, then the encode tests on the variant via its own library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib/ab
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/libmivq_nw96_16.so --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_nw96_16.so --data clustered --reps 8" \
  "python -u tools/ab_lib.py $L/libmivq_nw96_16.so --n 10000000 --reps 3"
