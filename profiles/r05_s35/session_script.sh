#!/bin/bash
# round-5 session 35: the dsub-48 filter's x-stream cache policy (VERDICT r4 #5, PQ32 overfetch):
# interleaved A/B of policy 0 / sc0 against nt (codes compared bit for bit), then one FETCH_SIZE
# pass per build over a PQ32 1M x 1536 encode run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=vector-quantization_amd/lib
pmc48() {  # $1 tag, $2 library
  MIVQ_LIB=$2 timeout -k 10 -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex pq_encode_cs_kernel \
    -d gpurun_out/pmc48_$1/p1 -o run --output-format csv -- python3 -u tools/ab_lib.py $2 --M 32 --reps 3 \
    > gpurun_out/pmc48_$1.log 2>&1 && python tools/pmc_summary.py gpurun_out/pmc48_$1 pq_encode_cs_kernelILi3ELi3ELi48 3
}
export -f pmc48
bash tools/gpu_session.sh \
  "python -u tools/ab_lib.py $L/ab/libmivq_x48a0.so --M 32 --reps 10" \
  "python -u tools/ab_lib.py $L/ab/libmivq_x48a1.so --M 32 --reps 10" \
  "pmc48 nt $PWD/$L/libmivq.so" \
  "pmc48 a0 $PWD/$L/ab/libmivq_x48a0.so" \
  "pmc48 a1 $PWD/$L/ab/libmivq_x48a1.so"
