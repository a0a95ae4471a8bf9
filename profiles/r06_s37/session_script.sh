#!/bin/bash
# round 6 session 37: where the bench's ADC wall time goes (reps, parts), plus a kernel trace of it;
# the LUT kernel's compile-time dsub variants under the bit-exact tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_kernels_gpu.py -k 'adc_bit_exact or adc_lut' -q -x --timeout 120 --timeout-method thread" \
  "python tools/probe_adc_wall.py" \
  "rocprofv3 --kernel-trace --stats -d gpurun_out/adcwall -o run --output-format csv -- python tools/probe_adc_wall.py --nq 1000"
