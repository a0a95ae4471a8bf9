#!/bin/bash
# round-5 session 7: filtered ADC with K1 = k + 4 lists (tests, both table widths), the callers'
# tests, PMC of the integer-LUT scan vs the fp32 scan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh \
  "python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "MIVQ_LIB=$PWD/vector-quantization_amd/lib/ab/libmivq_adce8.so python -u -m pytest tests/test_adc_filtered_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u -m pytest tests/test_kernels_gpu.py -k 'adc or flat or topk' tests/test_sharded_gpu.py tests/test_export_gpu.py tests/test_quantizers_gpu.py -m gpu -q -x -rf --timeout 300 --timeout-method thread" \
  "python -u tools/probe_adc.py" \
  "bash tools/pmc_qscan.sh u16"
