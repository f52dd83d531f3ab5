#!/bin/bash
# round 4: rmb_front lag variants -- parity then phase stamps / isolated times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread -k "rmb_front" > gpurun_out/r4b_front_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/exp/front_prof.py "" "rf_lag=8" "rf_lag=0" "rf_v=1" > gpurun_out/r4b_front_prof.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -x -v -s --timeout 240 --timeout-method thread -k "encoder or c3 or half or se_head or roi_align" > gpurun_out/r4b_enc_err.log 2>&1 || exit 1
