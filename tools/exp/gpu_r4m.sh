#!/bin/bash
# round 4: LSAP 16-lane shortcut (parity, breakdown, tracker), tightened chain tolerances,
# rf_sumlanes pipeline A/B
set -o pipefail
mkdir -p gpurun_out
./tools/exp/gpu_r4j.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_tracking_gpu.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread -k "lsap or track or bf16 or half or golden or c3" > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -1 gpurun_out/r4m_tests.log
tools/exp/ab_knob.sh r4sl "rf_sumlanes=0" "rf_sumlanes=1" 3
