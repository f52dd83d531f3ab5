#!/bin/bash
# round 4: rmb_front2 depthwise priority (rf_dwprio) -- parity, phase stamps, pipeline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -k "sum_lanes" > gpurun_out/r4n_tests.log 2>&1 || { tail -30 gpurun_out/r4n_tests.log; exit 1; }
tail -1 gpurun_out/r4n_tests.log
timeout -k 10 400 python -u tools/exp/front_prof.py "" "rf_dwprio=1" "rf_dwprio=2" "" "rf_dwprio=1" "rf_dwprio=2" 2>&1 | grep -v amdgpu.ids || exit 1
tools/exp/ab_knob.sh r4dwp "rf_dwprio=0" "rf_dwprio=1" 3
