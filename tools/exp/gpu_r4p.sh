#!/bin/bash
# round 4: persistent rmb_front (rf_v 3) -- parity, isolated stamps / timing, pipeline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "rmb_front_vs_two or sum_lanes" > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -1 gpurun_out/r4p_tests.log
timeout -k 10 400 python -u tools/exp/front_prof.py "" "rf_v=3" "" "rf_v=3" 2>&1 | grep -v amdgpu.ids | grep -v per_wave || exit 1
tools/exp/ab_knob.sh r4pers "rf_v=2" "rf_v=3" 3
