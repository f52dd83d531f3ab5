#!/bin/bash
# round 4: LSAP shortcut, chain printouts, rf_sumlanes parity + isolated A/B, rf_pf pipeline A/B
set -o pipefail
mkdir -p gpurun_out
./tools/exp/gpu_r4k.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -k "sum_lanes or trans4" > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -1 gpurun_out/r4l_tests.log
timeout -k 10 300 python -u tools/exp/front_prof.py "" "rf_sumlanes=1" "" "rf_sumlanes=1" 2>&1 | grep -v amdgpu.ids | grep -v per_wave || exit 1
timeout -k 10 200 python -u tools/exp/trans_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
tools/exp/ab_knob.sh r4pf "rf_pf=8" "rf_pf=0" 3
