#!/bin/bash
# round 4: 256 x 256 transition tiles -- parity, isolated A/B, pipeline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread -k "transition_wide or fused_gemms" > gpurun_out/r4g_tests.log 2>&1 || { tail -30 gpurun_out/r4g_tests.log; exit 1; }
tail -3 gpurun_out/r4g_tests.log
timeout -k 10 200 python -u tools/exp/trans_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
tools/exp/ab_knob.sh r4wide "enc_trans_wide=0" "enc_trans_wide=1" 3
