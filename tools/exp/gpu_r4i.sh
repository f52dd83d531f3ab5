#!/bin/bash
# round 4: trans4 pipeline depth variants -- parity, isolated A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -k "trans4" > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
timeout -k 10 200 python -u tools/exp/trans_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
