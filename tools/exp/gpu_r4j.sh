#!/bin/bash
# round 4: LSAP shortcut changes -- parity + isolated breakdown, then the judged round
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -k "lsap" > gpurun_out/r4j_tests.log 2>&1 || { tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -2 gpurun_out/r4j_tests.log
timeout -k 10 300 python -u tools/lsap_bench.py 10 2>&1 | grep -v amdgpu.ids || exit 1
