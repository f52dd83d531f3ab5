#!/bin/bash
# round 4: LSAP one-lane-per-row shortcut (parity + breakdown) and the chain tests' measured errors
set -o pipefail
mkdir -p gpurun_out
./tools/exp/gpu_r4j.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_e2e_c3.py tests/test_gpu_kernels.py -q -s --timeout 300 --timeout-method thread -k "bf16 or half or c3 or golden" > gpurun_out/r4k_chain.log 2>&1 || { tail -30 gpurun_out/r4k_chain.log; exit 1; }
grep -E "max \|d\||cosine|passed|failed" gpurun_out/r4k_chain.log
