#!/bin/bash
# round 4: fused rmb v2 (SE on the normal group) -- parity, phase stamps, pipeline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -x -v -s --timeout 240 --timeout-method thread -k "rmb_fused or fused_full" > gpurun_out/r4e_fused_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/exp/fused_prof.py > gpurun_out/r4e_fused_prof.log 2>&1 || exit 1
TRK_FULL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4e_bench_full.json 2> gpurun_out/r4e_bench_full.err || exit 1
TRK_FULL=1 TRK_ROI_AFTER= timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4e_bench_full_ungated.json 2> gpurun_out/r4e_bench_full_ungated.err || exit 1
