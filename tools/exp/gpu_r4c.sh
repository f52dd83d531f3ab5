#!/bin/bash
# round 4: fused rmb (front + SE + transition) -- parity, then timing vs the separate kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -x -v -s --timeout 240 --timeout-method thread -k "rmb_fused or fused_full or rmb_front" > gpurun_out/r4c_fused_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp/fused_ab.py > gpurun_out/r4c_fused_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/exp/front_prof.py "" "rf_lag=8" "rf_lag=0" "rf_v=1" > gpurun_out/r4c_front_prof.log 2>&1 || exit 1
TRK_FULL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4c_bench_full.json 2> gpurun_out/r4c_bench_full.err || exit 1
TRK_FULL=1 TRK_ROI_AFTER= timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4c_bench_full_ungated.json 2> gpurun_out/r4c_bench_full_ungated.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit 1
