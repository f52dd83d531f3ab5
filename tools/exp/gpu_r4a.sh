#!/bin/bash
# round 4: rmb_front decoupled halves -- parity, phase stamps, then the full GPU suite and a bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 240 --timeout-method thread -k "rmb_front" > gpurun_out/r4a_front_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp/front_prof.py "" "rf_v=1" > gpurun_out/r4a_front_prof.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || exit 1
