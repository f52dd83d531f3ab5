#!/bin/bash
# round 4: SE off the embedding stream (TRK_SE_DEFER=1) -- e2e parity through the pipeline, A/B
set -o pipefail
mkdir -p gpurun_out
TRK_SE_DEFER=1 timeout -k 10 600 python -u -m pytest tests/test_e2e_c3.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/r4o_e2e.log 2>&1 || { tail -30 gpurun_out/r4o_e2e.log; exit 1; }
grep -E "c3 e2e|passed|failed" gpurun_out/r4o_e2e.log
tools/exp/ab_env.sh r4sed "TRK_SE_DEFER=0" "TRK_SE_DEFER=1" 3
