#!/bin/bash
# encoder iteration: encoder GPU tests, then the GEMM breakdown with knob sweeps
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-x}; ITEMS=${2:-g1dw,dsc,trans}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -k "encoder or enc_ or dwconv" > "$OUT/encx_pytest_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/encx_pytest_$TAG.log"
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/encx_pytest_$TAG.log"; exit $rc; fi
timeout -k 10 300 python tools/exp/enc_breakdown.py "$ITEMS" > "$OUT/encx_$TAG.log" 2>&1
rc=$?; echo "breakdown rc=$rc"; grep -v amdgpu.ids "$OUT/encx_$TAG.log"; exit $rc
