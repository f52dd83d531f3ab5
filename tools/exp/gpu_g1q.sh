#!/bin/bash
# g1dw variant iteration: fused-GEMM parity tests, then the g1dw breakdown for the
# modes in $G1M (default 1 and 7), interleaved twice.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -x --timeout 120 --timeout-method thread \
  -k "enc_fused" > "$OUT/pytest_g1q.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 8 "$OUT/pytest_g1q.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  G1M=${G1M:-1,7} ENC_DBGS=${ENC_DBGS:-0,16,256,80,144} timeout -k 10 240 python tools/exp/enc_breakdown.py g1dw \
    > "$OUT/g1q_$rep.log" 2>&1
  rc=$?; echo "breakdown rc=$rc"; grep -v amdgpu.ids "$OUT/g1q_$rep.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
