#!/bin/bash
# DSC epilogue A/B: fused-GEMM parity tests, then enc_breakdown dsc with dsc_split 0 / 1 alternating
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -m gpu -q -rf -x --timeout 120 --timeout-method thread \
  -k "enc_fused or c3 or c2 or encoder" > "$OUT/pytest_dsc.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_dsc.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2 3; do
  for v in 0 1; do
    TRK_TUNE=dsc_split=$v ENC_DBG0=1 timeout -k 10 120 python tools/exp/enc_breakdown.py dsc > "$OUT/dsc_${v}_$rep.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 "$OUT/dsc_${v}_$rep.log"; exit $rc; }
    echo "split=$v $(grep '^{' "$OUT/dsc_${v}_$rep.log" | tr '\n' ' ')"
  done
done
