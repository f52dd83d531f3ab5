#!/bin/bash
# cost kernel iteration: cost / tracker parity tests, then tools/exp/cost_bench.py
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread \
  -k "cost or track or step or costcard or kalman" > "$OUT/pytest_cost.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 6 "$OUT/pytest_cost.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/exp/cost_bench.py > "$OUT/cost_bench.log" 2>&1
rc=$?; echo "cost_bench rc=$rc"; grep -v amdgpu.ids "$OUT/cost_bench.log"
exit $rc
