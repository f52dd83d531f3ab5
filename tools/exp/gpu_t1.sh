#!/bin/bash
# tracker + chain GPU tests, then one bench run (each step under its own limit)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-t1}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tracking_gpu.py tests/test_gpu_chain.py > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" "$OUT/${TAG}_pytest.log" | tail -n 30
[ $rc -ne 0 ] && { tail -n 40 "$OUT/${TAG}_pytest.log"; exit $rc; }
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 "$OUT/${TAG}_bench.log" | cut -c1-3000
exit $rc
