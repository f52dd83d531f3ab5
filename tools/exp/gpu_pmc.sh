#!/bin/bash
# HBM traffic per kernel launch: separate rocprofv3 --pmc passes for
# FETCH_SIZE and WRITE_SIZE (they do not fit one TCC pass on gfx950), kernel
# trace only -- no runtime/hip/hsa tracing alongside counters.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-r01}
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C ($(date +%T))"
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_${TAG}_$C" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/pmc_${TAG}_$C.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/pmc_${TAG}_$C.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd "$ROOT" && python3 tools/pmc_summary.py "$OUT/pmc_${TAG}_FETCH_SIZE" "$OUT/pmc_${TAG}_WRITE_SIZE" "$OUT/pmc_traffic_${TAG}.json" > "$OUT/pmc_${TAG}_summary.txt"
cat "$OUT/pmc_${TAG}_summary.txt"
