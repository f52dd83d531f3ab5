#!/bin/bash
# One gpurun call: GPU parity tests, smoke, short bench, rocprofv3 stats.
# Every GPU step has its own time limit; a crash / abort / timeout (rc > 1)
# ends the script before anything else touches the GPU.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:-r01}
step() {
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 8 "$OUT/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py --steps 20 --warmup 5 --cpu-budget 15 || exit $?
cd /tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline || exit $?
cd "$ROOT"
bash tools/exp/gpu_pmc.sh "$TAG" > "$OUT/pmc_$TAG.txt" 2>&1 || exit $?
echo "== done"
