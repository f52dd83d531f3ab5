#!/bin/bash
# One gpurun call with the round's judged evidence: GPU parity tests, smoke, the
# driver's bench command, a rocprofv3 kernel trace of one bench run split into the timed
# region's and the isolated pass's launches (bench.py's marker kernels, tools/prof_window.py),
# HBM traffic (FETCH / WRITE passes), two SQ counter passes (MFMA busy, waits, LDS) and a
# FETCH + GRBM pass (bytes and effective clock, timed vs isolated).  Each GPU step has its own
# time limit; any failure ends the script before the next GPU step.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:-r05a}
SKIP_TESTS=${SKIP_TESTS:-0}
step() {
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/${TAG}_$name.log" | cut -c1-400
  return $rc
}
if [ "$SKIP_TESTS" != 1 ]; then
  step pytest 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit $?
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench 600 python bench.py --steps 20 --warmup 5 || exit $?
fi
[ "${SKIP_PROF:-0}" = 1 ] && { echo "== done (no profiles)"; exit 0; }
cd /tmp
step stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline || exit $?
step pmc_clk 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  -d "$OUT/pmcclk_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline || exit $?
i=0
for PM in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  step pmc$i 180 rocprofv3 --pmc $PM --kernel-trace -d "$OUT/pmc${i}_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline || exit $?
done
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT/pmc1_$TAG" "$OUT/pmc2_$TAG" "$OUT/pmc_traffic_$TAG.json" > "$OUT/pmc_${TAG}_summary.txt"
python3 tools/pmc_sq_summary.py "$OUT/pmc3_$TAG" "$OUT/pmc4_$TAG" "$OUT/pmc_sq_$TAG.json" > "$OUT/pmc_sq_${TAG}.txt"
python3 tools/pmc_clock.py "$OUT/pmcclk_$TAG" "$OUT/pmc_clock_$TAG.json" > "$OUT/pmc_clock_$TAG.txt"
python3 tools/kernel_stats.py "$OUT/prof_$TAG" "$OUT/kernel_stats_$TAG" > "$OUT/kernel_stats_$TAG.log"
cat "$OUT/pmc_sq_${TAG}.txt" "$OUT/pmc_clock_$TAG.txt" "$OUT/kernel_stats_$TAG.log"
echo "== done"
