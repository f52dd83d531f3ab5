#!/bin/bash
# round 4: HBM traffic per kernel with and without rmb_front's L2 prefetch (rf_v 3)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in def pf0; do
  if [ $V = pf0 ]; then export TRK_TUNE="rf_pf=0"; else export TRK_TUNE=""; fi
  i=0
  for PM in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 180 rocprofv3 --pmc $PM --kernel-trace -d "$OUT/r4u_${V}_$i" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/r4u_${V}_$i.log" 2>&1) || exit 1
  done
  python3 tools/pmc_summary.py "$OUT/r4u_${V}_1" "$OUT/r4u_${V}_2" "$OUT/r4u_traffic_$V.json" > "$OUT/r4u_summary_$V.txt" || exit 1
  echo "== $V"; grep -E "rmb_front|total|step" "$OUT/r4u_summary_$V.txt" | head -8
done
