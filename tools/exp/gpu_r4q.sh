#!/bin/bash
# round 4: rf_v 3 in the pipeline -- per-variant rocprof kernel stats (front / transition /
# totals) and bench values, to see whether the persistent front's isolated gain survives
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for T in "" "rf_v=3" "rf_v=3,rf3_groups=14" "rf_v=3,rf3_groups=12"; do
  i=$((i+1))
  export TRK_TUNE="$T"
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/r4q_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/r4q_$i.json" 2> "$OUT/r4q_$i.err") || exit 1
  python3 - "$OUT/r4q_$i" "$T" "$OUT/r4q_$i.json" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
out = {r["Name"].split("(")[0][-40:]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e3, 1)) for r in rows
       if float(r["TotalDurationNs"]) > 0}
top = sorted(out.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:8]
print(repr(sys.argv[2]), "value", d["value"], {k: v[1] for k, v in top})
PY
done
