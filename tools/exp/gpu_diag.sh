#!/bin/bash
# Pipeline diagnosis: the driver's bench command several times (run-to-run
# spread, per-step breakdown), one variant run, and a kernel-trace timeline.
# usage: gpu_diag.sh TAG [env assignments for the variant run...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-d1}; shift || true
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/diag_${TAG}_b$i.log" 2>&1
  rc=$?; echo "bench $i rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/diag_${TAG}_b$i.log"; exit $rc; }
  python3 - "$OUT/diag_${TAG}_b$i.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(d["value"], d["ms_per_step"], r.get("step_breakdown"), {k: round(v) for k, v in r["kernel_us"].items()})
PY
done
if [ $# -gt 0 ]; then
  timeout -k 10 240 env "$@" python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/diag_${TAG}_var.log" 2>&1
  rc=$?; echo "variant ($*) rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/diag_${TAG}_var.log"; exit $rc; }
  python3 - "$OUT/diag_${TAG}_var.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(d["value"], d["ms_per_step"], r.get("step_breakdown"))
PY
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/diag_${TAG}_kt" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/diag_${TAG}_kt.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/diag_${TAG}_kt.log"; exit $rc; }
cd "$ROOT"
F=$(find "$OUT/diag_${TAG}_kt" -name '*kernel_trace.csv' -print -quit)
python3 tools/timeline.py "$F" 40 3 > "$OUT/diag_${TAG}_timeline.txt"
tail -n 60 "$OUT/diag_${TAG}_timeline.txt"
