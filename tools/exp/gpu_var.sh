#!/bin/bash
# bench variants: each argument is one env assignment list ("A=1,B=2"), one bench run each
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  timeout -k 10 240 env ${V//,/ } python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/var_$i.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "variant $V rc=$rc"; tail -n 5 "$OUT/var_$i.log"; exit $rc; }
  python3 - "$OUT/var_$i.log" "$V" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]; b = r["step_breakdown"]
        k = {x: round(v) for x, v in r["kernel_us"].items() if x not in ("roi_align", "encoder", "cost", "lsap")}
        print(sys.argv[2], d["value"], d["ms_per_step"], "sum", b["kernel_sum_us"], "ovl", b["overlap"], "wait", b["host_wait_us"], k)
PY
done
