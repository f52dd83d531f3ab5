#!/bin/bash
# rocprofv3 kernel stats of one python script: gpu_stats.sh TAG script args...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=$1; shift
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/st_$TAG" -o run --output-format csv -- python3 "$ROOT/$1" "${@:2}" > "$OUT/st_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/st_$TAG.log"; exit $rc; }
python3 - "$OUT/st_$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:25]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f}us {float(r['Percentage']):6.2f}%")
PY
