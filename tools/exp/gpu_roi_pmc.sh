#!/bin/bash
# SQ counters for the roi_align kernel alone (one --pmc pass, kernel trace only).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-roi}
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --kernel-trace -d "$OUT/pmc_$TAG" -o run --output-format csv -- python3 "$ROOT/tools/roi_only.py" 5 > "$OUT/pmc_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/pmc_$TAG.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  --kernel-trace -d "$OUT/pmc2_$TAG" -o run --output-format csv -- python3 "$ROOT/tools/roi_only.py" 5 > "$OUT/pmc2_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/pmc2_$TAG.log"
cd "$ROOT" && python3 - "$OUT/pmc_$TAG" "$OUT/pmc2_$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "roi" not in k and "nchw" not in k:
        continue
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
