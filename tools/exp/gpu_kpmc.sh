#!/bin/bash
# SQ/TCC counters for one kernel family: gpu_kpmc.sh TAG FILTER -- python script args
# (two --pmc passes, kernel trace only).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=$1; FILT=$2; shift 3
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --kernel-trace -d "$OUT/kpmc_$TAG" -o run --output-format csv -- python3 "$@" > "$OUT/kpmc_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/kpmc_$TAG.log"; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d "$OUT/kpmc2_$TAG" -o run --output-format csv -- python3 "$@" > "$OUT/kpmc2_$TAG.log" 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/kpmc2_$TAG.log"; exit $rc; }
cd "$ROOT" && python3 - "$FILT" "$OUT/kpmc_$TAG" "$OUT/kpmc2_$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
filt = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list)); dur = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if filt not in k:
        continue
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
