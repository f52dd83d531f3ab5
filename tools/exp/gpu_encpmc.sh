#!/bin/bash
# Encoder GEMM breakdown (timings) + two SQ PMC passes over the undisturbed kernels.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-e1}
timeout -k 10 300 python tools/exp/enc_breakdown.py > "$OUT/encbd_$TAG.log" 2>&1
rc=$?; echo "breakdown rc=$rc"; grep -v amdgpu.ids "$OUT/encbd_$TAG.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp
export ENC_DBG0=1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for PM in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PM --kernel-trace -d "$OUT/encpmc${i}_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/tools/exp/enc_breakdown.py" > "$OUT/encpmc${i}_$TAG.log" 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 "$OUT/encpmc${i}_$TAG.log"; exit $rc; }
done
cd "$ROOT" && python3 - "$OUT/encpmc1_$TAG" "$OUT/encpmc2_$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "at::" in k:
        continue
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
