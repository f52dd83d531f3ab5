#!/bin/bash
# rmb_front HBM traffic (FETCH_SIZE / WRITE_SIZE passes) per TRK_TUNE variant, isolated launches
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/front_pmc; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  for PM in FETCH_SIZE WRITE_SIZE; do
    TRK_TUNE="$v" timeout -k 10 120 rocprofv3 --pmc $PM --kernel-trace -d "$OUT/v${i}_$PM" -o run --output-format csv \
      -- python3 "$ROOT/tools/exp/front_run.py" > "$OUT/v${i}_$PM.log" 2>&1 || { echo "variant $v $PM failed"; exit 1; }
  done
  python3 - "$OUT" "$i" "$v" <<'PY'
import csv, glob, sys
out, i, v = sys.argv[1], sys.argv[2], sys.argv[3]
res = {}
for pm in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{out}/v{i}_{pm}/**/*counter_collection.csv", recursive=True)
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0])) if "rmb_front" in r["Kernel_Name"]]
    res[pm] = sum(vals) / max(len(vals), 1)
print(v or "default", "launches", len(vals), "read MB (2x FETCH KiB)", round(2 * res["FETCH_SIZE"] * 1024 / 1e6, 1),
      "write MB", round(res["WRITE_SIZE"] * 1024 / 1e6, 1))
PY
done
