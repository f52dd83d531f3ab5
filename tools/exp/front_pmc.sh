#!/bin/bash
# rmb_front3 per library build or environment (isolated launches): phase cycles (front_prof.py)
# and one L2 counter pass (fabric read requests, L2 hits / misses; RDREQ x 128 B = bytes read
# from beyond L2).  usage: front_pmc.sh TAG "ENV_A" ["ENV_B" ...]  (each ENV a space-separated
# VAR=value list, e.g. TRK_LIB_PATH=...; may be empty)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$ROOT/gpurun_out"
TAG=$1; shift
k=0
for E in "$@"; do
  k=$((k+1))
  env $E timeout -k 10 120 python tools/exp/front_prof.py "" > "gpurun_out/${TAG}_prof_$k.txt" 2>&1 || { echo "prof $k failed"; exit 1; }
  echo "== $k [$E]"; grep '"variant"' "gpurun_out/${TAG}_prof_$k.txt" | cut -c1-330
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace \
    -d "$ROOT/gpurun_out/${TAG}_pmc_$k" -o run --output-format csv -- python3 "$ROOT/tools/exp/front_timeline.py" 1 \
    > "$ROOT/gpurun_out/${TAG}_pmc_$k.log" 2>&1) || { echo "pmc $k failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/${TAG}_pmc_$k" <<'PY'
import csv, glob, sys, collections
res = collections.defaultdict(list)
f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "rmb_front3" in r["Kernel_Name"]:
        res[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: round(sum(v) / len(v) / 1e6, 3) for k, v in res.items()}, "(millions per launch)")
PY
done
