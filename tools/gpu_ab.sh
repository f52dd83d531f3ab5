#!/bin/bash
# A/B of the full bench on one box: each "ENV=..." argument is one configuration
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > "$OUT/ab_$i.log" 2>&1 || { echo "cfg $cfg failed"; tail -5 "$OUT/ab_$i.log"; exit 1; }
  grep '^{' "$OUT/ab_$i.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$cfg', d['value'], d['ms_per_step'], d['identity_rate'], {k: round(v) for k, v in r['kernel_us'].items() if k in ('cost','lsap','enc_g1_dwconv','enc_gemm_dsc','enc_gemm_trans','enc_rmb_front','roi_stage')})"
done
