#!/bin/bash
# interleaved pipeline A/B/C of library builds or environments (one bench each per round):
# ab3.sh TAG ROUNDS "ENV_A" "ENV_B" ["ENV_C"]  (each ENV a space-separated VAR=value list, may be
# empty); prints value, ms/step and the front / transition live times per run
set -o pipefail
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > "gpurun_out/${TAG}_${k}_${i}.json" 2> "gpurun_out/${TAG}_${k}_${i}.err" || { echo "run $k/$i failed"; tail -3 "gpurun_out/${TAG}_${k}_${i}.err"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; k=r['kernel_us']
print(sys.argv[2], d['value'], d['ms_per_step'], 'front', k.get('enc_rmb_front'), 'trans', k.get('enc_gemm_trans'), 'roi', k.get('roi_stage'), 'iso_front', r['isolated_us'].get('enc_rmb_front'), 'iso_trans', r['isolated_us'].get('enc_gemm_trans'))" \
      "gpurun_out/${TAG}_${k}_${i}.json" "$k/$i[$E]"
  done
done
