#!/bin/bash
# interleaved pipeline A/B of environment settings: ab_env.sh TAG "A-env" "B-env" [pairs]
# (each env string is a space-separated list of VAR=value, may be empty)
set -o pipefail
TAG=$1; A=$2; B=$3; N=${4:-3}
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > "gpurun_out/${TAG}_${v}${i}.json" 2> "gpurun_out/${TAG}_${v}${i}.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      "gpurun_out/${TAG}_${v}${i}.json" "$v$i[$E]"
  done
done
