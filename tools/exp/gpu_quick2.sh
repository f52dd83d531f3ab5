#!/bin/bash
# quick iteration: all GPU tests + a short bench (no CPU baseline)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/q_pytest_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/q_pytest_$TAG.log"
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/q_pytest_$TAG.log"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/q_bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' "$OUT/q_bench_$TAG.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('value', d['value'], 'ms', d['ms_per_step'], 'ident', d['identity_rate'])
print({k: round(v) for k, v in r['kernel_us'].items()}, 'idle', r['embed_stream_idle_us_per_step'])"
exit $rc
