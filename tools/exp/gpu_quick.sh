#!/bin/bash
# Quick GPU iteration: parity tests + kernel microbench (stops on a crash).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 "$OUT/pytest_gpu.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/kbench.py > "$OUT/kbench.log" 2>&1
rc=$?; echo "kbench rc=$rc"; cat "$OUT/kbench.log" | grep -v amdgpu.ids
exit $rc
