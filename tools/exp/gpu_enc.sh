#!/bin/bash
# encoder-kernel iteration: encoder/dwconv parity tests + encoder microbench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -x -k "encoder or dwconv or act_mean or scale or enc_fused" > "$OUT/pytest_enc.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 "$OUT/pytest_enc.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py enc > "$OUT/kbench_enc.log" 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids "$OUT/kbench_enc.log"
exit $rc
