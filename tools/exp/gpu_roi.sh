#!/bin/bash
# roi_align iteration: parity tests for roi_align only + microbench + SQ counters.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -x -k roi_align > "$OUT/pytest_roi.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 "$OUT/pytest_roi.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py roi > "$OUT/kbench_roi.log" 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids "$OUT/kbench_roi.log"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_roi_pmc.sh ${1:-roi}
