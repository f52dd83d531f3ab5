#!/bin/bash
# round 5: trans5 (32x32x16 transition) parity tests, isolated A/B + phase stamps vs trans4,
# then a pipeline A/B (enc_trans 1 vs 2), three interleaved pairs
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "trans" --timeout 120 \
  --timeout-method thread 2>&1 | tail -4 || exit 1
timeout -k 10 120 python tools/exp/trans_ab.py || exit 1
tools/exp/ab3.sh r5e 3 "" "TRK_TUNE=enc_trans=2"
