#!/bin/bash
# round 5: the ROI sweep's column prefetch (roi_pf 1) -- parity, isolated A/B, pipeline A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "roi_align or nchw" --timeout 120 \
  --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 120 python tools/exp/roi_ab.py "roi_pf=0" "roi_pf=1" || exit 1
tools/exp/ab3.sh r5n 3 "" "TRK_TUNE=roi_pf=1"
