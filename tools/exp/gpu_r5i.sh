#!/bin/bash
# round 5: the front with untied LDS waits (no s_nop before each tile's MFMAs) vs HEAD's library
# (built as libtrk_amd_tied.so), front stamps then three interleaved pipeline pairs; the front
# and transpose parity tests first
set -o pipefail
P=a-lightweight-unsupervised-feature-extractor-_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "rmb_front or nchw or roi_align" --timeout 120 \
  --timeout-method thread 2>&1 | tail -3 || exit 1
timeout -k 10 180 python tools/exp/front_prof.py "" || exit 1
TRK_LIB_PATH=$PWD/$P/libtrk_amd_tied.so timeout -k 10 180 python tools/exp/front_prof.py "" || exit 1
tools/exp/ab3.sh r5i 3 "" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_tied.so"
