#!/bin/bash
# round 5 experiments: the front's early X groups (libtrk_amd.so) vs HEAD~3 (libtrk_amd_base.so)
# vs + scalar depthwise FMAs (libtrk_amd_dws.so) vs all 16 pairs per XCD in 4 generations vs the
# ROI sweep's output stores non-temporal (libtrk_amd_roint.so); isolated phase stamps, then the
# pipeline A/B
set -o pipefail
P=a-lightweight-unsupervised-feature-extractor-_amd
for L in libtrk_amd_base.so libtrk_amd.so libtrk_amd_dws.so; do
  echo "== front_prof $L"
  TRK_LIB_PATH=$PWD/$P/$L timeout -k 10 180 python tools/exp/front_prof.py || exit 1
done
echo "== front_prof 16 pairs x 4 generations"
TRK_TUNE=rf3_groups=16,rf3_chunks=4 timeout -k 10 180 python tools/exp/front_prof.py || exit 1
tools/exp/ab3.sh r5b 2 "TRK_LIB_PATH=$PWD/$P/libtrk_amd_base.so" "" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_dws.so" \
  "TRK_TUNE=rf3_groups=16,rf3_chunks=4" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_roint.so"
