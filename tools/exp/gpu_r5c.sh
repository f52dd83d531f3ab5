#!/bin/bash
# round 5 experiments (2/2): pipeline A/B of HEAD vs all 16 pairs per XCD in 4 generations vs the
# ROI sweep's output stores non-temporal vs two embedding streams with frame f+1's encoder gated
# only behind frame f's front
set -o pipefail
P=a-lightweight-unsupervised-feature-extractor-_amd
echo "== front_prof 16 pairs x 4 generations"
TRK_TUNE=rf3_groups=16,rf3_chunks=4 timeout -k 10 180 python tools/exp/front_prof.py || exit 1
tools/exp/ab3.sh r5c 2 "" "TRK_TUNE=rf3_groups=16,rf3_chunks=4" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_roint.so" \
  "TRK_EMBED_STREAMS=2 TRK_EMBED_OVERLAP=1"
