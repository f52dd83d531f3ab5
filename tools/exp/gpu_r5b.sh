#!/bin/bash
# round 5: the front's early X groups (libtrk_amd.so) vs HEAD~ (libtrk_amd_base.so) vs + scalar
# depthwise FMAs (libtrk_amd_dws.so): isolated phase stamps, then the pipeline A/B/C
set -o pipefail
P=a-lightweight-unsupervised-feature-extractor-_amd
for L in libtrk_amd_base.so libtrk_amd.so libtrk_amd_dws.so; do
  echo "== front_prof $L"
  TRK_LIB_PATH=$PWD/$P/$L timeout -k 10 180 python tools/exp/front_prof.py || exit 1
done
tools/exp/ab3.sh r5b 3 "TRK_LIB_PATH=$PWD/$P/libtrk_amd_base.so" "" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_dws.so"
