#!/bin/bash
# round 5 experiments (1/2): the measured bf16 e2e error at HEAD; the front's early X groups
# (libtrk_amd.so) vs the cleanup commit (libtrk_amd_base.so) vs + scalar depthwise FMAs
# (libtrk_amd_dws.so): isolated phase stamps, then the pipeline A/B
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_e2e_c3.py -s -q --timeout 380 --timeout-method thread 2>&1 | grep -E "c3 e2e|passed|failed" || exit 1
P=a-lightweight-unsupervised-feature-extractor-_amd
for L in libtrk_amd_base.so libtrk_amd.so libtrk_amd_dws.so; do
  echo "== front_prof $L"
  TRK_LIB_PATH=$PWD/$P/$L timeout -k 10 180 python tools/exp/front_prof.py || exit 1
done
tools/exp/ab3.sh r5b 2 "TRK_LIB_PATH=$PWD/$P/libtrk_amd_base.so" "" "TRK_LIB_PATH=$PWD/$P/libtrk_amd_dws.so"
