#!/bin/bash
# round 5: 32x32x16 MFMA variants -- trans5 (enc_trans 2) and rmb_front3<32> (rf_mfma 32): their
# parity tests, isolated A/B with phase stamps, then pipeline A/B/C/D (two interleaved rounds)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "trans or rmb_front" --timeout 120 \
  --timeout-method thread 2>&1 | tail -4 || exit 1
timeout -k 10 120 python tools/exp/trans_ab.py || exit 1
timeout -k 10 180 python tools/exp/front_prof.py "" "rf_mfma=32" || exit 1
tools/exp/ab3.sh r5f 2 "" "TRK_TUNE=enc_trans=2" "TRK_TUNE=rf_mfma=32" "TRK_TUNE=enc_trans=2,rf_mfma=32"
