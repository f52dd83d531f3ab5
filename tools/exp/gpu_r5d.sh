#!/bin/bash
# round 5: the two-embedding-stream overlap (frame f+1's encoder gated only behind frame f's
# front) against HEAD's one embedding stream, four interleaved pipeline pairs, after the c3
# end-to-end chain test under the overlap setting
set -o pipefail
TRK_EMBED_STREAMS=2 TRK_EMBED_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests/test_e2e_c3.py -m gpu -x -q \
  --timeout 240 --timeout-method thread -s 2>&1 | tail -4 || exit 1
tools/exp/ab3.sh r5d 4 "" "TRK_EMBED_STREAMS=2 TRK_EMBED_OVERLAP=1"
