#!/bin/bash
# round 5: the ROI stream at high priority (it sits on the step's critical chain under the
# overlap: front f -> ROI f+1 -> front f+1) vs normal; four interleaved rounds
set -o pipefail
tools/exp/ab3.sh r5k 4 "" "TRK_ROI_PRIO=1"
