#!/bin/bash
# round 5: the ROI stage's placement under the two-stream overlap: gated behind the previous
# front (default) vs ungated (runs beside the front on the CUs it leaves free) vs the NCHW
# transpose two frames ahead on the tracker's stream; three interleaved rounds
set -o pipefail
tools/exp/ab3.sh r5j 3 "" "TRK_ROI_AFTER=" "TRK_MAP_AHEAD=1"
