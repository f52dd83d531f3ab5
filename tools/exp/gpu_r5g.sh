#!/bin/bash
# round 5: the persistent front's free-CU split under the two-stream overlap: 14 pairs per XCD
# (default) vs 13 and 15, three interleaved rounds
set -o pipefail
tools/exp/ab3.sh r5g 3 "" "TRK_TUNE=rf3_groups=13" "TRK_TUNE=rf3_groups=15"
