#!/bin/bash
# round 4: persistent front with CUs left free for the tracker / ROI streams (rf3_groups)
set -o pipefail
tools/exp/ab_knob.sh r4r14 "rf_v=2" "rf_v=3,rf3_groups=14" 4 || exit 1
tools/exp/ab_knob.sh r4r15 "rf_v=2" "rf_v=3,rf3_groups=15" 3
tools/exp/ab_knob.sh r4r32 "rf_v=2" "rf_v=3,rf3_groups=32" 3
