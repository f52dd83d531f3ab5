#!/bin/bash
# round 4: knobs around the persistent front (rf_v 3 default): prefetch off, lag, groups
set -o pipefail
tools/exp/ab_knob.sh r4t_pf "" "rf_pf=0" 4 || exit 1
tools/exp/ab_knob.sh r4t_lag "" "rf_lag=8" 3 || exit 1
tools/exp/ab_knob.sh r4t_g13 "" "rf3_groups=13" 3
