#!/bin/bash
# round 4: trk_lsap_dev split into a 256-column kernel + the bound's kernel (lsap_split)
set -o pipefail
tools/exp/ab_knob.sh r4x "lsap_split=0" "" 3 || exit 1
for f in gpurun_out/r4x_*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t=d['roofline']['tracker_live_us_per_launch']; print(sys.argv[1], d['value'], 'lsap', t['lsap'], 'cost', t['cost'])" "$f"
done
