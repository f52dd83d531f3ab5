#!/bin/bash
# round 4: the SE inside the persistent front (TRK_FRONT_SE) -- pipeline A/B and live times
set -o pipefail
tools/exp/ab_env.sh r4z "TRK_FRONT_SE=0" "TRK_FRONT_SE=1" 4 || exit 1
for f in gpurun_out/r4z_A*.json gpurun_out/r4z_B*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; k=r['kernel_us']; print(sys.argv[1], d['value'], 'front', k.get('enc_rmb_front'), 'se', k.get('enc_se'), 'trans', k.get('enc_gemm_trans'), 'idle', r.get('embed_stream_idle_us_per_step'))" "$f"
done
