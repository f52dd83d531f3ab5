#!/bin/bash
# round 4: the front writing the squeeze means (TRK_FRONT_MEANS) -- parity, then pipeline A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "rmb_front or se_head or fused_tail" > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -1 gpurun_out/r4m_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "chain or e2e or encoder or smoke or pipeline" > gpurun_out/r4m_tests2.log 2>&1 || { tail -30 gpurun_out/r4m_tests2.log; exit 1; }
tail -1 gpurun_out/r4m_tests2.log
tools/exp/ab_env.sh r4mab "TRK_FRONT_MEANS=0" "TRK_FRONT_MEANS=1" 4 || exit 1
for f in gpurun_out/r4mab_A*.json gpurun_out/r4mab_B*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; k=r['kernel_us']; print(sys.argv[1], d['value'], 'front', k.get('enc_rmb_front'), 'se', k.get('enc_se'), 'trans', k.get('enc_gemm_trans'), 'idle', r.get('embed_stream_idle_us_per_step'))" "$f"
done
