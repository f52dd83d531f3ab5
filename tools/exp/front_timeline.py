"""rmb_front3 phase timeline of one workgroup pair (trk_enc_set_prof: per ROI and wave the 7 phase
durations and the ROI's absolute s_memtime start): for the pair's first workgroups (group 0 and
group 1 of XCD 0, pair 0) prints, for SIMD 0's two waves (wave 0: half A, wave 4: half B), every
ROI's phase start times relative to the pair's first ROI, so waits between the halves show as
phases that start late.  usage: python tools/exp/front_timeline.py [rois] [pairs_per_xcd]"""
import ctypes, importlib, json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(R * 100, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
L = ops.lib()
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
buf = torch.zeros(2 * R * 8 * 8, dtype=torch.int64, device=dev)
for _ in range(3):
    ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
p = buf.view(R, 2, 8, 8).cpu()
names = ["gemm1", "y1", "dw", "gemm2", "act", "stage", "store"]
nroi = int(sys.argv[1]) if len(sys.argv) > 1 else 6
# the pair's ROIs: xcd 0, pair 0 -> ROIs 0, 8 P, 16 P, ... with P pairs per XCD (stride 8 P;
# rf3_groups 0: CUs / 16 - 2 = 14 on 256 CUs)
P = int(sys.argv[2]) if len(sys.argv) > 2 else torch.cuda.get_device_properties(0).multi_processor_count // 16 - 2
rois = [8 * P * k for k in range(nroi)]
M56 = (1 << 56) - 1
p = p.clone()
xcc = p[..., 7] >> 56
p[..., 7] = p[..., 7] & M56                 # ROI start, 100 MHz ticks (10 ns)
t0 = int(p[rois[0], 0, 0, 7])
for gi in (0, 1):
    for w in (0, 4):
        rows = [{"start_us": round((int(p[r, gi, w, 7]) - t0) / 100, 2), "xcc": int(xcc[r, gi, w]),
                 **{n: int(p[r, gi, w, k]) for k, n in enumerate(names)}} for r in rois]
        print(json.dumps({"group": gi, "wave": w, "pairs_per_xcd": P, "rois": rows}), flush=True)
# every pair: |start(group 0) - start(group 1)| of the same ROI (wave 0 of each), us, whether the
# two workgroups share an XCD, and the ROI period (start of ROI k + 8 P minus ROI k, same workgroup)
st = p[:, :, 0, 7].double() / 100
lag = (st[:, 0] - st[:, 1]).abs()
per = st[8 * P:, 0] - st[:-8 * P, 0]
q = lambda t, f: round(float(t.quantile(f)), 2)
print(json.dumps({"pair_lag_us": {"p50": q(lag, 0.5), "p90": q(lag, 0.9), "max": round(float(lag.max()), 2)},
                  "same_xcd": float((xcc[:, 0, 0] == xcc[:, 1, 0]).double().mean()),
                  "roi_period_us": {"p50": q(per, 0.5), "p10": q(per, 0.1), "p90": q(per, 0.9)}}), flush=True)
