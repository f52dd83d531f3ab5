"""rmb_front3 phase timeline of one workgroup pair (trk_enc_set_prof: per ROI and wave the 7 phase
durations and the ROI's absolute s_memtime start): for the pair's first workgroups (group 0 and
group 1 of XCD 0, pair 0) prints, for SIMD 0's two waves (wave 0: half A, wave 4: half B), every
ROI's phase start times relative to the pair's first ROI, so waits between the halves show as
phases that start late.  usage: python tools/exp/front_timeline.py [rois]"""
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
# the pair's ROIs: xcd 0, pair 0 -> ROIs 0, 8 P, 16 P, ... with P pairs per XCD (stride 8 P)
starts = p[:, 0, 0, 7]
P = None
for cand in range(1, 65):
    if R > 8 * cand and starts[8 * cand] > starts[0]:
        # the pair's next ROI starts after its first one ends (same workgroup), the neighbours' do not
        d = int(starts[8 * cand] - starts[0])
        if abs(d - int(p[0, 0, 0, :7].sum())) < 0.25 * int(p[0, 0, 0, :7].sum()):
            P = cand
            break
rois = [8 * (P or 14) * k for k in range(nroi)]
t0 = int(p[rois[0], 0, 0, 7])
for gi in (0, 1):
    for w in (0, 4):
        rows = []
        for r in rois:
            st = int(p[r, gi, w, 7]) - t0
            acc, ph = st, {}
            for k, n in enumerate(names):
                ph[n] = acc
                acc += int(p[r, gi, w, k])
            ph["end"] = acc
            rows.append(ph)
        print(json.dumps({"group": gi, "wave": w, "pairs_per_xcd": P, "rois": rows}), flush=True)
