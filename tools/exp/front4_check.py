"""rmb_front4 (rf_front 4) vs rmb_front3: XRN / means at R ROIs, and timing.  usage: front4_check.py [R]"""
import importlib, json, os, sys, statistics
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(R * 100, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
L = ops.lib()
def run(front):
    assert L.trk_set_tuning(b"rf_front", front) == 0
    out = ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(5):
        ev[0].record()
        for _ in range(3):
            ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / 3)
    L.trk_set_tuning(b"rf_front", 3)
    return out, statistics.median(ts)
ref, t3 = run(3)
out, t4 = run(4)
d = {"R": R, "front3_us": round(t3, 1), "front4_us": round(t4, 1), "xrn_equal": bool(torch.equal(out[0], ref[0])),
     "xrn_maxdiff": float((out[0].float() - ref[0].float()).abs().max()),
     "means_maxdiff": max(float((out[i] - ref[i]).abs().max()) for i in (1, 2))}
print(json.dumps(d), flush=True)
