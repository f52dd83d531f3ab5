"""rmb_front (one kernel: first 1x1 convs + depthwise + DSC GEMMs, Y2 in LDS) vs the
two-kernel path (g1dw4 -> Y2 in HBM -> gemm4<DSC>) at the bench shape (2048 ROIs):
outputs compared (XRN bit for bit, reduced ROI sums), then interleaved timing rounds
(medians, HIP events on the current stream).  usage: python tools/exp/front_ab.py [R]"""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = R * 100, 100
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 10
W1p, W2p = ops.enc_pack_fragments(W1), ops.enc_pack_fragments(W2)


def two():
    Y2 = ops.enc_g1_dwconv(X, W1, wdw)
    return ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True)


def one():
    return ops.enc_rmb_front(X, W1p, wdw, W2p, b2)


x2, s2 = two()
x1, s1 = one()
torch.cuda.synchronize()
f2, f1 = ops.enc_sums_reduce(s2, P), ops.enc_sums_reduce(s1, P)
d = (x1.float() - x2.float()).abs()
print(json.dumps({"xrn_identical": bool(torch.equal(x1, x2)), "xrn_n_diff": int((d > 0).sum().item()),
                  "xrn_max_abs_diff": d.max().item(),
                  "sums_max_rel_diff": ((f1 - f2).abs().max() / f2.abs().max()).item()}), flush=True)
res = {"two_kernel": [], "rmb_front": []}
fns = {"two_kernel": two, "rmb_front": one}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for rnd in range(10):
    for k in (list(fns) if rnd % 2 == 0 else list(fns)[::-1]):
        fns[k]()
        ev[0].record()
        for _ in range(5):
            fns[k]()
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 1000 / 5)
print(json.dumps({k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in res.items()}), flush=True)
