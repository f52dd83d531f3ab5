"""trans_front (one ROI per workgroup) vs gemm4<TRANS> at the bench shape: reduced sums
compared, then interleaved timing rounds (medians).  usage: python tools/exp/trans_ab.py [R]"""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
XRN = torch.randn(R * 100, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(R, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 4
Wtp = ops.enc_pack_fragments_nk(Wt)
fns = {"gemm4": lambda: ops.enc_transition_gemm(XRN, 100, s, Wt, bt, raw=True),
       "trans_roi": lambda: ops.enc_transition_roi(XRN, s, Wtp, bt)}
a, b = (ops.enc_sums_reduce(f(), 100) for f in fns.values())
print(json.dumps({"max_rel_diff": ((a - b).abs().max() / a.abs().max()).item()}), flush=True)
res = {k: [] for k in fns}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for rnd in range(10):
    for k in (list(fns) if rnd % 2 == 0 else list(fns)[::-1]):
        fns[k]()
        ev[0].record()
        for _ in range(5):
            fns[k]()
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 200)
print(json.dumps({k: {"median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1)} for k, v in res.items()}))
