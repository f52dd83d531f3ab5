"""trk_build_cost_dev at the bench's tracking shape (8 streams x 256 tracks x 256
detections, T = 30, gate on): det-tile cost_kernel (no workspace) vs the
bank-resident det_prep + cost3 (workspace).  usage: python tools/exp/cost_bench.py"""
import ctypes, importlib, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
F, M, N, T, S = 8, 256, 256, 30, 8 * 256
g = torch.Generator(device=dev).manual_seed(0)
bank = torch.nn.functional.normalize(torch.randn(S, T, 128, device=dev, generator=g), dim=-1)
blen = torch.full((S,), T, device=dev, dtype=torch.int32)
pbox = torch.rand(S, 4, device=dev, generator=g) * 600
pbox[:, 2:] += pbox[:, :2] + 30
lconf = torch.rand(S, device=dev, generator=g)
gm = torch.rand(S, 4, device=dev, generator=g, dtype=torch.float64) * 600
gs = torch.eye(4, device=dev, dtype=torch.float64).repeat(S, 1, 1).reshape(S, 16) * 1e-3
gon = torch.ones(S, device=dev, dtype=torch.int32)
det = torch.randn(F, N, 128, device=dev, generator=g)
dbox = torch.rand(F, N, 4, device=dev, generator=g) * 600
dbox[..., 2:] += dbox[..., :2] + 30
dconf = torch.rand(F, N, device=dev, generator=g)
Ms = torch.full((F,), M, device=dev, dtype=torch.int32)
Ns = torch.full((F,), N, device=dev, dtype=torch.int32)
slots = torch.arange(S, device=dev, dtype=torch.int32).reshape(F, M)
C = torch.empty(F, M, N, device=dev)
L = trk.lib()
P = ops._ptr
prm = trk.default_cost_params(gate=True)
work = torch.empty(int(L.trk_cost_work_bytes(F, N)), device=dev, dtype=torch.uint8)
prm8 = trk.default_cost_params(gate=True)
prm8.topk = 8   # timing only: cost3's 8-slot top-k network (topk <= 5 runs the 5-slot one)
def run(w, pr=prm):
    assert L.trk_build_cost_dev(F, M, N, P(Ms), P(Ns), P(slots), M, T, P(bank), P(blen), P(pbox), P(lconf), P(gm),
                                P(gs), P(gon), P(det), P(dbox), P(dconf), ctypes.byref(pr), P(C), None,
                                P(w) if w is not None else None, ops._stream(dev)) == 0
for split in (0, 1):
    L.trk_set_tuning(b"cost_split", split)
    for name, w, pr in (("cost_kernel", None, prm), ("cost3", work, prm), ("cost3_topk8", work, prm8)):
        run_ = lambda w: run(w, pr)
        for _ in range(3): run_(w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): run_(w)
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(json.dumps({"split": split, "kernel": name, "us": round(us, 2)}), flush=True)
    prof = torch.zeros(F * ((M + 3) // 4) * 16, dtype=torch.int64, device=dev)
    L.trk_cost_set_prof(P(prof))
    run(work); torch.cuda.synchronize()
    L.trk_cost_set_prof(None)
    pr = prof.view(-1, 4).double().cpu()
    print(json.dumps({"split": split, "prof_ticks_mean": {"bank": round(pr[:, 1].mean().item()),
                                                          "chain_topk": round(pr[:, 2].mean().item()),
                                                          "epilogue": round(pr[:, 3].mean().item())},
                      "tiles": (N + 31) // 32}), flush=True)
L.trk_set_tuning(b"cost_split", 1)
