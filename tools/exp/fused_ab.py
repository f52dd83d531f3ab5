"""rmb_fused (one kernel: front + SE + transition) vs rmb_front -> enc_se -> transition GEMM
at the bench shape (2048 ROIs): interleaved timing rounds, medians (HIP events on the current
stream).  usage: python tools/exp/fused_ab.py [R]"""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = R * 100, 100
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
Wtp = ops.enc_pack_fragments_k(Wt)
bt = torch.randn(512, device=dev, generator=g) / 10
sw1, sb1 = torch.randn(128, 512, device=dev, generator=g) / 22, torch.randn(128, device=dev, generator=g) / 10
sw2, sb2 = torch.randn(512, 128, device=dev, generator=g) / 11, torch.randn(512, device=dev, generator=g) / 10


def fused():
    return ops.enc_rmb_fused(X, W1p, wdw, W2p, b2, Wtp, bt, sw1, sb1, sw2, sb2)


def separate():
    XRN, sums = ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
    m_r, m_n, s = ops.enc_se(sums, P, sw1, sb1, sw2, sb2)
    return m_r, m_n, s, ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True)


def front():
    return ops.enc_rmb_front(X, W1p, wdw, W2p, b2)


fns = {"fused": fused, "separate": separate, "front_only": front}
res = {k: [] for k in fns}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for f in fns.values():
    f()
for rnd in range(8):
    for k in (list(fns) if rnd % 2 == 0 else list(fns)[::-1]):
        ev[0].record()
        for _ in range(5):
            fns[k]()
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 1000 / 5)
print(json.dumps({k: {"median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1)} for k, v in res.items()}),
      flush=True)
