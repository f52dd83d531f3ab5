"""Isolated A/B of the transition GEMM variants at the bench shape (2,048 ROIs x 100 rows,
K 1,024, N 512): gemm4 (128 x 256, weights through LDS), gemm4 wide (enc_trans_wide 1:
256 x 256, 8 waves) and trans4 (enc_trans 1: weights straight into VGPRs), interleaved
rounds of 10 launches, medians.  usage: python tools/exp/trans_ab.py"""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R, P = 2048, 100
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
XRN = torch.randn(R * P, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(R, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 4
Wtp = ops.enc_pack_fragments_k(Wt)
L = ops.lib()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
VARS = {"gemm4": (0, 0, 0), "t4_mid": (0, 1, 5), "t4_mid_asm": (0, 1, 8), "t4_2x3_mid_asm": (0, 1, 9)}
res = {k: [] for k in VARS}
outs = {}


def setv(k):
    L.trk_set_tuning(b"enc_trans_wide", VARS[k][0])
    L.trk_set_tuning(b"enc_trans", VARS[k][1])
    L.trk_set_tuning(b"t4_mode", VARS[k][2])


for k in VARS:
    setv(k)
    outs[k] = ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
names = list(VARS)
for rnd in range(8):
    for k in (names if rnd % 2 == 0 else names[::-1]):
        setv(k)
        ev[0].record()
        for _ in range(10):
            ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 100)
setv("t4_mid")
print(json.dumps({"us": {k: round(statistics.median(v), 1) for k, v in res.items()},
                  "all": {k: [round(x, 1) for x in v] for k, v in res.items()},
                  "identical": all(torch.equal(outs[k], outs["gemm4"]) for k in VARS)}), flush=True)
