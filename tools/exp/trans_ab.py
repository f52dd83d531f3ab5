"""Isolated A/B of the transition kernels at the bench shape (2,048 ROIs x 100 rows, K 1,024,
N 512): trans4 (enc_trans 1: 16x16x32 MFMAs) and trans5 (enc_trans 2: 32x32x16), interleaved
rounds of 10 launches, medians; then each one's per-tile phase cycles (trk_enc_set_prof stamps
of wave 0: K loop, SiLU, sums, sum stores, total; medians over the 3,200 tiles) and the largest
difference of their sums.  usage: python tools/exp/trans_ab.py"""
import ctypes, importlib, json, os, statistics, sys
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
VARS = {"trans4": 1, "trans5": 2}
res = {k: [] for k in VARS}
outs = {}
for k, v in VARS.items():
    L.trk_set_tuning(b"enc_trans", v)
    outs[k] = ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
names = list(VARS)
for rnd in range(8):
    for k in (names if rnd % 2 == 0 else names[::-1]):
        L.trk_set_tuning(b"enc_trans", VARS[k])
        ev[0].record()
        for _ in range(10):
            ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 100)  # us per launch
top = outs["trans4"].abs().max().item()
print(json.dumps({k: round(statistics.median(v), 1) for k, v in res.items()}
                 | {"max_rel_diff": (outs["trans5"] - outs["trans4"]).abs().max().item() / top}), flush=True)
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
nwg = (R * P + 127) // 128 * 2
buf = torch.zeros(nwg * 8, dtype=torch.int64, device=dev)
for k, v in VARS.items():
    L.trk_set_tuning(b"enc_trans", v)
    L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
    ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
    torch.cuda.synchronize()
    L.trk_enc_set_prof(None)
    p = buf.view(nwg, 8)[:, :5].double().cpu()
    med = p.median(0).values.tolist()
    print(json.dumps({"kernel": k, "k_loop": round(med[0]), "silu": round(med[1]), "sums": round(med[2]),
                      "store": round(med[3]), "total": round(med[4])}), flush=True)
L.trk_set_tuning(b"enc_trans", 1)
