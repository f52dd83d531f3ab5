"""trans4 phase cycles per workgroup (s_memtime stamps of wave 0, trk_enc_set_prof): K loop,
SiLU, ROI sums (MFMA), sum stores, total; medians over the 3,200 tiles of the bench shape.
usage: python tools/exp/t4_prof.py"""
import ctypes, importlib, json, os, sys
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
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
for kv in sys.argv[1:]:  # tuning knobs k=v
    k, v = kv.split("=")
    assert L.trk_set_tuning(k.encode(), int(v)) == 0
nwg = (R * P + 127) // 128 * 2
buf = torch.zeros(nwg * 8, dtype=torch.int64, device=dev)
for _ in range(3):
    ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
med = buf.view(nwg, 8)[:, :5].double().cpu().median(0).values.tolist()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(10):
    ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
ev[1].record()
torch.cuda.synchronize()
print(json.dumps({"args": sys.argv[1:], "us": round(ev[0].elapsed_time(ev[1]) * 100, 1), "k_loop": round(med[0]), "silu": round(med[1]), "sums": round(med[2]), "store": round(med[3]),
                  "total": round(med[4])}), flush=True)
