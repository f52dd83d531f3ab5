"""trans4 variant (trk_set_tuning enc_trans=V) vs the default: the per-ROI sums must be identical.
usage: t4_check.py V"""
import importlib, os, sys
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
ref = ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True, Wtp=Wtp)
assert L.trk_set_tuning(b"enc_trans", int(sys.argv[1])) == 0
out = ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True, Wtp=Wtp)
L.trk_set_tuning(b"enc_trans", 1)
torch.cuda.synchronize()
# (raw partials past a ROI's count are never written: compare the reduced sums)
print("enc_trans", sys.argv[1], "sums identical:",
      bool(torch.equal(ops.enc_sums_reduce(out, P), ops.enc_sums_reduce(ref, P))))
