"""gemm4 (default encoder GEMM) per-workgroup phase stamps for DSC and the transition
at the bench shape: [K loop, activation, ROI sums, staging + barrier, sums stores,
output stores drained], mean ticks per tile (trk_enc_set_prof)."""
import importlib, json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = 204800, 100
Y2 = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 10
XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(M // P, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
L = ops.lib()
names = ["kloop", "act", "sums", "stage_bar", "sums_st", "stores", "total"]
for name, fn, ntile in (("dsc", lambda: ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True), M // 128 * 2 * 2),
                        ("trans", lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True), M // 128 * 2)):
    fn(); torch.cuda.synchronize()
    buf = torch.zeros(ntile * 8, dtype=torch.int64, device=dev)
    L.trk_enc_set_prof(ops._ptr(buf)); fn(); torch.cuda.synchronize(); L.trk_enc_set_prof(None)
    b = buf.view(ntile, 8)[:, :7].double()
    print(json.dumps({"kernel": name, "mean_ticks": dict(zip(names, [round(x) for x in b.mean(0).tolist()]))}), flush=True)
