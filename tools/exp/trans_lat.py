import importlib, json, os, sys
import torch
sys.path.insert(0, "/root/repo" if os.path.exists("/root/repo") else os.environ["GRAFT_REPO_ROOT"])
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
P = 100
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
L = ops.lib()
def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
for M in (204800, 51200, 20480):
    R = M // P
    XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
    s = torch.rand(R, 512, device=dev, generator=g)
    for mode in (1, 2):
        L.trk_set_tuning(b"enc_gemm", mode)
        t = timeit(lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True))
        print(json.dumps({"M": M, "mode": mode, "us": round(t, 1), "ns_per_row": round(t * 1e3 / M, 3), "TF": round(2 * M * 1024 * 512 / t / 1e6, 1)}), flush=True)
L.trk_set_tuning(b"enc_gemm", 1)
