"""Transition GEMM (bench shape M = 204800, K = 1024, N = 512, P = 100) per
enc_gemm mode, interleaved rounds, median per mode.
usage: python tools/exp/trans_lat.py [modes, e.g. 1,2,3] [rounds]"""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
modes = (sys.argv[1] if len(sys.argv) > 1 else "1,2,3").split(",")  # enc_gemm[:enc_gemm_dbg]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
P, M = 100, 204800
R = M // P
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(R, 512, device=dev, generator=g)
L = ops.lib()


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = {m: [] for m in modes}
for _ in range(rounds):
    for m in modes:
        mm, _, dbg = m.partition(":")
        L.trk_set_tuning(b"enc_gemm", int(mm))
        L.trk_set_tuning(b"enc_gemm_dbg", int(dbg or 0))
        res[m].append(timeit(lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True)))
L.trk_set_tuning(b"enc_gemm", 1)
L.trk_set_tuning(b"enc_gemm_dbg", 0)
for m in modes:
    med = statistics.median(res[m])
    print(json.dumps({"mode": m, "median_us": round(med, 1), "min_us": round(min(res[m]), 1),
                      "TF": round(2 * M * 1024 * 512 / med / 1e6, 1)}), flush=True)
