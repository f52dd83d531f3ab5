"""A/B of the DSC / transition GEMM kernels (gemm8 knob) at the bench shape
(2048 ROIs x 100 rows); prints isolated per-launch times."""
import importlib, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
R, P = 2048, 100
M = R * P
Y2 = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 4
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 4
s = torch.rand(R, 512, device=dev, generator=g)
XRN, _ = ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True)
L = ops.lib()
modes = [x for x in (sys.argv[1:] or ["0", "1:0:0", "1:0:2", "1:0:4", "1:0:8", "1:0:16", "1:1"])]
for mode in modes:
    m8, dbg, off = (mode.split(":") + ["0", "4"])[:3]
    L.trk_set_tuning(b"enc_gemm", int(m8))
    L.trk_set_tuning(b"enc_gemm_dbg", int(dbg))
    L.trk_set_tuning(b"enc_gemm_offset", int(off))
    for name, fn in (("dsc", lambda: ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True)),
                     ("trans", lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(10):
            fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(json.dumps({"mode": mode, "kernel": name, "us": round(us, 1),
                          "tflops": round(2 * M * 1024 * 512 / us / 1e6, 1)}), flush=True)

# g1dw: first 1x1 convs + depthwise (dbg 16 = no depthwise, 32 = 2 K steps only)
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
for impl, dbg, off in ((1, 0, 8), (1, 16, 8), (1, 32, 8)):
    L.trk_set_tuning(b"enc_gemm", impl)
    L.trk_set_tuning(b"enc_gemm_dbg", dbg)
    L.trk_set_tuning(b"enc_gemm_offset", off)
    fn = lambda: ops.enc_g1_dwconv(X, W1, wdw)
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(10):
        fn()
    e1.record(); torch.cuda.synchronize()
    print(json.dumps({"kernel": "g1dw", "impl": impl, "dbg": dbg, "off": off,
                      "us": round(e0.elapsed_time(e1) / 10 * 1e3, 1)}), flush=True)
L.trk_set_tuning(b"enc_gemm_dbg", 0)
L.trk_set_tuning(b"enc_gemm_offset", 8)
L.trk_set_tuning(b"enc_gemm", 1)
