"""Encoder GEMM time breakdown at the bench shape (M = 204800 rows, 2048 ROIs of
10x10): each fused kernel with parts of its work switched off through the
enc_gemm_dbg knob.  g1dw: 16 = no depthwise phase, 32 = K loop of 2 steps, 256 = depthwise without the Y2 stores.
gemm4: 1 = no epilogue, 2 = no stores, 4 = no ROI sums.  One JSON line each."""
import importlib, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = 204800, 100
R = M // P
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
Y2 = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 10
XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(R, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
L = ops.lib()
only = sys.argv[1] if len(sys.argv) > 1 else "all"


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


items = {
    "g1dw": (lambda: ops.enc_g1_dwconv(X, W1, wdw), [0, 256, 16, 32, 48, 16 | 64, 16 | 128, 16 | 64 | 128],
             2 * M * 512 * 1024),
    "plain256": (lambda: ops.enc_gemm(X, W1), [0], 2 * M * 512 * 1024),
    "dsc": (lambda: ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True), [0, 1, 2, 4], 2 * M * 1024 * 512),
    "trans": (lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True), [0, 1, 4], 2 * M * 1024 * 512),
}
offsets = [int(v) for v in os.environ.get("ENC_OFFSETS", "0").split(",")]
g1p = [int(v) for v in os.environ.get("G1P", "0").split(",")]
g1m = [int(v) for v in os.environ.get("G1M", "0").split(",")]   # g1dw_mode: DMA placement
for name, (fn, dbgs, flops) in items.items():
    if only != "all" and name not in only.split(","):
        continue
    for off in ([p * 10 + m for p in g1p for m in g1m] if name == "g1dw" else offsets):
        if name == "g1dw":
            L.trk_set_tuning(b"g1dw_persist", off // 10)
            L.trk_set_tuning(b"g1dw_mode", off % 10)
        else:
            L.trk_set_tuning(b"enc_gemm_offset", off)
        if os.environ.get("ENC_DBGS"):
            dbgs = [int(v) for v in os.environ["ENC_DBGS"].split(",")]
        for d in (dbgs if not os.environ.get("ENC_DBG0") else [0]):
            L.trk_set_tuning(b"enc_gemm_dbg", d)
            t = timeit(fn)
            print(json.dumps({"item": name, "offset": off, "dbg": d, "us": round(t, 1),
                              "TFLOPs": round(flops / t / 1e6, 1)}), flush=True)
L.trk_set_tuning(b"enc_gemm_dbg", 0)
L.trk_set_tuning(b"enc_gemm_offset", 0)
L.trk_set_tuning(b"g1dw_persist", 0)
L.trk_set_tuning(b"g1dw_mode", 7)
torch.cuda.synchronize()
