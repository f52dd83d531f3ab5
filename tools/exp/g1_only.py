"""g1dw old vs g1dw4 (enc_gemm knob), a few launches each, for PMC collection."""
import importlib, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M = 204800
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
L = ops.lib()
dbg = int(sys.argv[1]) if len(sys.argv) > 1 else 0
L.trk_set_tuning(b"enc_gemm_dbg", dbg)
for impl in (0, 1):
    L.trk_set_tuning(b"enc_gemm", impl)
    for _ in range(3):
        ops.enc_g1_dwconv(X, W1, wdw)
torch.cuda.synchronize()
