"""Encoder pieces at the bench shape (for PMC passes): dwconv5 bf16 on
[2048,10,10,1024], act_mean, scale_rows."""
import importlib, os, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda:0")
K = 2048
y1 = torch.randn(K, 10, 10, 1024, device=dev).bfloat16()
w = torch.randn(25, 1024, device=dev)
xr = torch.randn(K, 100, 512, device=dev).bfloat16()
s = torch.rand(K, 512, device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    ops.dwconv5_nhwc(y1, w)
    ops.act_mean(xr, "silu")
    ops.scale_rows(xr, s)
torch.cuda.synchronize()
print("ok")
