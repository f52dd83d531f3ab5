"""g1dw under `g1dw` knob values (argv), three launches each, for PMC collection:
rocprofv3 --pmc FETCH_SIZE -- python3 tools/exp/g1_only.py 4 6"""
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
for v in (sys.argv[1:] or ["6"]):
    assert L.trk_set_tuning(b"g1dw", int(v)) == 0
    for _ in range(3):
        ops.enc_g1_dwconv(X, W1, wdw)
torch.cuda.synchronize()
print("ok")
