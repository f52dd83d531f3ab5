"""roi_align at the bench shape only (for PMC passes): 8 x [512,40,40] NHWC
f32 maps, 8 x 256 ROIs, 10x10 bins, bf16 NHWC output."""
import importlib, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
B, C, H, N, S = 8, 512, 40, 256, 10
feat = torch.from_numpy((lambda x: x / (1 + np.exp(-x)))(rng.standard_normal((B, C, H, H)).astype(np.float32))).to(dev)
w = rng.uniform(32, 320, B * N); h = rng.uniform(32, 320, B * N)
x1 = rng.uniform(-8, 1280 - w + 8); y1 = rng.uniform(272, 1008 - h)
rois = torch.from_numpy(np.stack([np.repeat(np.arange(B), N), x1, y1, x1 + w, y1 + h], 1).astype(np.float32)).to(dev)
nhwc = feat.contiguous(memory_format=torch.channels_last)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    trk.roi_align(nhwc, rois, (S, S), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True)
torch.cuda.synchronize()
print("ok")
