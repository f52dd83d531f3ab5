"""Encoder forward at the bench shape (bf16, 2048 ROIs of 10x10), for rocprof."""
import importlib, os, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden")]
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
import gen_common as G
dev = torch.device("cuda:0")
model = trk.Model(512, 512, 10, 128).eval()
model.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}, strict=True)
model = model.to(dev)
x = torch.randn(2048, 512, 10, 10, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
        model(x)
torch.cuda.synchronize()
print("ok")
