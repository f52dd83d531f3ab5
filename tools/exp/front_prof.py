"""rmb_front phase cycles (s_memtime stamps of wave 0 per workgroup, trk_enc_set_prof):
GEMM1, Y1 -> LDS, depthwise, GEMM2, activation + sums, output staging, stores, total."""
import importlib, json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(R * 100, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
L = ops.lib()
buf = torch.zeros(2 * R * 8, dtype=torch.int64, device=dev)
for _ in range(3):
    ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
import ctypes
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
p = buf.view(-1, 8).double().cpu()
names = ["gemm1", "y1_store", "depthwise", "gemm2", "act_sums", "staging", "stores", "total"]
med = p.median(0).values.tolist()
print(json.dumps({n: round(v) for n, v in zip(names, med)}), flush=True)
# s_memtime counts at 100 MHz on gfx950? report the ratio to the total
print(json.dumps({n: round(v / med[-1], 3) for n, v in zip(names, med)}), flush=True)
