"""rmb_fused phase cycles (s_memtime stamps per wave, trk_enc_set_prof): slot 0 = kernel
start -> tail (GEMM1, depthwise, GEMM2, activation); reinforce group: y image + m_r, flag
wait, CYF wait + ring issue, FC1, FC2, y scaling, GEMM3 + epilogue; normal group: staging,
XN copy (sc1), publish.  Medians over workgroups, per wave.  Also interleaved timings of
the fused kernel and rmb_front alone.  usage: python tools/exp/fused_prof.py [variant ...]"""
import ctypes, importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
R = 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(R * 100, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
Wtp = ops.enc_pack_fragments_k((torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16())
bt = torch.randn(512, device=dev, generator=g) / 10
sw1, sb1 = torch.randn(128, 512, device=dev, generator=g) / 22, torch.randn(128, device=dev, generator=g) / 10
sw2, sb2 = torch.randn(512, 128, device=dev, generator=g) / 11, torch.randn(512, device=dev, generator=g) / 10
L = ops.lib()
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
nwg = (2 * R + 15) // 16 * 16
buf = torch.zeros(nwg * 8 * 8, dtype=torch.int64, device=dev)
fused = lambda: ops.enc_rmb_fused(X, W1p, wdw, W2p, b2, Wtp, bt, sw1, sb1, sw2, sb2)
front = lambda: ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
res = {"fused": [], "front": []}
for f in (fused, front):
    f()
for rnd in range(6):
    for k, f in (("fused", fused), ("front", front)) if rnd % 2 == 0 else (("front", front), ("fused", fused)):
        ev[0].record()
        for _ in range(5):
            f()
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) * 200)
print(json.dumps({k: round(statistics.median(v), 1) for k, v in res.items()}), flush=True)
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
fused()
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
p = buf.view(nwg // 2, 2, 8, 8)[:R].double().cpu()  # [roi][group][wave][slot]
names_r = ["to_tail", "mr_pub_y_image", "xn_flag_ring", "gemm3_xn", "s_flag_wait", "scale", "gemm3_xf", "epilogue"]
names_n = ["to_tail", "staging", "xn_copy_publish", "mr_wait_load", "fc1", "fc2_publish", "-", "-"]
for gi, names in ((0, names_r), (1, names_n)):
    med = p[:, gi].median(0).values  # [wave][slot]
    print(json.dumps({"group": "reinforce" if gi == 0 else "normal",
                      "wave0": {n: round(x) for n, x in zip(names, med[0].tolist())},
                      "wave4": {n: round(x) for n, x in zip(names, med[4].tolist())},
                      "total_wave0": round(float(p[:, gi, 0].sum(1).median()))}), flush=True)
