"""ROI Align at the bench shape (8 frames x 256 ROIs, 512x40x40 maps, 10x10
bins, NHWC bf16 out) under tuning-knob variants, interleaved rounds, median.
usage: python tools/exp/roi_ab.py "roi_wlds=0" "roi_wlds=1" ..."""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
F, K = 8, 256
feat = torch.randn(F, 512, 40, 40, device=dev, generator=g)
if os.environ.get("ROI_LAYOUT", "nhwc") == "nhwc":
    feat = feat.contiguous(memory_format=torch.channels_last)
xy = torch.rand(F * K, 2, device=dev, generator=g) * 1100
wh = 20 + torch.rand(F * K, 2, device=dev, generator=g) * 300
rois = torch.cat([torch.arange(F, device=dev).repeat_interleave(K)[:, None].float(), xy, xy + wh], 1)
L = trk.lib()
variants = sys.argv[1:] or ["roi_wlds=0", "roi_wlds=1"]


DEFAULTS = {"roi_wlds": 1, "roi_sweep": 1, "roi_fma": 1, "roi_asm": 1}


def setv(v, reset=False):
    for kv in v.split(","):
        k, x = kv.split("=")
        L.trk_set_tuning(k.encode(), DEFAULTS[k] if reset else int(x))


def run():
    return trk.roi_align(feat, rois, (10, 10), 40 / 1280.0, 2, True, out_dtype=torch.bfloat16, channels_last=True)


print("layout", os.environ.get("ROI_LAYOUT", "nhwc"))


ref = run()
res = {v: [] for v in variants}
diff = {}
for _ in range(8):
    for v in variants:
        setv(v)
        out = run(); torch.cuda.synchronize()
        if not torch.equal(out, ref):
            d = (out.view(torch.int16).int() - ref.view(torch.int16).int()).abs()
            diff[v] = (int((d > 0).sum()), int(d.max()), out.numel())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): run()
        e1.record(); torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        setv(v, reset=True)
for v in variants:
    print(json.dumps({"variant": v, "median_us": round(statistics.median(res[v]), 1), "min_us": round(min(res[v]), 1),
                      "bf16_diff_vs_first (n, max_ulp, numel)": diff.get(v)}))
