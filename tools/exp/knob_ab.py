"""Encoder kernel under trk_set_tuning variants, interleaved rounds, medians, and the
outputs compared with the first variant's.  usage:
  python tools/exp/knob_ab.py dsc "enc_gemm_split=0" "enc_gemm_split=1"
kernel: g1dw | dsc | trans; a variant is "k=v;k=v" ("" = defaults)."""
import importlib, json, os, statistics, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
kern, variants = sys.argv[1], sys.argv[2:]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = 204800, 100
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
Y2 = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 10
XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(M // P, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
# outputs compared: Y2 / XRN + the reduced ROI sums (raw partial buffers hold unused slots)
fn = {"g1dw": lambda: ops.enc_g1_dwconv(X, W1, wdw),
      "dsc": lambda: ops.enc_dsc_gemm(Y2, P, W2, b2),
      "trans": lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt)}[kern]
L = ops.lib()
defaults = {}


def apply(v, reset=False):
    for kv in filter(None, v.split(";")):
        k, x = kv.split("=")
        if reset:
            L.trk_set_tuning(k.encode(), defaults[k])
        else:
            L.trk_set_tuning(k.encode(), int(x))


for v in variants:  # the defaults to restore: every knob's first-listed value in variant 0, else 0
    for kv in filter(None, v.split(";")):
        k, x = kv.split("=")
        defaults.setdefault(k, {"enc_trans": 1, "rf3_chunks": 1}.get(k, 0))
ref = None
for v in variants:
    apply(v)
    out = fn(); torch.cuda.synchronize()
    o = out if isinstance(out, torch.Tensor) else torch.cat([t.flatten().float() for t in out])
    if ref is None:
        ref = o.clone()
    d = (o.double() - ref.double()).abs().flatten()
    print(json.dumps({"variant": v, "identical_to_first": bool(torch.equal(o, ref)),
                      "max_abs_diff": d.max().item(), "n_diff": int((d > 0).sum().item()),
                      "first_diff": int((d > 0).nonzero()[0].item()) if bool((d > 0).any()) else -1,
                      "numel": o.numel()}), flush=True)
    apply(v, reset=True)
res = {v: [] for v in variants}
for rnd in range(8):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        apply(v)
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): fn()
        e1.record(); torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        apply(v, reset=True)
for v in variants:
    print(json.dumps({"kernel": kern, "variant": v, "median_us": round(statistics.median(res[v]), 1),
                      "min_us": round(min(res[v]), 1)}), flush=True)
