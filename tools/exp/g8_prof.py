"""gemm8 (enc_gemm=2) transition: per-workgroup timestamp breakdown (trk_enc_set_prof)."""
import importlib, json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
P, M = 100, 204800
R = M // P
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
XRN = torch.randn(M, 1024, device=dev, generator=g).bfloat16()
s = torch.rand(R, 512, device=dev, generator=g)
L = ops.lib()
L.trk_set_tuning(b"enc_gemm", 2)
nwg = (M + 255) // 256 * 2
buf = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
f = lambda: ops.enc_transition_gemm(XRN, P, s, Wt, bt, raw=True)
for _ in range(3): f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); f(); e1.record(); torch.cuda.synchronize()
t_plain = e0.elapsed_time(e1) * 1e3
L.trk_enc_set_prof(ops._ptr(buf))
e0.record(); f(); e1.record(); torch.cuda.synchronize()
t_prof = e0.elapsed_time(e1) * 1e3
L.trk_enc_set_prof(None)
L.trk_set_tuning(b"enc_gemm", 1)
b = buf.view(nwg, 2, 8).cpu().double()
t0, t1, t2, t3, w, br = (b[..., i] for i in range(6))
span = t3.max() - t0.min()
out = {"us_plain": round(t_plain, 1), "us_prof": round(t_prof, 1), "span_ticks": span.item(),
       "ticks_per_us": round(span.item() / t_prof, 1)}
for name, v in (("prologue", t1 - t0), ("kloop", t2 - t1), ("epilogue", t3 - t2), ("wait_vm", w), ("wait_bar", br), ("total", t3 - t0)):
    out[name] = {"mean": round(v.mean().item(), 0), "p10": round(v.quantile(0.1).item(), 0), "p90": round(v.quantile(0.9).item(), 0)}
# workgroups by start order: rounds of residency
st = (t0[:, 0] - t0.min()).sort().values
out["start_quantiles"] = [round(st[int(q * (nwg - 1))].item(), 0) for q in (0, .1, .2, .3, .4, .5, .6, .7, .8, .9, 1)]
print(json.dumps(out), flush=True)
