"""A/B of one encoder kernel between two builds of libtrk_amd.so in one process
(interleaved rounds, medians).  usage: python tools/exp/ab_lib.py OLD.so [kernel]
kernel: g1dw (default) | dsc | trans"""
import ctypes, importlib, json, os, statistics, sys
import torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
new = ops.lib()
old = ctypes.CDLL(os.path.abspath(sys.argv[1]))
kern = sys.argv[2] if len(sys.argv) > 2 else "g1dw"
P_, i64 = ctypes.c_void_p, ctypes.c_int64
for L in (new, old):
    L.trk_enc_g1_dwconv.argtypes = [P_, i64, P_, i64, P_, P_, P_]
    L.trk_enc_dsc_gemm.argtypes = [P_, i64, i64, i64, P_, P_, i64, P_, P_, P_]
    L.trk_enc_transition_gemm.argtypes = [P_, i64, i64, i64, P_, i64, P_, P_, i64, P_, P_]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
M, P = 204800, 100
X = torch.randn(M, 512, device=dev, generator=g).bfloat16()
W1 = (torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16()
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
Y2 = torch.empty(M, 1024, device=dev, dtype=torch.bfloat16)
W2 = (torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16()
b2 = torch.randn(1024, device=dev, generator=g) / 10
XRN = torch.empty(M, 1024, device=dev, dtype=torch.bfloat16)
sums = torch.empty(M // P, 3, 1024, device=dev, dtype=torch.int64)
s = torch.rand(M // P, 512, device=dev, generator=g)
Wt = (torch.randn(512, 1024, device=dev, generator=g) / 32).bfloat16()
bt = torch.randn(512, device=dev, generator=g) / 10
ts = torch.empty(M // P, 3, 512, device=dev, dtype=torch.int64)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call(L):
    if kern == "g1dw":
        return L.trk_enc_g1_dwconv(p(X), M, p(W1), 1024, p(wdw), p(Y2), st())
    if kern == "dsc":
        return L.trk_enc_dsc_gemm(p(Y2), M, P, 512, p(W2), p(b2), 512, p(XRN), p(sums), st())
    return L.trk_enc_transition_gemm(p(XRN), M, P, 1024, p(s), 512, p(Wt), p(bt), 512, p(ts), st())


outs = {}
for name, L in (("new", new), ("old", old)):
    assert call(L) == 0
    torch.cuda.synchronize()
    outs[name] = (Y2 if kern == "g1dw" else XRN if kern == "dsc" else ts).clone()
print(json.dumps({"identical": bool(torch.equal(outs["new"], outs["old"]))}), flush=True)
res = {"new": [], "old": []}
for rnd in range(8):
    for name, L in ((("new", new), ("old", old)) if rnd % 2 == 0 else (("old", old), ("new", new))):
        call(L); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): call(L)
        e1.record(); torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
for name in res:
    print(json.dumps({"kernel": kern, "lib": name, "median_us": round(statistics.median(res[name]), 1),
                      "min_us": round(min(res[name]), 1)}), flush=True)
