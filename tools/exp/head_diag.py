"""enc_head variants (head_waves 16 / 8) on the same inputs: max difference vs the
16-wave kernel, and which rows / columns differ (diagnostics; round 3 also tried a
4-wave / 8-ROI head capped at 96 VGPRs to sit beside g1dw: 1.56-1.65 vs 1.68M ROIs/s)."""
import sys, importlib, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/tests/golden")
import gen_common as G
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
from test_gpu_kernels import _partials
gpu = torch.device("cuda")
m = trk.Model(512, 512, 10, 128).eval()
m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
m = m.to(gpu)
W = m._fused_weights(torch.bfloat16, gpu)
L = trk.lib()
R, P = 37, 100
g = torch.Generator().manual_seed(R)
sums = (torch.randn(R, 1024, generator=g) * 40 * 2 ** 24).to(torch.int64)
m_r, m_n, s = ops.enc_se(_partials(sums, P).to(gpu), P, W["se_w1"], W["se_b1"], W["se_w2"], W["se_b2"])
tsums = (torch.randn(R, 512, generator=g) * 30 * 2 ** 24).to(torch.int64)
tpart = _partials(tsums, P).to(gpu)
out = {}
for hw in (16, 8):
    assert L.trk_set_tuning(b"head_waves", hw) == 0
    out[hw] = ops.enc_head(tpart, P, s, m_r, m_n, 0.5, W["h0"], W["ln_w"], W["ln_b"], m.head.net[1].eps, W["h4"], W["h4b"])
    torch.cuda.synchronize()
for hw in (8,):
    d = (out[hw] - out[16]).abs()
    bad = (d.max(1).values > 1e-4).nonzero().flatten().tolist()
    print(hw, "maxdiff", d.max().item(), "bad rows", bad[:20], "bad cols of row0", (d[bad[0]] > 1e-4).nonzero().flatten().tolist()[:20] if bad else None)
