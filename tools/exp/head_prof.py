"""enc_se / enc_head at R = 2048 ROIs: timing and enc_head's per-wave phase stamps."""
import importlib, json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests", "golden"))
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
import gen_common as G
dev = torch.device("cuda")
m = trk.Model(512, 512, 10, 128).eval()
m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
m = m.to(dev)
W = m._fused_weights(torch.bfloat16, dev)
R, P = 2048, 100
g = torch.Generator().manual_seed(0)
sums = (torch.randn(R, 1024, generator=g) * 40 * 2 ** 24).to(torch.int64)
parts = torch.zeros(R, 3, 1024, dtype=torch.int64); parts[:, 0] = sums
parts = parts.to(dev)
tparts = torch.zeros(R, 3, 512, dtype=torch.int64); tparts[:, 0] = (torch.randn(R, 512, generator=g) * 30 * 2 ** 24).to(torch.int64)
tparts = tparts.to(dev)
se = lambda: ops.enc_se(parts, P, W["se_w1_pk"], W["se_b1"], W["se_w2_pk"], W["se_b2"])
m_r, m_n, s = se()
hd = lambda: ops.enc_head(tparts, P, s, m_r, m_n, 0.5, W["h0_pk"], W["ln_w"], W["ln_b"], 1e-5, W["h4_pk"], W["h4b"])
def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)
L = trk.lib()
for hw in (8, 16, 8, 16):
    L.trk_set_tuning(b"head_waves", hw)
    L.trk_set_tuning(b"se_waves", hw)
    print(json.dumps({"head_waves": hw, "se_waves": hw, "enc_se_us": t(se), "enc_head_us": t(hd)}), flush=True)
L.trk_set_tuning(b"se_waves", 16)
prof = torch.zeros(R // 16 * 16 * 5, dtype=torch.int64, device=dev)
L.trk_head_set_prof(ops._ptr(prof)); hd(); torch.cuda.synchronize(); L.trk_head_set_prof(None)
pr = prof.view(-1, 5).double()
print(json.dumps({"head_ticks_mean": dict(zip(["prologue", "W0", "LN", "W4", "normalize"], [round(x) for x in pr.mean(0).tolist()])),
                  "head_ticks_max": dict(zip(["prologue", "W0", "LN", "W4", "normalize"], [round(x) for x in pr.max(0).values.tolist()]))}), flush=True)
