"""Isolated timing of the encoder tail kernels (enc_se / enc_head) at R = 2048."""
import importlib, json, sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "golden"))
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
import gen_common as G
dev = torch.device("cuda")
m = trk.Model(512, 512, 10, 128).eval()
m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
m = m.to(dev)
W = m._fused_weights(torch.bfloat16, dev)
R = 2048
NP = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd._lib").TRK_ENC_PARTS
sums = (torch.randn(R, NP, 1024, device=dev) * 40 * 2 ** 24).to(torch.int64)
tsums = (torch.randn(R, NP, 512, device=dev) * 30 * 2 ** 24).to(torch.int64)
se = lambda: ops.enc_se(sums, 100, W["se_w1"], W["se_b1"], W["se_w2"], W["se_b2"])
m_r, m_n, s = se()
hd = lambda: ops.enc_head(tsums, 100, s, m_r, m_n, 0.5, W["h0"], W["ln_w"], W["ln_b"], 1e-5, W["h4"], W["h4b"])
for name, fn in (("enc_se", se), ("enc_head", hd)):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize()
    print(json.dumps({"kernel": name, "us": round(e0.elapsed_time(e1) / 20 * 1e3, 2)}))
