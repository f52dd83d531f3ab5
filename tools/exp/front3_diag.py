"""rf_v 3 (persistent rmb_front) vs rf_v 2 on the same operands: where XRN / sums differ."""
import importlib, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
L = ops.lib()
dev = torch.device("cuda")
for R in (1, 2, 9, 37, 2048):
    g = torch.Generator().manual_seed(R)
    X = torch.randn(R * 100, 512, generator=g).to(dev).bfloat16()
    W1p = ops.enc_pack_fragments((torch.randn(1024, 512, generator=g) / 24).to(dev).bfloat16())
    wdw = (torch.randn(25, 1024, generator=g) / 5).to(dev)
    W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, generator=g) / 24).to(dev).bfloat16())
    b2 = (torch.randn(1024, generator=g) / 10).to(dev)
    out = {}
    for v in (2, 3):
        L.trk_set_tuning(b"rf_v", v)
        XRN, s = ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
        out[v] = (XRN.float(), ops.enc_sums_reduce(s, 100))
    L.trk_set_tuning(b"rf_v", 3)
    d = (out[2][0] - out[3][0]).abs()
    bad = d > 0
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print(R, "XRN diff elems", int(bad.sum()), "max", float(d.max()), "rows", rows[:8].tolist(), "...", rows.numel(),
          "cols", cols[:8].tolist(), "...", cols.numel(),
          "sums maxdiff", float((out[2][1] - out[3][1]).abs().max()), flush=True)
