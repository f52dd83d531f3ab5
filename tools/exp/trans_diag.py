"""trans_front determinism / parity diagnostics: ROIs whose sums differ from gemm4<TRANS>."""
import importlib, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
for R in (37, 300, 2048):
    g = torch.Generator().manual_seed(R + 1)
    XRN = torch.randn(R * 100, 1024, generator=g).to(dev).bfloat16()
    s = torch.rand(R, 512, generator=g).to(dev)
    Wt = (torch.randn(512, 1024, generator=g) / 32).to(dev).bfloat16()
    bt = (torch.randn(512, generator=g) / 4).to(dev)
    ref = ops.enc_sums_reduce(ops.enc_transition_gemm(XRN, 100, s, Wt, bt, raw=True), 100)
    Wtp = ops.enc_pack_fragments_nk(Wt)
    for it in range(3):
        got = ops.enc_sums_reduce(ops.enc_transition_roi(XRN, s, Wtp, bt), 100)
        d = (got - ref).abs()
        bad = (d > 1e-4 * ref.abs().max()).nonzero()
        rois = sorted(set(bad[:, 0].tolist()))
        cols = sorted(set(bad[:, 1].tolist()))
        print(f"R={R} it={it} nbad={bad.shape[0]} nrois={len(rois)} rois={rois[:12]} ncols={len(cols)} cols={cols[:16]} max={d.max().item():.3g}", flush=True)
