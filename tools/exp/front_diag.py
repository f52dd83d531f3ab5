"""rmb_front determinism diagnostics: repeated launches vs the two-kernel path, with the
(row % 100, column) pattern of every mismatch."""
import importlib, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda")
for R in (1, 37):
    g = torch.Generator().manual_seed(R)
    M, P = R * 100, 100
    X = torch.randn(M, 512, generator=g).to(dev).bfloat16()
    W1 = (torch.randn(1024, 512, generator=g) / 24).to(dev).bfloat16()
    wdw = (torch.randn(25, 1024, generator=g) / 5).to(dev)
    W2 = (torch.randn(2, 512, 512, generator=g) / 24).to(dev).bfloat16()
    b2 = (torch.randn(1024, generator=g) / 10).to(dev)
    ref, _ = ops.enc_dsc_gemm(ops.enc_g1_dwconv(X, W1, wdw), P, W2, b2, raw=True)
    W1p, W2p = ops.enc_pack_fragments(W1), ops.enc_pack_fragments(W2)
    for it in range(6):
        x, _ = ops.enc_rmb_front(X, W1p, wdw, W2p, b2)
        torch.cuda.synchronize()
        bad = (x != ref).nonzero()
        rows = sorted(set((bad[:, 0] % 100).tolist()))
        cols = sorted(set(bad[:, 1].tolist()))
        print(f"R={R} it={it} n_bad={bad.shape[0]} rows%100={rows[:20]} ncols={len(cols)} cols={cols[:12]}..{cols[-4:]}", flush=True)
        if it == 0 and bad.shape[0]:
            r, c = bad[0].tolist()
            print("  first", r, c, x[r, c].item(), ref[r, c].item(), flush=True)
