"""Kernel A/B microbench (one process, interleaved rounds): roi_align variants,
LSAP, cost, encoder pieces at the bench shapes.  Prints one JSON line per item."""
import importlib, json, os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden")]
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
from importlib import import_module
L = import_module("a-lightweight-unsupervised-feature-extractor-_amd._lib")
dev = torch.device("cuda:0")


def timeit(fn, reps=20, rounds=1):
    st = torch.cuda.current_stream()
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    rng = np.random.default_rng(0)
    mode = sys.argv[1] if len(sys.argv) > 1 else "all"
    B, C, H, N, S = 8, 512, 40, 256, 10
    feat = torch.from_numpy((lambda x: x / (1 + np.exp(-x)))(rng.standard_normal((B, C, H, H)).astype(np.float32))).to(dev)
    w = rng.uniform(32, 320, B * N); h = rng.uniform(32, 320, B * N)
    x1 = rng.uniform(-8, 1280 - w + 8); y1 = rng.uniform(272, 1008 - h)
    rois = torch.from_numpy(np.stack([np.repeat(np.arange(B), N), x1, y1, x1 + w, y1 + h], 1).astype(np.float32)).to(dev)
    nhwc = feat.contiguous(memory_format=torch.channels_last)
    ref = trk.roi_align(feat, rois, (S, S), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True)
    K = B * N
    algo = B * C * H * H * 4 + K * C * S * S * 2 + K * 20
    res = {}
    variants = [(1, 0, 0), (2, 0, 0), (0, 0, 4)] if mode in ("all", "roi") else []
    for rnd in range(3):
        for sw, wk, vec in variants:
            L.set_tuning("roi_sweep", sw); L.set_tuning("roi_window_kb", wk); L.set_tuning("roi_vec", vec)
            f = lambda: trk.roi_align(nhwc, rois, (S, S), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True)
            out = f()
            ok = torch.equal(out, ref)
            t = timeit(f)
            res.setdefault((sw, wk, vec), []).append(t)
            if rnd == 2:
                tm = float(np.median(res[(sw, wk, vec)]))
                print(json.dumps({"item": "roi_align_nhwc_in", "sweep": sw, "window_kb": wk, "vec": vec, "us": round(tm, 1),
                                  "GBps": round(algo / tm / 1e3, 1), "bitexact": ok}), flush=True)
    L.set_tuning("roi_sweep", 1); L.set_tuning("roi_window_kb", 0); L.set_tuning("roi_vec", 0)
    if mode in ("all", "roi"):
        t = timeit(lambda: trk.roi_align(feat, rois, (S, S), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True))
        print(json.dumps({"item": "roi_align_nchw_in(default)", "us": round(t, 1)}), flush=True)
    if mode == "roi":
        return
    # encoder pieces
    y1t = torch.randn(K, S, S, 1024, device=dev).bfloat16()
    wdw = torch.randn(25, 1024, device=dev)
    t = timeit(lambda: ops.dwconv5_nhwc(y1t, wdw))
    print(json.dumps({"item": "dwconv5_bf16", "us": round(t, 1), "GBps": round(2 * y1t.numel() * 2 / t / 1e3, 1)}), flush=True)
    xr = torch.randn(K, S * S, 512, device=dev).bfloat16()
    t = timeit(lambda: ops.act_mean(xr, "silu"))
    print(json.dumps({"item": "act_mean_bf16_rw", "us": round(t, 1), "GBps": round(2 * xr.numel() * 2 / t / 1e3, 1)}), flush=True)
    s_ = torch.rand(K, 512, device=dev)
    t = timeit(lambda: ops.scale_rows(xr, s_))
    print(json.dumps({"item": "scale_rows_bf16", "us": round(t, 1), "GBps": round(2 * xr.numel() * 2 / t / 1e3, 1)}), flush=True)
    # whole encoder forward at the bench shape (bf16, NHWC ROI input)
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_common as G
    model = trk.Model(512, 512, 10, 128).eval()
    model.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}, strict=True)
    model = model.to(dev)
    roi = ref
    with torch.no_grad():
        t = timeit(lambda: model(roi), reps=10)
    print(json.dumps({"item": "encoder_bf16_2048rois", "us": round(t, 1),
                      "TFLOPs": round(K * 320.61e6 / t / 1e6, 1)}), flush=True)
    if mode == "enc":
        return
    # LSAP: tracking-like (near-identity, gated) and uniform random, 8 frames of 256x256
    F = 8
    Ct = np.full((F, 256, 256), 1e9, np.float32)
    for f in range(F):
        perm = rng.permutation(256)
        Ct[f, np.arange(256), perm] = rng.uniform(0.1, 0.5, 256)
        m = rng.random((256, 256)) < 0.05
        Ct[f][m] = rng.uniform(0.6, 2.0, m.sum())
    Cr = rng.random((F, 256, 256)).astype(np.float32)
    for name, Cn in (("lsap_tracking_8x256", Ct), ("lsap_random_8x256", Cr)):
        Cd = torch.from_numpy(Cn).to(dev)
        out = trk.lsap_batched(Cd, [256] * F, [256] * F, cost_max=50.0)
        t = timeit(lambda: trk.lsap_batched(Cd, [256] * F, [256] * F, cost_max=50.0, out=out), reps=5)
        print(json.dumps({"item": name, "us": round(t, 1)}), flush=True)
    # scaling: frames and size (tracking-like)
    for Fq, n in ((1, 256), (64, 256), (8, 64), (8, 128), (8, 512)):
        Cq = np.full((Fq, n, n), 1e9, np.float32)
        for f in range(Fq):
            Cq[f, np.arange(n), rng.permutation(n)] = rng.uniform(0.1, 0.5, n)
        Cd = torch.from_numpy(Cq).to(dev)
        out = trk.lsap_batched(Cd, [n] * Fq, [n] * Fq, cost_max=50.0)
        t = timeit(lambda: trk.lsap_batched(Cd, [n] * Fq, [n] * Fq, cost_max=50.0, out=out), reps=5)
        print(json.dumps({"item": f"lsap_tracking_{Fq}x{n}", "us": round(t, 1), "us_per_row": round(t / n, 3)}), flush=True)


if __name__ == "__main__":
    main()
