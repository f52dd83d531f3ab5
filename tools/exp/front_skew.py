"""How evenly the persistent front's workgroups finish inside the bench pipeline.

Runs bench.py's Pipeline (c3 shape) for its preroll and warm-up, then a few steps with the front's
phase stamps on (trk_enc_set_prof: per ROI, group and wave the ROI's start on the 100 MHz clock
every CU shares; each launch overwrites the buffer, so what is read back is the last step's
front).  Per workgroup (XCD, pair, group): its first ROI's start and its last ROI's estimated end
(last start + the workgroup's median ROI period).  If the workgroups end unevenly, the front's
window is set by the last one and a dynamic ROI queue could hand the late pairs' ROIs to the early
ones: max(end) - mean(end) bounds what that could save.  The stamps add s_memtime waits, so the
absolute times run a little long.
usage: python tools/exp/front_skew.py [steps]"""
import ctypes, importlib, json, os, sys
import numpy as np
import torch

REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import bench  # noqa: E402
import gen_common as G  # noqa: E402

trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
dev = torch.device("cuda", 0)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S, N = 8, 256
R = S * N
sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
model = trk.Model(512, 512, 10, 128).eval()
model.load_state_dict(sd, strict=True)
model = model.to(dev)
frames = bench.PREROLL + 5 + steps + 3
sc = bench.make_scenes(dev, S, N, frames, seed=1000)
pipe = bench.Pipeline(sc, model)
f = 0
for _ in range(bench.PREROLL + 5):
    pipe.step(f)
    f += 1
torch.cuda.synchronize()
L = ops.lib()
L.trk_enc_set_prof.argtypes = [ctypes.c_void_p]
buf = torch.zeros(2 * R * 8 * 8, dtype=torch.int64, device=dev)
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
for _ in range(steps):
    pipe.step(f)
    f += 1
pipe.tracker.drain()
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
M56 = (1 << 56) - 1
P = torch.cuda.get_device_properties(0).multi_processor_count // 16 - 2  # pairs per XCD (rf3_groups 0)


def stats(tag, buf):
    p = buf.view(R, 2, 8, 8).cpu().numpy()
    start = (p[:, :, 0, 7] & M56).astype(np.float64) / 100.0  # us, [roi, group] (wave 0)
    stride = 8 * P
    rows = []
    for g in (0, 1):
        for xcd in range(8):
            for pr in range(P):
                rois = list(range(xcd + 8 * pr, R, stride))
                ok = (p[rois, g, 0, 7] & M56) > 0  # (the transition's stamps overwrite the first ~200 ROIs')
                if not ok[-1] or ok.sum() < 2:
                    continue
                k0 = int(np.argmax(ok))  # the first stamped ROI's index in the workgroup's sequence
                st = start[rois, g][ok]
                med = float(np.median(np.diff(st)))
                rows.append({"g": g, "xcd": xcd, "pair": pr, "n": len(rois), "last_end": float(st[-1] + med),
                             "est_start": float(st[0] - k0 * med), "period": med})
    t0 = min(r["est_start"] for r in rows)  # the earliest (estimated) workgroup start
    end = np.array([r["last_end"] - t0 for r in rows])
    est = np.array([r["est_start"] - t0 for r in rows])
    per = np.array([r["period"] for r in rows])
    q = lambda a, x: round(float(np.quantile(a, x)), 1)
    print(json.dumps({
        "run": tag, "workgroups": len(rows), "pairs_per_xcd": P,
        "est_start_us (first stamped ROI - its index x period)": {"p50": q(est, .5), "p90": q(est, .9),
                                                                   "max": round(float(est.max()), 1)},
        "end_us": {"min": round(float(end.min()), 1), "p10": q(end, .1), "p50": q(end, .5),
                                    "p90": q(end, .9), "max": round(float(end.max()), 1),
                                    "mean": round(float(end.mean()), 1)},
        "roi_period_us": {"p10": q(per, .1), "p50": q(per, .5), "p90": q(per, .9), "max": round(float(per.max()), 1)},
        "balanced_gain_bound_us": round(float(end.max() - end.mean()), 1),
        "latest": [{k: (round(v - t0, 1) if k in ("last_end", "est_start") else v) for k, v in r.items()}
                   for r in sorted(rows, key=lambda r: -r["last_end"])[:4]],
    }), flush=True)


stats("pipeline (last step's front)", buf)
# the same front alone: X of the pipeline's shape, its own weights
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(R * 100, 512, device=dev, generator=g).bfloat16()
W1p = ops.enc_pack_fragments((torch.randn(1024, 512, device=dev, generator=g) / 24).bfloat16())
wdw = torch.randn(25, 1024, device=dev, generator=g) / 5
W2p = ops.enc_pack_fragments((torch.randn(2, 512, 512, device=dev, generator=g) / 24).bfloat16())
b2 = torch.randn(1024, device=dev, generator=g) / 10
for _ in range(3):
    ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
buf.zero_()
L.trk_enc_set_prof(ctypes.c_void_p(buf.data_ptr()))
ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
torch.cuda.synchronize()
L.trk_enc_set_prof(None)
stats("isolated", buf)
