"""LSAP latency breakdown on the bench's own stage-1 cost matrices (8 streams x
256 tracks x 256 detections after the 30-frame pre-roll) and on two synthetic
extremes; prints us per matrix batch and the solver's shader-clock breakdown
(trk_lsap_set_prof).  usage: python tools/lsap_bench.py [reps]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench as B  # noqa: E402

trk, ops = B.trk, B.ops


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def breakdown(C, nr, nc):
    L = ops.lib()
    F = C.shape[0]
    buf = torch.zeros(F * 16, dtype=torch.int64, device=C.device)
    L.trk_lsap_set_prof(ops._ptr(buf))
    trk.lsap_batched(C, nr, nc, cost_max=50.0)
    torch.cuda.synchronize()
    L.trk_lsap_set_prof(None)
    p = buf.view(F, 16).cpu().numpy().astype(np.float64)
    tot = max(p[:, 5].mean(), 1.0)
    nrow = max(float(np.asarray(nr).mean()), 1.0)
    return {"wg_cycles": {"shortcut": round(p[:, 8].mean()), "solver": round(p[:, 9].mean()),
                          "outputs": round(p[:, 10].mean()), "total": round(p[:, 11].mean()),
                          "setup": round(p[:, 12].mean()), "scans": round(p[:, 13].mean()),
                          "scan_barrier": round(p[:, 14].mean()), "claims_duals": round(p[:, 15].mean())},
            "wait%": round(100 * p[:, 0].mean() / tot, 1), "scan%": round(100 * p[:, 1].mean() / tot, 1),
            "dual%": round(100 * p[:, 2].mean() / tot, 1), "aug%": round(100 * p[:, 3].mean() / tot, 1),
            "iters/row": round(p[:, 4].sum() / max(p[:, 6].sum(), 1.0), 3),
            "cyc/row": round(p[:, 5].mean() / nrow), "cyc/iter_scan": round(p[:, 1].sum() / max(p[:, 4].sum(), 1))}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_common as G
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    model = trk.Model(512, 512, 10, 128).eval()
    model.load_state_dict(sd, strict=True)
    model = model.to(dev)
    sc = B.make_scenes(dev, 8, 256, B.PREROLL + 3, seed=1000)
    pipe = B.Pipeline(sc, model)
    for f in range(B.PREROLL + 1):
        pipe.step(f).result()
    tr = pipe.tracker
    Mb, Nm = tr.last_Mb, tr._nmax
    m1 = tr._scr["m1"].cpu().numpy().tolist()
    N = tr._scr["ndet"].cpu().numpy().tolist()
    C1 = tr._C[0][:8 * Mb * Nm].view(8, Mb, Nm).clone()
    cases = {"bench stage-1 (gated)": (C1, m1, N)}
    g = torch.Generator().manual_seed(0)
    cases["uniform random 256^2"] = (torch.rand(8, 256, 256, generator=g).to(dev), [256] * 8, [256] * 8)
    eye = torch.full((8, 256, 256), 1.0)
    eye[:, torch.arange(256), torch.randperm(256, generator=g)] = 0.1
    cases["permutation (1 iter/row)"] = (eye.to(dev), [256] * 8, [256] * 8)
    for name, (C, nr, nc) in cases.items():
        out = trk.lsap_batched(C, nr, nc, cost_max=50.0)  # preallocated outputs: time the launches
        us = timed(lambda: trk.lsap_batched(C, nr, nc, cost_max=50.0, out=out), reps)
        print(f"{name:28s} {us:8.1f} us/batch  {us / max(nr):6.3f} us/row  {breakdown(C, nr, nc)}", flush=True)


if __name__ == "__main__":
    main()
