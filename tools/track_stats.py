"""Per-frame tracker statistics on the bench scene (live tracks, stage-1 / stage-2
rows, matches, unmatched detections) from the device results' headers.
usage: python tools/track_stats.py [frames]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench as B  # noqa: E402

trk = B.trk


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_common as G
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    model = trk.Model(512, 512, 10, 128).eval()
    model.load_state_dict(sd, strict=True)
    model = model.to(dev)
    sc = B.make_scenes(dev, 8, 256, F + 2, seed=1000)
    pipe = B.Pipeline(sc, model)
    tr = pipe.tracker
    for f in range(F):
        res = pipe.step(f).result()
        hdr = tr._scr["result"].view(8, -1)[:, :8].cpu().numpy()
        nm = [len(r.matches) for r in res]
        ud = [len(r.unmatched_dets) for r in res]
        print(f"frame {f:3d} live {hdr[:, 3].tolist()} m1 {hdr[:, 6].tolist()} m2 {hdr[:, 7].tolist()} "
              f"match {nm} unmatched_dets {ud} ident {pipe.check_identity(f, res):.4f}", flush=True)


if __name__ == "__main__":
    main()
