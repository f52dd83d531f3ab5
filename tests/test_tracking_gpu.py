"""The product tracker (device-resident state, HIP kernels) reproduces the
reference mainTracking.Tracking.update outputs frame by frame on the golden
scenes: matches, unmatched track ids and unmatched detections, bit-exact."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _frames(d):
    off = d["det_off"]
    for f in range(int(d["n_frames"])):
        a, b = off[f], off[f + 1]
        yield f, d["embs"][a:b], d["boxes"][a:b], d["confs"][a:b]


def _expected(d, f):
    m = d["matches"][d["m_off"][f]:d["m_off"][f + 1]]
    ut = d["um_tracks"][d["um_t_off"][f]:d["um_t_off"][f + 1]]
    ud = d["um_dets"][d["um_d_off"][f]:d["um_d_off"][f + 1]]
    return [tuple(map(int, x)) for x in m], [int(x) for x in ut], [int(x) for x in ud]


@pytest.mark.parametrize("name", ["s16", "s64", "reid"])
def test_tracking_update_matches_reference_golden(trk, gpu, name):
    d = np.load(os.path.join(GOLDEN, f"track_golden_{name}.npz"))
    t = trk.Tracking()
    for f, emb, box, conf in _frames(d):
        obj = {"embs": [e for e in emb], "bboxes": box.tolist(), "confs": conf.tolist(),
               "input_hw": (1280, 1280), "frame_id": f}
        got = t.update(obj)
        assert got == _expected(d, f), f"{name} frame {f}"


def test_multistream_tracker_equals_per_stream_reference(trk, gpu):
    """Three scenes advanced as three streams of one MultiStreamTracker."""
    names = ["s16", "s64", "reid"]
    ds = [np.load(os.path.join(GOLDEN, f"track_golden_{n}.npz")) for n in names]
    mst = trk.MultiStreamTracker(len(names))
    frames = [list(_frames(d)) for d in ds]
    F = max(len(fr) for fr in frames)
    for f in range(F):
        Ns, confs = [], []
        Nmax = max([len(fr[f][2]) if f < len(fr) else 0 for fr in frames] + [1])
        E = torch.zeros(len(names), Nmax, 128)
        B = torch.zeros(len(names), Nmax, 4)
        C = torch.zeros(len(names), Nmax)
        for s, fr in enumerate(frames):
            if f < len(fr):
                _, emb, box, conf = fr[f]
                n = len(conf)
                E[s, :n] = torch.from_numpy(emb)
                B[s, :n] = torch.from_numpy(box.astype(np.float32))
                C[s, :n] = torch.from_numpy(conf.astype(np.float32))
                Ns.append(n); confs.append(conf.tolist())
            else:
                Ns.append(0); confs.append([])
        res = mst.step(E.to(gpu), B.to(gpu), C.to(gpu), Ns, confs, [f] * len(names))
        for s, fr in enumerate(frames):
            if f < len(fr):
                got = res[s].as_tuple()
                assert (got[0], got[1], got[2]) == _expected(ds[s], f), f"{names[s]} frame {f}"


def test_tracking_helpers_match_reference_costs(trk, oracle, gpu):
    """cal_cost / build_C_app_topk / apply_kalman_gating, evaluated on the
    product's own track state (float64 Kalman state) at the
    golden dump frames, reproduce the reference's costs within the north-star
    tolerance 1e-4 and its gating decisions exactly."""
    d = np.load(os.path.join(GOLDEN, "track_golden_s16.npz"))
    t = trk.Tracking()
    checked = 0
    for f, emb, box, conf in _frames(d):
        if f in d["dump_frames"] and f"f{f}_C_app" in d.files:
            # advance to frame f-1 done; run predict + cost on frame f's dets
            t.predict_all()
            rows = [int(x) for x in d[f"f{f}_rows_main"]]
            capp = t.build_C_app_topk(row_to_tid=rows, det_embs=list(emb), topk=5).cpu().numpy()
            assert np.max(np.abs(capp - d[f"f{f}_C_app"])) <= 1e-4
            cc = t.cal_cost(row_to_tid=rows, det_embs=list(emb), det_boxes=box.tolist(),
                            det_confs=conf.tolist(), input_hw=(1280, 1280))
            assert np.max(np.abs(cc["C_total"].cpu().numpy() - d[f"f{f}_C_total"])) <= 1e-4
            g = t.apply_kalman_gating(d[f"f{f}_C_total"].copy(), rows, box.tolist(), maha_thr=9.49)
            assert np.array_equal(g >= 1e9, d[f"f{f}_C_gated"] >= 1e9)
            checked += 1
            # undo the extra predict by rebuilding the tracker up to here
            t = trk.Tracking()
            for f2, e2, b2, c2 in _frames(d):
                if f2 > f:
                    break
                t.update({"embs": list(e2), "bboxes": b2.tolist(), "confs": c2.tolist(),
                          "input_hw": (1280, 1280), "frame_id": f2})
            continue
        t.update({"embs": list(emb), "bboxes": box.tolist(), "confs": conf.tolist(),
                  "input_hw": (1280, 1280), "frame_id": f})
    assert checked >= 2


def test_tracking_argument_errors(trk, gpu):
    t = trk.Tracking()
    with pytest.raises(ValueError, match="input_hw"):
        t.update({"frame_id": 0})
    with pytest.raises(ValueError, match="frame_id"):
        t.update({"input_hw": (1, 1)})
    with pytest.raises(ValueError, match="Length mismatch"):
        t.update({"input_hw": (1, 1), "frame_id": 0, "embs": [np.zeros(128)], "bboxes": [], "confs": []})
    with pytest.raises(ValueError, match="128D"):
        t.update({"input_hw": (1, 1), "frame_id": 0, "embs": [np.zeros(64)], "bboxes": [[0, 0, 1, 1]],
                  "confs": [0.9]})
    assert t.update({"input_hw": (1, 1), "frame_id": 0}) == ([], [], [])
