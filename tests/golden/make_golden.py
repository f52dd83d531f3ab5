"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
code in this (survey) container.  The reference never travels: only the
numeric inputs/outputs written here do.

Run:  cd /root/repo && python tests/golden/make_golden.py  [n256]

What runs as-is from /root/reference (no edits, read-only tree):
  model.utils.modules.encoderAndHead.Model       (encoder golden)
  model.utils.costTool.costCard.cal_cost          (cost-formula golden)
  model.utils.costTool.hung.hungarian_assign      (assignment golden, scipy inside)
  model.mainTracking.Tracking.update              (per-frame tracker golden)

Third-party modules the reference imports that are absent from this image:
  filterpy (pinned filterpy==1.4.5, requirements.txt:15): provided by
      oracle.KalmanFilterRestated, a restatement of filterpy's published
      KalmanFilter.predict/update -- so KF arithmetic in the tracker golden is
      "restated", not pinned by filterpy itself.
  model.utils.inferScr.infer (pulls cv2/torchvision): mainTracking.py:1 only
      imports MainInfer and never uses it inside Tracking; a placeholder class
      is installed for that import.
scipy 1.15.3 (reference pins 1.16.3; LSAP algorithm unchanged) is real.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.dont_write_bytecode = True

import gen_common as G  # noqa: E402


def _import_reference():
    import torch  # noqa: F401
    sys.path.insert(0, REF)
    os.chdir(REF)  # mainTracking.py:47 reads model/conf/conf.yaml relative to cwd
    import oracle as O
    fp = types.ModuleType("filterpy")
    fpk = types.ModuleType("filterpy.kalman")
    fpk.KalmanFilter = O.KalmanFilterRestated
    fp.kalman = fpk
    sys.modules.setdefault("filterpy", fp)
    sys.modules.setdefault("filterpy.kalman", fpk)
    inf = types.ModuleType("model.utils.inferScr.infer")

    class MainInfer:  # placeholder: imported by mainTracking.py:1, unused by Tracking
        pass
    inf.MainInfer = MainInfer
    sys.modules.setdefault("model.utils.inferScr.infer", inf)
    import model.utils.modules.encoderAndHead as eh
    import model.utils.costTool.costCard as cc
    import model.utils.costTool.hung as hg
    import model.mainTracking as mt
    return eh, cc, hg, mt


def gen_encoder(eh):
    import torch
    import torch.nn.functional as F
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    m = eh.Model(in_channels=512, out_channels=512, warmup_epochs=10, proj_dim=128).eval()
    m.load_state_dict(sd, strict=True)
    out = {}
    with torch.no_grad():
        for s, seed in ((7, 101), (10, 102)):
            x = torch.from_numpy(G.encoder_input(seed, 16, s))
            z = F.normalize(m(x).float(), dim=-1)
            out[f"z_s{s}"] = z.numpy()
            out[f"seed_s{s}"] = np.array(seed)
    np.savez_compressed(os.path.join(HERE, "encoder_golden.npz"), **out)


def gen_costcard(cc):
    import torch
    rng = np.random.default_rng(7)
    out = {}
    for tag, (M, N) in {"a": (16, 16), "b": (37, 23), "c": (1, 9)}.items():
        bp = np.sort(rng.uniform(-20, 1300, (M, 2, 2)), axis=1).transpose(0, 2, 1).reshape(M, 4)
        bp = bp[:, [0, 2, 1, 3]]
        bc = np.sort(rng.uniform(-20, 1300, (N, 2, 2)), axis=1).transpose(0, 2, 1).reshape(N, 4)
        bc = bc[:, [0, 2, 1, 3]]
        bc[0, 2] = bc[0, 0] + 0.25  # degenerate width < 1
        bp[0, 3] = bp[0, 1] + 0.5   # degenerate height < 1
        cp = rng.uniform(0.0, 1.0, M); cp[0] = 0.0
        cu = rng.uniform(0.0, 1.0, N); cu[-1] = 1e-9
        capp = torch.from_numpy(rng.uniform(0, 2, (M, N)).astype(np.float32))
        res = cc.cal_cost(C_app=capp, boxes_prev=bp.tolist(), boxes_cur=bc.tolist(),
                          input_hw=(1280, 1280), conf_prev=cp.tolist(), conf_cur=cu.tolist(),
                          w_app=1.0, w_bbox=0.3, w_conf=0.2, alpha=1.0, beta=0.5)
        out[f"{tag}_bp"] = bp; out[f"{tag}_bc"] = bc
        out[f"{tag}_cp"] = cp; out[f"{tag}_cu"] = cu
        out[f"{tag}_capp"] = capp.numpy()
        for k in ("C_total", "C_center", "C_scale", "C_conf", "C_bbox"):
            out[f"{tag}_{k}"] = res[k].numpy()
    np.savez_compressed(os.path.join(HERE, "costcard_golden.npz"), **out)


def gen_lsap(hg):
    from scipy.optimize import linear_sum_assignment
    cases = G.lsap_cases()
    rng = np.random.default_rng(9)
    # +inf entries that keep the problem feasible, and one infeasible matrix
    fin = rng.random((12, 12)).astype(np.float32)
    fin[rng.random((12, 12)) < 0.5] = np.inf
    fin[np.arange(12), rng.permutation(12)] = 0.5
    cases.append(fin)
    infeas = np.ones((4, 4), np.float32); infeas[2, :] = np.inf
    cases.append(infeas)
    nanm = np.ones((3, 3), np.float32); nanm[1, 1] = np.nan
    cases.append(nanm)
    shapes, flat, rows, cols, offs, status = [], [], [], [], [0], []
    hm_cm = []
    for C in cases:
        shapes.append(C.shape)
        flat.append(C.ravel())
        try:
            r, c = linear_sum_assignment(C)
            st = 0
        except ValueError as e:
            r = c = np.zeros(0, np.int64)
            st = -1 if "invalid" in str(e) else -2
        status.append(st)
        rows.append(r.astype(np.int64)); cols.append(c.astype(np.int64))
        offs.append(offs[-1] + len(r))
    # hungarian_assign with cost gates on a subset
    hm_out = []
    for q, C in enumerate(cases[:90]):
        cm = [50.0, 0.4, 1.0][q % 3]
        try:
            m, ut, ud = hg.hungarian_assign(C, cost_max=cm)
        except ValueError:
            continue
        hm_cm.append((q, cm))
        hm_out.append((m, ut, ud))
    hm_q = np.array([q for q, _ in hm_cm], np.int64)
    hm_c = np.array([c for _, c in hm_cm], np.float64)
    hm_match = [np.array(m, np.int64).reshape(-1, 2) for m, _, _ in hm_out]
    hm_moff = np.cumsum([0] + [len(m) for m in hm_match])
    np.savez_compressed(
        os.path.join(HERE, "lsap_golden.npz"),
        shapes=np.array(shapes, np.int64), data=np.concatenate(flat).astype(np.float32),
        rows=np.concatenate(rows), cols=np.concatenate(cols), offs=np.array(offs, np.int64),
        status=np.array(status, np.int64), hm_q=hm_q, hm_cost_max=hm_c,
        hm_match=np.concatenate(hm_match) if hm_match else np.zeros((0, 2), np.int64),
        hm_moff=hm_moff)


def gen_tracking(mt, name, dump_frames):
    """Drive the reference Tracking.update over a synthetic scene; record
    per-frame outputs and, at dump_frames, the full pre-cost track state."""
    frames = G.scene(name)
    trk = mt.Tracking()
    rec = {"cur": None}
    orig_predict = trk.predict_all
    orig_cal = trk.cal_cost
    orig_gate = trk.apply_kalman_gating
    orig_app = trk.build_C_app_topk
    orig_hung = mt.hungarian_assign

    def predict_all():
        orig_predict()
        f = rec["cur"]
        if f["frame_id"] in dump_frames:
            st = {}
            tids = sorted(trk.tracks.keys())
            M = len(tids)
            bank = np.zeros((M, 30, 128), np.float32)
            blen = np.zeros(M, np.int32)
            pbox = np.zeros((M, 4), np.float32)
            lconf = np.zeros(M, np.float32)
            kx = np.zeros((M, 8)); kP = np.zeros((M, 8, 8)); miss = np.zeros(M, np.int64)
            for r, tid in enumerate(tids):
                ts = trk.tracks[tid]
                hist = ts.memory.feat_historical
                blen[r] = len(hist)
                if len(hist):
                    bank[r, :len(hist)] = np.stack(hist)
                pbox[r] = np.asarray(ts.memory.last_bbox, np.float32)
                lconf[r] = ts.memory.last_conf
                kx[r] = np.asarray(ts.kf.x, np.float64).reshape(-1)
                kP[r] = np.asarray(ts.kf.P, np.float64)
                miss[r] = ts.miss_count
            st.update(tids=np.array(tids, np.int64), bank=bank, bank_len=blen, pbox=pbox,
                      last_conf=lconf, kf_x=kx, kf_P=kP, miss=miss)
            f["state"] = st

    def cal_cost(**kw):
        out = orig_cal(**kw)
        f = rec["cur"]
        f["rows_main"] = np.array(kw["row_to_tid"], np.int64)
        for k in ("C_total", "C_app", "C_center", "C_scale", "C_conf"):
            f[k] = out[k].detach().cpu().numpy().copy()
        return out

    def apply_kalman_gating(C, row_to_tid, det_boxes, **kw):
        out = orig_gate(C, row_to_tid, det_boxes, **kw)
        rec["cur"]["C_gated"] = out.copy()
        return out

    def build_C_app_topk(**kw):
        out = orig_app(**kw)
        f = rec["cur"]
        if kw["row_to_tid"] is not None and "C_app" in f and len(kw["det_embs"]) and f.get("_stage2"):
            pass
        f.setdefault("app_calls", []).append((list(kw["row_to_tid"]), out.detach().cpu().numpy().copy()))
        return out

    def hungarian_assign(C, cost_max=1e9):
        res = orig_hung(C, cost_max=cost_max)
        rec["cur"].setdefault("hung", []).append((C.copy(), cost_max, res))
        return res

    trk.predict_all = predict_all
    trk.cal_cost = cal_cost
    trk.apply_kalman_gating = apply_kalman_gating
    trk.build_C_app_topk = build_C_app_topk
    mt.hungarian_assign = hungarian_assign
    out = {}
    det_off = [0]
    embs, boxes, confs = [], [], []
    m_all, m_off, um_t, um_t_off, um_d, um_d_off = [], [0], [], [0], [], [0]
    try:
        for fr in frames:
            rec["cur"] = {"frame_id": fr["frame_id"]}
            obj = {"embs": [e for e in fr["embs"]], "bboxes": fr["bboxes"], "confs": fr["confs"],
                   "input_hw": (1280, 1280), "frame_id": fr["frame_id"]}
            matches, ut, ud = trk.update(obj)
            f = rec["cur"]
            n = len(fr["confs"])
            det_off.append(det_off[-1] + n)
            embs.append(fr["embs"]); boxes.append(np.asarray(fr["bboxes"], np.float64).reshape(-1, 4))
            confs.append(np.asarray(fr["confs"], np.float64))
            m_all.append(np.asarray(matches, np.int64).reshape(-1, 2)); m_off.append(m_off[-1] + len(matches))
            um_t.append(np.asarray(ut, np.int64)); um_t_off.append(um_t_off[-1] + len(ut))
            um_d.append(np.asarray(ud, np.int64)); um_d_off.append(um_d_off[-1] + len(ud))
            fid = fr["frame_id"]
            if "rows_main" in f and name not in G.OUTPUT_ONLY:  # (n256: 1.5 MB per frame)
                out[f"f{fid}_rows_main"] = f["rows_main"]
                out[f"f{fid}_C_gated"] = f["C_gated"]
                for k in ("C_total", "C_app", "C_center", "C_scale", "C_conf"):
                    out[f"f{fid}_{k}"] = f[k]
            hung = f.get("hung", [])
            if len(hung) == 2:  # stage 2 ran
                rows_reid, capp2 = f["app_calls"][-1]
                out[f"f{fid}_rows_reid"] = np.array(rows_reid, np.int64)
                out[f"f{fid}_C_reid"] = capp2
            if "state" in f:
                for k, v in f["state"].items():
                    out[f"f{fid}_state_{k}"] = v
    finally:
        mt.hungarian_assign = orig_hung
    if name in G.OUTPUT_ONLY:  # inputs regenerated from the seed by the tests; digest kept
        out.update(det_off=np.array(det_off, np.int64), digest=np.array(G.scene_digest(frames)))
    else:
        out.update(det_off=np.array(det_off, np.int64), embs=np.concatenate(embs).astype(np.float32),
                   boxes=np.concatenate(boxes), confs=np.concatenate(confs))
    out.update(matches=np.concatenate(m_all), m_off=np.array(m_off, np.int64),
               um_tracks=np.concatenate(um_t), um_t_off=np.array(um_t_off, np.int64),
               um_dets=np.concatenate(um_d), um_d_off=np.array(um_d_off, np.int64),
               n_frames=np.array(len(frames)), dump_frames=np.array(sorted(dump_frames), np.int64))
    np.savez_compressed(os.path.join(HERE, f"track_golden_{name}.npz"), **out)
    return out


def main():
    eh, cc, hg, mt = _import_reference()
    if sys.argv[1:] == ["n256"]:  # the N = 256 tracker scene only (~3 min: per-pair gating loop)
        gen_tracking(mt, "n256", set())
        print("track_golden_n256.npz written to", HERE)
        return
    gen_encoder(eh)
    gen_costcard(cc)
    gen_lsap(hg)
    gen_tracking(mt, "s16", {1, 2, 12, 35, 39})
    gen_tracking(mt, "s64", {1, 3, 7})
    gen_tracking(mt, "reid", {58, 59, 61})
    gen_tracking(mt, "n256", set())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
