"""CPU restatement of the reference tracker step -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench.py's cpu_baseline leg may import this module (it is the
checker, never the thing measured on the GPU or shipped).

TrackerRef.update(obj) restates reference model/mainTracking.py Tracking.update
(:450-610) with its helpers -- creat_item (:99-140), predict_all (:340-345),
mark_missed (:347-355), purge_dead (:357-360), create_new_tracks (:362-373),
update_matched (:375-448) -- over the oracle's numeric restatements:
  cost + Kalman gate   oracle.cost_build (build_C_app_topk + costCard.cal_cost +
                       apply_kalman_gating; the gate's d2 in float64 like the
                       product's, DESIGN.md §5 "Known deviation")
  assignment           oracle.hungarian_assign (scipy LSAP restated, hung.py:5-45)
  Kalman filter        oracle.KalmanFilterRestated (filterpy 1.4.5) initialised as
                       KalmanFilter.init_kf_from_bbox (KalmanFilter.py:36-101)
Pinned frame by frame against the reference's own outputs in
tests/golden/track_golden_{s16,s64,reid}.npz (tests/test_oracle.py).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

import oracle as O

# conf.yaml tracker section (reference model/conf/conf.yaml:1-24)
CONF = dict(init_conf_min=0.5, hist_max=30, emb_top_k=5, w_app=1.0, w_bbox=0.3, w_conf=0.2, alpha=1.0,
            beta=0.5, cost_max=50.0, max_age=120, ema_alpha=0.9, conf_update_min=0.55, cost_update_max=30.0,
            maha_thr=9.49, lost_reid_after=50, reid_only_cost_max=0.4)


def bbox_xyxy_to_z(b):
    """KalmanFilter.py:5-16"""
    x1, y1, x2, y2 = map(float, b)
    w, h = max(1.0, x2 - x1), max(1.0, y2 - y1)
    return np.array([x1 + 0.5 * w, y1 + 0.5 * h, w / h, h], dtype=np.float32)


def x_to_bbox_xyxy(x):
    """KalmanFilter.py:19-33"""
    cx, cy, a, h = float(x[0]), float(x[1]), float(x[2]), float(x[3])
    h = max(h, 1.0)
    a = max(a, 1e-3)
    w = max(a * h, 1.0)
    return (cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h)


def init_kf(b):
    """KalmanFilter.init_kf_from_bbox defaults (dt 1, std_pos 1, std_vel 10, R = I4)"""
    kf = O.KalmanFilterRestated(8, 4)
    F = np.eye(8, dtype=np.float32)
    F[np.arange(4), np.arange(4) + 4] = 1.0
    kf.F = F
    H = np.zeros((4, 8), np.float32)
    H[np.arange(4), np.arange(4)] = 1.0
    kf.H = H
    kf.x = np.zeros((8, 1), np.float32)
    kf.x[0:4, 0] = bbox_xyxy_to_z(b)
    kf.P = np.diag(np.array([10.0] * 4 + [1000.0] * 4, np.float32))
    q = np.array([1.0] * 4 + [10.0] * 4, np.float32)
    kf.Q = np.diag(q * q)
    r = np.ones(4, np.float32)
    kf.R = np.diag(r * r)
    return kf


def gating_d2(kf, b):
    """KalmanFilter.gating_distance_maha (KalmanFilter.py:105-116), numpy dtypes as there"""
    z = bbox_xyxy_to_z(b).reshape(4, 1).astype(np.float32)
    y = z - (kf.H @ kf.x)
    S = kf.H @ kf.P @ kf.H.T + kf.R
    Sinv = np.linalg.inv(S + 1e-9 * np.eye(4, dtype=np.float32))
    return float((y.T @ Sinv @ y)[0, 0])


def _unit(e):
    e = np.asarray(e, dtype=np.float32).reshape(-1)
    return e / float(np.linalg.norm(e) + 1e-12)


class _Track:
    __slots__ = ("kf", "bank", "enc", "last_conf", "last_bbox", "miss", "age")


class TrackerRef:
    """One stream's tracker, the reference's update() semantics on the oracle."""

    def __init__(self, conf: Dict = None):
        self.c = dict(CONF)
        if conf:
            self.c.update(conf)
        self.tracks: Dict[int, _Track] = {}
        self.next_id = 0

    # ------------------------------------------------------------ helpers --
    def _cost(self, tids, embs, boxes, confs, *, gate: bool):
        T = self.c["hist_max"]
        M, N = len(tids), len(embs)
        bank = np.zeros((M, T, 128), np.float32)
        blen = np.zeros(M, np.int32)
        pbox = np.zeros((M, 4), np.float32)
        lconf = np.zeros(M, np.float32)
        for r, tid in enumerate(tids):
            t = self.tracks[tid]
            blen[r] = len(t.bank)
            if len(t.bank):
                bank[r, :len(t.bank)] = np.stack(t.bank)
            pbox[r] = np.asarray(t.last_bbox, np.float32)
            lconf[r] = t.last_conf
        kw = {}
        if gate:
            xs = np.stack([np.asarray(self.tracks[t].kf.x, np.float64).reshape(-1) for t in tids])
            Ps = np.stack([np.asarray(self.tracks[t].kf.P, np.float64) for t in tids])
            gm, gs = O.gate_params(xs, Ps)
            kw = dict(gmean=gm, gsinv=gs, gate_mask=np.ones(M, np.int32), maha_thr=self.c["maha_thr"])
        return O.cost_build(bank, blen, np.asarray(embs, np.float32).reshape(N, 128),
                            pbox, np.asarray(boxes, np.float32).reshape(N, 4), lconf,
                            np.asarray(confs, np.float32).reshape(N), w_app=self.c["w_app"],
                            w_bbox=self.c["w_bbox"], w_conf=self.c["w_conf"], alpha=self.c["alpha"],
                            beta=self.c["beta"], topk=self.c["emb_top_k"], **kw)

    def _mark_missed(self, tids):
        for tid in tids:
            if tid in self.tracks:
                self.tracks[tid].miss += 1

    def _purge(self):
        for tid in [t for t, s in self.tracks.items() if s.miss > self.c["max_age"]]:
            del self.tracks[tid]

    def _update_matched(self, matches, rows, embs, boxes, confs, C, cost_update_max, maha_thr):
        for i, j in matches:
            t = self.tracks[rows[i]]
            b, conf = boxes[j], float(confs[j])
            t.kf.update(bbox_xyxy_to_z(b))
            t.last_bbox = tuple(map(float, b))
            t.last_conf = conf
            t.age += 1
            t.miss = 0
            if conf < self.c["conf_update_min"] or float(C[i, j]) > cost_update_max:
                continue
            if gating_d2(t.kf, b) > maha_thr:
                continue
            e = _unit(embs[j])
            a = self.c["ema_alpha"]
            f = (a * t.enc + (1.0 - a) * e).astype(np.float32)
            t.enc = f / (np.linalg.norm(f) + 1e-12)
            t.bank.append(e)
            if len(t.bank) > self.c["hist_max"]:
                t.bank = t.bank[-self.c["hist_max"]:]

    def _create(self, det_ids, embs, boxes, confs):
        for j in det_ids:
            conf = float(confs[j])
            if conf < self.c["init_conf_min"]:
                continue
            t = _Track()
            e = _unit(embs[j])
            t.enc, t.bank = e, [e]
            t.last_conf, t.last_bbox = conf, tuple(map(float, boxes[j]))
            t.kf = init_kf(boxes[j])
            t.miss, t.age = 0, 1
            self.tracks[self.next_id] = t
            self.next_id += 1

    # -------------------------------------------------------------- update --
    def update(self, embs: List, boxes: List, confs: List):
        """-> (matches [(tid, det)], unmatched track ids, unmatched dets), :450-610"""
        N = len(boxes)
        if N == 0:
            ids = list(self.tracks.keys())
            self._mark_missed(ids)
            self._purge()
            return [], ids, []
        for t in self.tracks.values():  # predict_all
            t.kf.predict()
            t.last_bbox = x_to_bbox_xyxy(t.kf.x.reshape(-1))
        main = sorted(t for t, s in self.tracks.items() if s.miss <= self.c["lost_reid_after"])
        reid = sorted(t for t, s in self.tracks.items() if s.miss > self.c["lost_reid_after"])
        matches, unmatched = [], list(range(N))
        um_main = []
        if main:
            C = self._cost(main, embs, boxes, confs, gate=True)["C_total"]
            m1, um_rows, unmatched = O.hungarian_assign(C, cost_max=self.c["cost_max"])
            self._update_matched(m1, main, embs, boxes, confs, C, self.c["cost_update_max"], self.c["maha_thr"])
            matches += [(main[r], d) for r, d in m1]
            um_main = [main[r] for r in um_rows]
            self._mark_missed(um_main)
        um_reid = []
        if reid and unmatched:
            eu = [embs[j] for j in unmatched]
            bu = [boxes[j] for j in unmatched]
            cu = [confs[j] for j in unmatched]
            C2 = self._cost(reid, eu, bu, cu, gate=False)["C_app"]
            m2, um_rows2, um_u = O.hungarian_assign(C2, cost_max=self.c["reid_only_cost_max"])
            self._update_matched(m2, reid, eu, bu, cu, C2, self.c["reid_only_cost_max"], 1e18)
            matches += [(reid[r], unmatched[d]) for r, d in m2]
            um_reid = [reid[r] for r in um_rows2]
            self._mark_missed(um_reid)
            unmatched = [unmatched[d] for d in um_u]
        elif reid:
            self._mark_missed(reid)
            um_reid = reid
        self._create(unmatched, embs, boxes, confs)
        self._purge()
        return [(int(a), int(b)) for a, b in matches], um_main + um_reid, unmatched
