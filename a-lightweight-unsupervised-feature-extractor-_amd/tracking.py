"""Tracker state machine over device-resident track tables.

Drop-in for reference model/mainTracking.py (class Tracking):
the per-frame association runs on gfx950 kernels --

  predict_all          -> trk_kf_predict   (KF predict + predicted box + gate inputs)
  cal_cost + gating    -> trk_build_cost   (bank top-k appearance, bbox, conf, Mahalanobis)
  hungarian_assign     -> trk_lsap         (scipy-exact SAP + the cost_max gate)
  update_matched       -> trk_track_update (KF update, appearance gates, EMA, bank push)
  create_new_tracks    -> trk_track_init

-- while the per-track bookkeeping that the reference keeps in Python dicts
(ids, miss counts, ages, the main / ReID-only row split, purge) stays on the
host as numpy arrays.  ``MultiStreamTracker`` batches S independent video
streams through one launch per stage; ``Tracking`` is its single-stream form
with the reference's method names, argument meanings and error behaviour.
Host syncs: one per frame after stage 1 (plus one after stage 2 when a
long-lost ReID-only stage runs), where the reference already syncs
(mainTracking.py:503,559).
"""
from __future__ import annotations

import ctypes
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, lib
from .ops import (_device, _ptr, _stream, build_cost, cost_combine, default_cost_params,
                  lsap_batched)

D = 128

# conf.yaml tracker section (reference model/conf/conf.yaml:1-24) -- the YAML
# values, which differ from the in-code defaults of mainTracking.py:55-96
CONF_DEFAULTS: Dict[str, Any] = dict(
    init_conf_min=0.5, hist_max=30, emb_top_k=5, app_tau=0.07, eps=1.0e-12,
    w_app=1.0, w_bbox=0.3, w_conf=0.2, alpha=1.0, beta=0.5, unmatch_cost=10.0,
    cost_max=50.0, max_age=120, ema_alpha=0.9, conf_update_min=0.55,
    cost_update_max=30.0, maha_thr=9.49, lost_reid_after=50, reid_sim_min=0.6,
    reid_only_cost_max=0.4)


def load_conf(path: str) -> Dict[str, Any]:
    """mainTracking.load_conf (mainTracking.py:11-13)."""
    import yaml
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


def tracker_conf(conf: Optional[Dict[str, Any]] = None, conf_path: Optional[str] = None) -> Dict[str, Any]:
    """Resolve the tracker constants like Tracking.__init__ (mainTracking.py:46-96):
    a given dict, else the YAML at conf_path, else model/conf/conf.yaml relative
    to the cwd when present, else the conf.yaml values."""
    if conf is None:
        path = conf_path or ("model/conf/conf.yaml" if os.path.exists("model/conf/conf.yaml") else None)
        if path is not None:
            full = load_conf(path)
            if "tracker" not in full:
                raise KeyError("Missing 'tracker' section in YAML config.")
            conf = full["tracker"]
        else:
            conf = {}
    t = dict(CONF_DEFAULTS)
    t.update(conf)
    if "reid_only_cost_max" not in conf and "reid_sim_min" in conf:
        t["reid_only_cost_max"] = 1.0 - float(conf["reid_sim_min"])
    return t


class TrackTable:
    """Slot arrays of every track of every stream (layout: include/trk_amd.h)."""

    def __init__(self, slots: int, hist_max: int, device):
        self.S, self.T, self.device = slots, hist_max, device
        z = lambda *s, dt=torch.float32: torch.zeros(s, device=device, dtype=dt)
        self.x = z(slots, 8, dt=torch.float64)
        self.P = z(slots, 64, dt=torch.float64)
        self.pbox = z(slots, 4)
        self.last_conf = z(slots)
        self.gmean = z(slots, 4, dt=torch.float64)
        self.gsinv = z(slots, 16, dt=torch.float64)
        self.gate_on = torch.ones(slots, device=device, dtype=torch.int32)
        self.enc = z(slots, D)
        self.bank = z(slots, hist_max, D)
        self.bank_len = z(slots, dt=torch.int32)
        self.bank_head = z(slots, dt=torch.int32)


@dataclass
class StreamState:
    """Host bookkeeping of one stream's tracks (Tracking.tracks of the reference)."""
    cap: int
    base: int
    alive: np.ndarray = None
    tid: np.ndarray = None
    miss: np.ndarray = None
    age: np.ndarray = None
    last_frame: np.ndarray = None
    next_id: int = 0

    def __post_init__(self):
        self.alive = np.zeros(self.cap, bool)
        self.tid = np.full(self.cap, -1, np.int64)
        self.miss = np.zeros(self.cap, np.int64)
        self.age = np.zeros(self.cap, np.int64)
        self.last_frame = np.zeros(self.cap, np.int64)

    def live_sorted(self) -> np.ndarray:
        """local slots of live tracks in ascending track id (= dict order)."""
        s = np.flatnonzero(self.alive)
        return s[np.argsort(self.tid[s], kind="stable")]


_EMPTY = np.zeros(0, np.int64)


@dataclass
class FrameResult:
    """One stream's frame result as arrays: matches [K, 2] (track_id, det_idx)
    in the reference's order (stage-1 rows ascending, then stage-2), unmatched
    track ids (stage-1 then stage-2 order) and unmatched detections."""
    matches: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.int64))
    unmatched_tracks: np.ndarray = _EMPTY
    unmatched_dets: np.ndarray = _EMPTY

    def as_tuple(self):
        """the reference's return value: ([(tid, det)], [tid], [det]) lists"""
        return ([(int(a), int(b)) for a, b in self.matches], [int(x) for x in self.unmatched_tracks],
                [int(x) for x in self.unmatched_dets])


class MultiStreamTracker:
    """S independent trackers (one per video stream) advanced together.

    step() takes the detections of one frame of every stream, already on the
    device: det_emb [S, Nmax, 128] f32, dbox [S, Nmax, 4] f32, dconf [S, Nmax]
    f32, plus the host copies of the confidences (creation gate) and the
    counts N[s].  Returns one FrameResult per stream, identical to what
    mainTracking.Tracking.update would return for that stream."""

    def __init__(self, n_streams: int, conf: Optional[Dict[str, Any]] = None, *,
                 capacity: int = 1024, device=None, conf_path: Optional[str] = None):
        self.cfg = tracker_conf(conf, conf_path)
        self.n_streams = n_streams
        self.cap = capacity
        self.device = torch.device(device) if device is not None else _device()
        self.T = int(self.cfg["hist_max"])
        if self.T > 32:
            raise NotImplementedError("hist_max > 32 is not supported by the cost kernel")
        self.table = TrackTable(n_streams * capacity, self.T, self.device)
        self.streams = [StreamState(capacity, s * capacity) for s in range(n_streams)]
        self.params = default_cost_params(self.cfg, gate=True)
        self.params_nogate = default_cost_params(self.cfg, gate=False)
        self.sync_wait_s = 0.0  # host time blocked on the per-frame index copies (bench diagnostics)

    # ------------------------------------------------------------ helpers --
    def _i32(self, a) -> torch.Tensor:
        return torch.as_tensor(np.ascontiguousarray(a, np.int32)).to(self.device, non_blocking=True)

    def _predict(self, slots: np.ndarray):
        if len(slots) == 0:
            return
        t = self.table
        s = self._i32(slots)
        check(lib().trk_kf_predict(len(slots), _ptr(s), _ptr(t.x), _ptr(t.P), _ptr(t.pbox), _ptr(t.gmean),
                                   _ptr(t.gsinv), _stream(self.device)), "kf_predict")

    def _update(self, slots, dets, cost: Optional[torch.Tensor], cost_idx, cost_update_max, maha_thr,
                det_emb, dbox, dconf):
        if len(slots) == 0:
            return
        t = self.table
        s, d = self._i32(slots), self._i32(dets)
        ci = (torch.as_tensor(np.asarray(cost_idx, np.int64)).to(self.device, non_blocking=True)
              if cost is not None else None)
        check(lib().trk_track_update(len(slots), _ptr(s), _ptr(d), _ptr(ci), _ptr(cost), _ptr(dbox),
                                     _ptr(dconf), _ptr(det_emb), _ptr(t.x), _ptr(t.P), _ptr(t.pbox),
                                     _ptr(t.last_conf), _ptr(t.enc), _ptr(t.bank), _ptr(t.bank_len),
                                     _ptr(t.bank_head), self.T, float(self.cfg["ema_alpha"]),
                                     float(self.cfg["conf_update_min"]), float(cost_update_max),
                                     float(maha_thr), _stream(self.device)), "track_update")

    def _init(self, slots, dets, det_emb, dbox, dconf):
        if len(slots) == 0:
            return
        t = self.table
        s, d = self._i32(slots), self._i32(dets)
        check(lib().trk_track_init(len(slots), _ptr(s), _ptr(d), _ptr(dbox), _ptr(dconf), _ptr(det_emb),
                                   _ptr(t.x), _ptr(t.P), _ptr(t.pbox), _ptr(t.last_conf), _ptr(t.enc),
                                   _ptr(t.bank), _ptr(t.bank_len), _ptr(t.bank_head), self.T,
                                   _stream(self.device)), "track_init")

    # --------------------------------------------------------------- step --
    def step(self, det_emb: torch.Tensor, dbox: torch.Tensor, dconf: torch.Tensor,
             N: Sequence[int], confs_host: Sequence[Sequence[float]],
             frame_ids: Optional[Sequence[int]] = None,
             after_launch: Optional[Any] = None) -> List[FrameResult]:
        """after_launch: optional callable run once the stage-1 LSAP is enqueued and
        before the host waits for its indices -- e.g. to enqueue the next frame's
        ROI Align + encoder on another stream while the solver runs."""
        cfg = self.cfg
        S = self.n_streams
        if det_emb.dim() != 3 or det_emb.shape[0] != S or det_emb.shape[2] != D:
            raise ValueError(f"det_embs must be [S, Nmax, {D}], got {tuple(det_emb.shape)}")
        Nmax = det_emb.shape[1]
        det_emb, dbox, dconf = det_emb.contiguous(), dbox.contiguous(), dconf.contiguous()
        frame_ids = list(frame_ids) if frame_ids is not None else [0] * S
        res = [FrameResult() for _ in range(S)]
        lost_after = int(cfg["lost_reid_after"])

        # frames without detections: every track missed, then purge (:467-471)
        active = [s for s in range(S) if int(N[s]) > 0]
        for s in range(S):
            if int(N[s]) == 0:
                st = self.streams[s]
                live = st.live_sorted()
                res[s].unmatched_tracks = st.tid[live].copy()
                st.miss[live] += 1
                self._purge(st)

        # predict every live track of the active streams (:474-475)
        live = {s: self.streams[s].live_sorted() for s in active}
        self._predict(np.concatenate([self.streams[s].base + live[s] for s in active])
                      if active else np.zeros(0, np.int32))

        # row split (:478-487): rows sorted by track id
        main = {s: live[s][self.streams[s].miss[live[s]] <= lost_after] for s in active}
        reid = {s: live[s][self.streams[s].miss[live[s]] > lost_after] for s in active}

        # ---- stage 1: fused cost + gate + LSAP over all active streams
        Mrow = max([len(main[s]) for s in active], default=0)
        unmatched_dets = {s: np.arange(int(N[s]), dtype=np.int64) for s in active}
        stage1 = {}
        C1 = None
        if Mrow > 0:
            row_slot = np.zeros((S, Mrow), np.int32)
            Ms = [0] * S
            Ns = [0] * S
            for s in active:
                m = main[s]
                row_slot[s, :len(m)] = self.streams[s].base + m
                Ms[s], Ns[s] = len(m), int(N[s])
            t = self.table
            C1 = build_cost(M=Ms, N=Ns, bank=t.bank, bank_len=t.bank_len, pbox=t.pbox,
                            conf_prev=t.last_conf, det_emb=det_emb, dbox=dbox, conf_cur=dconf,
                            params=self.params, gmean=t.gmean, gsinv=t.gsinv, gate_on=t.gate_on,
                            row_slot=self._i32(row_slot))["C_total"]
            lres = lsap_batched(C1, Ms, Ns, cost_max=float(cfg["cost_max"]))
            if after_launch is not None:
                after_launch()
                after_launch = None
            t_w = time.perf_counter()
            st_h = lres["status"].cpu().numpy()
            assign = lres["assign"].cpu().numpy()  # the host sync of mainTracking.py:503
            self.sync_wait_s += time.perf_counter() - t_w
            for s in active:
                if len(main[s]) == 0:
                    continue
                if st_h[s] == -1:
                    raise ValueError("matrix contains invalid numeric entries")
                if st_h[s] == -2:
                    raise ValueError("cost matrix is infeasible")
                a = assign[s, :len(main[s])]
                rows = np.flatnonzero(a >= 0)
                stage1[s] = (rows, a[rows].astype(np.int64))
                taken = np.zeros(int(N[s]), bool)
                taken[a[rows]] = True
                unmatched_dets[s] = np.flatnonzero(~taken)

        if after_launch is not None:  # no stage-1 rows this frame
            after_launch()

        # stage-1 state updates (:520-538)
        up_slots, up_dets, up_ci = [], [], []
        for s in active:
            st = self.streams[s]
            if s in stage1:
                rows, cols = stage1[s]
                sl = main[s][rows]
                up_slots.append(st.base + sl)
                up_dets.append(s * Nmax + cols)
                up_ci.append((s * Mrow + rows) * Nmax + cols)
                st.miss[sl] = 0
                st.age[sl] += 1
                st.last_frame[sl] = frame_ids[s]
                res[s].matches = np.stack([st.tid[sl], cols], 1)
                keep = np.ones(len(main[s]), bool)
                keep[rows] = False
                res[s].unmatched_tracks = st.tid[main[s][keep]].copy()
                st.miss[main[s][keep]] += 1
        if up_slots:
            self._update(np.concatenate(up_slots), np.concatenate(up_dets), C1, np.concatenate(up_ci),
                         cfg["cost_update_max"], cfg["maha_thr"], det_emb, dbox, dconf)

        # ---- stage 2: long-lost tracks, ReID-only (:545-599)
        s2 = [s for s in active if len(reid[s]) > 0 and len(unmatched_dets[s]) > 0]
        for s in active:
            if len(reid[s]) > 0 and len(unmatched_dets[s]) == 0:
                st = self.streams[s]
                res[s].unmatched_tracks = np.concatenate([res[s].unmatched_tracks, st.tid[reid[s]]])
                st.miss[reid[s]] += 1
        if s2:
            M2 = max(len(reid[s]) for s in s2)
            N2 = max(len(unmatched_dets[s]) for s in s2)
            F2 = len(s2)
            row_slot = np.zeros((F2, M2), np.int32)
            gidx = np.zeros((F2, N2), np.int64)
            for q, s in enumerate(s2):
                row_slot[q, :len(reid[s])] = self.streams[s].base + reid[s]
                u = np.asarray(unmatched_dets[s], np.int64)
                gidx[q, :len(u)] = s * Nmax + u
            g = torch.as_tensor(gidx.reshape(-1)).to(self.device)
            e2 = det_emb.reshape(-1, D).index_select(0, g).view(F2, N2, D)
            b2 = dbox.reshape(-1, 4).index_select(0, g).view(F2, N2, 4)
            c2 = dconf.reshape(-1).index_select(0, g).view(F2, N2)
            t = self.table
            Ms2 = [len(reid[s]) for s in s2]
            Ns2 = [len(unmatched_dets[s]) for s in s2]
            C2 = build_cost(M=Ms2, N=Ns2, bank=t.bank, bank_len=t.bank_len, pbox=t.pbox,
                            conf_prev=t.last_conf, det_emb=e2, dbox=b2, conf_cur=c2,
                            params=self.params_nogate, row_slot=self._i32(row_slot),
                            want=("C_app",))["C_app"]
            lres = lsap_batched(C2, Ms2, Ns2, cost_max=float(cfg["reid_only_cost_max"]))
            assign2 = lres["assign"].cpu().numpy()  # mainTracking.py:559
            st2 = lres["status"].cpu().numpy()
            up_slots, up_dets, up_ci = [], [], []
            for q, s in enumerate(s2):
                if st2[q] == -1:
                    raise ValueError("matrix contains invalid numeric entries")
                st = self.streams[s]
                a = assign2[q, :len(reid[s])]
                rows = np.flatnonzero(a >= 0)
                du = a[rows]
                u = np.asarray(unmatched_dets[s], np.int64)
                sl = reid[s][rows]
                up_slots.append(st.base + sl)
                up_dets.append(s * Nmax + u[du])
                up_ci.append((q * M2 + rows) * N2 + du)
                st.miss[sl] = 0
                st.age[sl] += 1
                st.last_frame[sl] = frame_ids[s]
                res[s].matches = np.concatenate([res[s].matches, np.stack([st.tid[sl], u[du]], 1)])
                keep = np.ones(len(reid[s]), bool)
                keep[rows] = False
                res[s].unmatched_tracks = np.concatenate([res[s].unmatched_tracks, st.tid[reid[s][keep]]])
                st.miss[reid[s][keep]] += 1
                left = np.ones(len(u), bool)
                left[du] = False
                unmatched_dets[s] = u[left]
            if up_slots:  # stage-2 gates: cost = C_app <= reid_only_cost_max, no motion gate
                self._update(np.concatenate(up_slots), np.concatenate(up_dets), C2, np.concatenate(up_ci),
                             cfg["reid_only_cost_max"], 1e18, det_emb, dbox, dconf)

        # ---- new tracks (:602 -> :362-373), then purge (:605)
        ini_slots, ini_dets = [], []
        for s in active:
            st = self.streams[s]
            ch = np.asarray(confs_host[s], np.float64)
            ud = unmatched_dets[s]
            new = ud[ch[ud] >= float(cfg["init_conf_min"])] if len(ud) else ud
            if len(new):
                free = np.flatnonzero(~st.alive)
                if len(free) < len(new):
                    raise RuntimeError(f"stream {s}: track capacity {st.cap} exhausted")
                sl = free[:len(new)]
                st.alive[sl] = True
                st.tid[sl] = np.arange(st.next_id, st.next_id + len(new))
                st.next_id += len(new)
                st.miss[sl] = 0
                st.age[sl] = 1
                st.last_frame[sl] = frame_ids[s]
                ini_slots.append(st.base + sl)
                ini_dets.append(s * Nmax + np.asarray(new, np.int64))
            res[s].unmatched_dets = unmatched_dets[s]
            self._purge(st)
        if ini_slots:
            self._init(np.concatenate(ini_slots), np.concatenate(ini_dets), det_emb, dbox, dconf)
        return res

    def _purge(self, st: StreamState):
        dead = st.alive & (st.miss > int(self.cfg["max_age"]))
        st.alive[dead] = False
        st.tid[dead] = -1


# ---------------------------------------------------------------- views --
@dataclass
class TrackMemory:
    """Read-only snapshot of reference TrackMemory fields (mainTracking.py:15-32)."""
    encoder_feat: Optional[np.ndarray] = None
    feat_historical: List[np.ndarray] = field(default_factory=list)
    last_conf: Optional[float] = None
    last_update_frame: Optional[int] = None
    last_bbox: Optional[Tuple[float, float, float, float]] = None
    age: int = 0
    misss_count: int = 0
    state: Optional[str] = None


@dataclass
class TrackState:
    """Read-only snapshot of reference TrackState (mainTracking.py:35-42)."""
    track_id: int
    kf_x: np.ndarray
    kf_P: np.ndarray
    memory: TrackMemory
    age: int = 1
    miss_count: int = 0
    state: str = "ACTIVE"


class Tracking:
    """mainTracking.Tracking drop-in (one stream).

    update(obj) takes the reference's obj dict {"embs", "bboxes", "confs",
    "input_hw", "frame_id"} and returns (matches [(track_id, det_idx)],
    unmatched_track_ids, unmatched_dets)."""

    def __init__(self, conf: Optional[Dict[str, Any]] = None, *, conf_path: Optional[str] = None,
                 capacity: int = 1024, device=None):
        self._mst = MultiStreamTracker(1, conf, capacity=capacity, device=device, conf_path=conf_path)
        c = self._mst.cfg
        self.init_conf_min = float(c["init_conf_min"]); self.hist_max = int(c["hist_max"])
        self.emb_top_k = int(c["emb_top_k"]); self.tau = float(c["app_tau"]); self.eps = float(c["eps"])
        self.w_app = float(c["w_app"]); self.w_bbox = float(c["w_bbox"]); self.w_conf = float(c["w_conf"])
        self.alpha = float(c["alpha"]); self.beta = float(c["beta"]); self.unmatch_cost = float(c["unmatch_cost"])
        self.cost_max = float(c["cost_max"]); self.max_age = int(c["max_age"]); self.ema_alpha = float(c["ema_alpha"])
        self.conf_update_min = float(c["conf_update_min"]); self.cost_update_max = float(c["cost_update_max"])
        self.maha_thr = float(c["maha_thr"]); self.lost_reid_after = int(c["lost_reid_after"])
        self.reid_sim_min = float(c["reid_sim_min"]); self.reid_only_cost_max = float(c["reid_only_cost_max"])

    @property
    def device(self):
        return self._mst.device

    @property
    def next_id(self) -> int:
        return self._mst.streams[0].next_id

    # -------------------------------------------------------------- update --
    def _dets(self, det_embs, det_boxes, det_confs):
        N = len(det_boxes)
        if N:
            emb = np.stack([np.asarray(e, dtype=np.float32).reshape(-1) for e in det_embs], 0)
            if emb.shape[1] != D:
                raise ValueError(f"det_embs must be {D}D, got {emb.shape}")
        else:
            emb = np.zeros((0, D), np.float32)
        dev = self.device
        e = torch.from_numpy(emb).to(dev).view(1, N, D)
        b = torch.as_tensor(np.asarray(det_boxes, np.float32).reshape(N, 4)).to(dev).view(1, N, 4)
        c = torch.as_tensor(np.asarray(det_confs, np.float32).reshape(N)).to(dev).view(1, N)
        return e, b, c

    def update(self, obj: Dict):
        """mainTracking.Tracking.update (mainTracking.py:450-610)."""
        det_embs = obj.get("embs", []) or []
        det_boxes = obj.get("bboxes", []) or []
        det_confs = obj.get("confs", []) or []
        input_hw = obj.get("input_hw", None)
        frame_id = obj.get("frame_id", None)
        if input_hw is None:
            raise ValueError("obj['input_hw'] is required")
        if frame_id is None:
            raise ValueError("obj['frame_id'] is required")
        if not (len(det_embs) == len(det_boxes) == len(det_confs)):
            raise ValueError("Length mismatch: embs/bboxes/confs must have same length")
        e, b, c = self._dets(det_embs, det_boxes, det_confs)
        r = self._mst.step(e, b, c, [len(det_boxes)], [list(det_confs)], [int(frame_id)])[0]
        return r.as_tuple()

    # --------------------------------------------- reference helper methods --
    def _rows(self, row_to_tid: Sequence[int]) -> np.ndarray:
        st = self._mst.streams[0]
        lut = {int(t): i for i, t in enumerate(st.tid) if st.alive[i]}
        try:
            return np.asarray([lut[int(t)] for t in row_to_tid], np.int32)
        except KeyError as k:
            raise KeyError(k.args[0]) from None

    def predict_all(self):
        """mainTracking.py:340-345 on the device table."""
        st = self._mst.streams[0]
        self._mst._predict(st.base + st.live_sorted())

    def build_C_app_topk(self, *, row_to_tid: List[int], det_embs, device=None, topk: int = 5,
                         use_topk_mean: bool = True, fallback_to_ema: bool = True) -> torch.Tensor:
        """mainTracking.py:141-211 -> [M, N] device tensor (1 - top-k mean)."""
        M, N = len(row_to_tid), len(det_embs)
        if M == 0 or N == 0:
            return torch.zeros((M, N), device=self.device)
        rows = self._rows(row_to_tid)
        e, b, c = self._dets(det_embs, [[0.0, 0.0, 1.0, 1.0]] * N, [1.0] * N)
        p = default_cost_params(self._mst.cfg, gate=False)
        p.topk = int(topk) if use_topk_mean else 1
        t = self._mst.table
        out = build_cost(M=[M], N=[N], bank=t.bank, bank_len=t.bank_len, pbox=t.pbox, conf_prev=t.last_conf,
                         det_emb=e, dbox=b, conf_cur=c, params=p, row_slot=self._mst._i32(rows[None]),
                         want=("C_app",))
        return out["C_app"][0]

    def cal_cost(self, *, row_to_tid: List[int], det_embs, det_boxes, det_confs, input_hw,
                 device=None, assign: Optional[List[int]] = None) -> Dict[str, Any]:
        """mainTracking.py:213-303 (ungated, like the reference's cal_cost)."""
        M, N = len(row_to_tid), len(det_embs)
        if M == 0 or N == 0:
            z = torch.zeros((M, N), device=self.device)
            return {"C_total": z, "C_app": z, "C_bbox": z, "C_center": z, "C_scale": z, "C_conf": z}
        rows = self._rows(row_to_tid)
        e, b, c = self._dets(det_embs, det_boxes, det_confs)
        t = self._mst.table
        out = build_cost(M=[M], N=[N], bank=t.bank, bank_len=t.bank_len, pbox=t.pbox, conf_prev=t.last_conf,
                         det_emb=e, dbox=b, conf_cur=c, params=self._mst.params_nogate,
                         row_slot=self._mst._i32(rows[None]),
                         want=("C_total", "C_app", "C_center", "C_scale", "C_conf"))
        o = {k: v[0] for k, v in out.items()}
        o["C_bbox"] = self.alpha * o["C_center"] + self.beta * o["C_scale"]
        if assign is not None:
            C_np = o["C_total"].cpu().numpy()
            cost, used = 0.0, set()
            for i, j in enumerate(assign):
                if j == -1:
                    cost += self.unmatch_cost
                elif j in used:
                    cost += 1e6
                else:
                    cost += C_np[i, j]
                    used.add(j)
            o["total_cost"] = float(cost)
        return o

    def apply_kalman_gating(self, C_total_np: np.ndarray, row_to_tid: List[int], det_boxes, *,
                            maha_thr: float = 13.28, INF: float = 1e9) -> np.ndarray:
        """mainTracking.py:306-338: C[i,j] = INF where the Mahalanobis d2 of
        det j under track i's predicted state exceeds maha_thr (in place)."""
        M, N = C_total_np.shape
        if M == 0 or N == 0:
            return C_total_np
        rows = self._rows(row_to_tid)
        dev = self.device
        t = self._mst.table
        idx = self._mst._i32(rows).long()
        p = default_cost_params(dict(w_app=1.0, w_bbox=0.0, w_conf=0.0, maha_thr=maha_thr), gate=True)
        p.inf_cost = float(INF)
        out = cost_combine(torch.from_numpy(np.ascontiguousarray(C_total_np, np.float32)).to(dev),
                           t.pbox.index_select(0, idx), t.last_conf.index_select(0, idx),
                           torch.as_tensor(np.asarray(det_boxes, np.float32).reshape(N, 4)).to(dev),
                           torch.ones(N, device=dev), p, t.gmean.index_select(0, idx),
                           t.gsinv.index_select(0, idx), torch.ones(M, device=dev, dtype=torch.int32))
        gated = out["C_total"].cpu().numpy() >= np.float32(INF)
        C_total_np[gated] = INF
        return C_total_np

    # ----------------------------------------------------------------- views --
    @property
    def tracks(self) -> Dict[int, TrackState]:
        """Snapshot of the live tracks (device -> host copy), keyed by track id
        in creation order, like the reference's self.tracks dict."""
        st = self._mst.streams[0]
        t = self._mst.table
        live = st.live_sorted()
        if len(live) == 0:
            return {}
        g = torch.as_tensor(st.base + live).to(self.device)
        x = t.x.index_select(0, g).cpu().numpy()
        P = t.P.index_select(0, g).cpu().numpy().reshape(-1, 8, 8)
        pb = t.pbox.index_select(0, g).cpu().numpy()
        lc = t.last_conf.index_select(0, g).cpu().numpy()
        enc = t.enc.index_select(0, g).cpu().numpy()
        bank = t.bank.index_select(0, g).cpu().numpy()
        bl = t.bank_len.index_select(0, g).cpu().numpy()
        bh = t.bank_head.index_select(0, g).cpu().numpy()
        out = {}
        for q, sl in enumerate(live):
            n, h = int(bl[q]), int(bh[q])
            order = [(h - n + k) % self._mst.T for k in range(n)]  # oldest first
            mem = TrackMemory(encoder_feat=enc[q], feat_historical=[bank[q, k] for k in order],
                              last_conf=float(lc[q]), last_update_frame=int(st.last_frame[sl]),
                              last_bbox=tuple(float(v) for v in pb[q]), age=int(st.age[sl]),
                              misss_count=int(st.miss[sl]),
                              state="ACTIVE" if st.miss[sl] == 0 else "LOST")
            out[int(st.tid[sl])] = TrackState(int(st.tid[sl]), x[q], P[q], mem, age=int(st.age[sl]),
                                              miss_count=int(st.miss[sl]), state=mem.state)
        return out
