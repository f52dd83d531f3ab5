"""Test-side second implementation of the tracker step: the per-track
bookkeeping (ids, miss counts, ages, row split, births, purge) on the host in
numpy, the numeric stages on the product kernels (trk_kf_predict,
trk_build_cost, trk_lsap, trk_track_update, trk_track_init).  It was the
product path of round 1 (frame-exact against the reference goldens); the
product now makes every bookkeeping decision on the device (trk_step_*), and
tests/test_tracking_gpu.py runs both over long random scenes and requires
identical results.  Test infrastructure only.
"""
from __future__ import annotations

import importlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

_trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
_t = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.tracking")
_ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
check, lib = _trk._lib.check, _trk._lib.lib
_device, _ptr, _stream = _ops._device, _ops._ptr, _ops._stream
build_cost, cost_combine, default_cost_params, lsap_batched = (_ops.build_cost, _ops.cost_combine,
                                                               _ops.default_cost_params, _ops.lsap_batched)
tracker_conf, FrameResult, D = _t.tracker_conf, _t.FrameResult, _t.D


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




class HostBookkeepingTracker:
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
        self.table = TrackTable(n_streams * capacity, self.T, self.device)
        self.streams = [StreamState(capacity, s * capacity) for s in range(n_streams)]
        self.params = default_cost_params(self.cfg, gate=True)
        self.params_nogate = default_cost_params(self.cfg, gate=False)

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
            st_h = lres["status"].cpu().numpy()
            assign = lres["assign"].cpu().numpy()  # the host sync of mainTracking.py:503
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


