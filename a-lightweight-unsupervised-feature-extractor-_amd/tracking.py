"""Tracker state machine over device-resident track tables.

Drop-in for reference model/mainTracking.py (class Tracking).
Every per-frame decision runs on gfx950 kernels, for all video streams at once:

  predict_all + row split        -> trk_step_begin   (:474-487)
  cal_cost + apply_kalman_gating -> trk_build_cost_dev (bank top-k appearance, bbox, conf, Mahalanobis)
  hungarian_assign               -> trk_lsap_dev     (scipy-exact SAP + the cost_max gate)
  stage-1 bookkeeping            -> trk_step_mid     (matches, misses, unmatched dets, stage-2 inputs)
  stage 2 (ReID-only)            -> trk_build_cost_dev (C_app) + trk_lsap_dev
  stage-2 bookkeeping, create_new_tracks, purge_dead -> trk_step_end
  update_matched + new tracks    -> trk_step_apply   (KF update, appearance gates, EMA, bank push, init)

The ids, miss counts, ages and live lists the reference keeps in Python dicts
live in HBM next to the Kalman state (TrackTable), so the host enqueues a frame
and never waits inside it; the frame's results reach the host through one
device->pinned copy.  ``MultiStreamTracker`` batches S independent streams;
``Tracking`` is its single-stream form with the reference's method names,
argument meanings and error behaviour (it waits for each frame, as the
reference returns each frame's matches).
"""
from __future__ import annotations

import ctypes
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import (_STEP_PTRS, TRK_F32, TRK_LSAP_MAX_DIM, StepConfig, StepState, TrkError, check,
                   lib)
from .ops import (_device, _ptr, _stream, current_stream as _current_stream, build_cost, cost_combine, default_cost_params,
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
    """Slot arrays of every track of every stream (layout: include/trk_amd.h):
    the Kalman state and memory bank, plus the bookkeeping the reference keeps
    in its Python dicts (alive, track id, miss count, age, last frame) and, per
    stream, the live slots in ascending track id with their count and next id."""

    def __init__(self, n_streams: int, cap: int, hist_max: int, device):
        S = n_streams * cap
        self.n_streams, self.cap, self.S, self.T, self.device = n_streams, cap, S, hist_max, device
        z = lambda *s, dt=torch.float32: torch.zeros(s, device=device, dtype=dt)
        self.x = z(S, 8, dt=torch.float64)
        self.P = z(S, 64, dt=torch.float64)
        self.pbox = z(S, 4)
        self.last_conf = z(S)
        self.gmean = z(S, 4, dt=torch.float64)
        self.gsinv = z(S, 16, dt=torch.float64)
        self.gate_on = torch.ones(S, device=device, dtype=torch.int32)
        self.enc = z(S, D)
        self.bank = z(S, hist_max, D)
        self.bank_len = z(S, dt=torch.int32)
        self.bank_head = z(S, dt=torch.int32)
        self.alive = z(S, dt=torch.int32)
        self.tid = torch.full((S,), -1, device=device, dtype=torch.int64)
        self.miss = z(S, dt=torch.int32)
        self.age = z(S, dt=torch.int32)
        self.last_frame = z(S, dt=torch.int64)
        self.order = z(n_streams, cap, dt=torch.int32)
        self.n_live = z(n_streams, dt=torch.int32)
        self.next_id = z(n_streams, dt=torch.int64)

    SLOT_ARRAYS = ("x", "P", "pbox", "last_conf", "gmean", "gsinv", "gate_on", "enc", "bank", "bank_len",
                   "bank_head", "alive", "tid", "miss", "age", "last_frame")

    def grown(self, cap: int) -> "TrackTable":
        """A copy with `cap` slots per stream (local slot numbers are kept)."""
        t = TrackTable(self.n_streams, cap, self.T, self.device)
        n = self.n_streams
        for k in self.SLOT_ARRAYS:
            old, new = getattr(self, k), getattr(t, k)
            new.view(n, cap, *new.shape[1:])[:, :self.cap].copy_(old.view(n, self.cap, *old.shape[1:]))
        t.order[:, :self.cap].copy_(self.order)
        t.n_live.copy_(self.n_live)
        t.next_id.copy_(self.next_id)
        return t


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


class SolverStallError(TrkError):
    """The LSAP solver's bounded wait expired (an internal stall, not an
    infeasible matrix); the frame's result is not valid."""


def _raise_status(st: int, s: int):
    if st == -1:
        raise ValueError("matrix contains invalid numeric entries")
    if st == -2:
        raise ValueError("cost matrix is infeasible")
    if st == -3:
        raise SolverStallError(f"stream {s}: LSAP solver stalled (bounded wait expired)")
    if st == -4:
        raise TrkError(f"stream {s}: live tracks exceed the frame's launch bound (internal error)")
    if st == -5:
        raise TrkError(f"stream {s}: track capacity exhausted (internal error: the table grows before a frame)")
    raise TrkError(f"stream {s}: tracker step failed with status {st}")


class StepHandle:
    """A frame in flight: its results are copied into pinned host memory by the
    stream; result() waits for that copy only (frames are consumed in order)."""

    def __init__(self, tracker, seq, buf, event, S, Nmax, cap, stride, after_N):
        self._tr, self.seq, self._buf, self._ev = tracker, seq, buf, event
        # the results layout of the frame's launch (the scratch may be re-sized later)
        self._S, self._Nmax, self._cap, self._stride, self._after = S, Nmax, cap, stride, after_N
        self._res = None

    def done(self) -> bool:
        return self._res is not None or self._ev.query()

    def result(self) -> List[FrameResult]:
        if self._res is None:
            self._tr._consume_through(self)
        if isinstance(self._res, Exception):
            raise self._res
        return self._res

    def _parse(self):
        self._ev.synchronize()
        stride, Nmax, cap = self._stride, self._Nmax, self._cap
        r = self._buf.numpy()[:self._S * stride].reshape(self._S, stride)
        out, err = [], None
        for s in range(self._S):
            h = r[s, :8]
            if h[4] != 0 and err is None:
                try:
                    _raise_status(int(h[4]), s)
                except Exception as e:  # noqa: BLE001 -- re-raised by result()
                    err = e
            nm, nu, nd = int(h[0]), int(h[1]), int(h[2])
            mt, md = r[s, 8:8 + Nmax], r[s, 8 + Nmax:8 + 2 * Nmax]
            ut, ud = r[s, 8 + 2 * Nmax:8 + 2 * Nmax + cap], r[s, 8 + 2 * Nmax + cap:8 + 3 * Nmax + cap]
            out.append(FrameResult(np.stack([mt[:nm], md[:nm]], 1).copy(), ut[:nu].copy(), ud[:nd].copy()))
        live = r[:, 3].copy()
        self._res = err if err is not None else out
        return live


class MultiStreamTracker:
    """S independent trackers (one per video stream) advanced together.

    step() takes the detections of one frame of every stream, already on the
    device: det_emb [S, Nmax, 128] f32, dbox [S, Nmax, 4] f32, dconf [S, Nmax]
    f32 and the counts N[s].  Returns one FrameResult per stream, identical to
    what mainTracking.Tracking.update would return for that stream.

    Every per-frame decision is made on the device (trk_step_* + the cost and
    LSAP kernels, one launch sequence per frame for all streams): the host
    enqueues a frame and never waits inside it.  step_async() returns a
    StepHandle whose results arrive through one device->pinned-host copy; at
    most `max_inflight` frames are left unread (the oldest is then consumed).
    The table grows (doubling `capacity`) when a frame could overflow it, as the
    reference's dict of tracks does (mainTracking.py:362-373)."""

    def __init__(self, n_streams: int, conf: Optional[Dict[str, Any]] = None, *,
                 capacity: int = 1024, device=None, conf_path: Optional[str] = None, max_inflight: int = 3):
        self.cfg = tracker_conf(conf, conf_path)
        self.n_streams = n_streams
        self.device = torch.device(device) if device is not None else _device()
        self.T = int(self.cfg["hist_max"])
        if not 1 <= self.T <= 1024:
            raise ValueError(f"hist_max must be in [1, 1024], got {self.T}")
        self.table = TrackTable(n_streams, int(capacity), self.T, self.device)
        self.params = default_cost_params(self.cfg, gate=True)
        self.params_nogate = default_cost_params(self.cfg, gate=False)
        self._cost_max = float(self.cfg["cost_max"])
        self._reid_max = float(self.cfg["reid_only_cost_max"])
        self.max_inflight = max(1, int(max_inflight))
        self._nmax = 0
        self._pending: List[StepHandle] = []
        self._pool: List[torch.Tensor] = []
        self._seq = 0
        self._live_exact = np.zeros(n_streams, np.int64)   # n_live after the last consumed frame
        self._cum_N = np.zeros(n_streams, np.int64)        # detections launched so far
        self._cum_at_exact = np.zeros(n_streams, np.int64)
        self._last_stream = None  # raw stream handle of the last frame's launches
        self.sync_wait_s = 0.0  # host time blocked waiting on results (bench diagnostics)

    @property
    def cap(self) -> int:
        return self.table.cap

    # ---------------------------------------------------------- buffers --
    def _scratch(self, Nmax: int):
        """per-frame device scratch sized for (capacity, Nmax)"""
        if Nmax <= self._nmax and self._scr_cap == self.cap:
            return
        # frames in flight still use the old scratch (their kernels hold its pointers): let
        # them finish before it is freed
        self.drain()
        self._nmax = max(Nmax, self._nmax)
        self._scr_cap = self.cap
        S, cap, Nm, dev = self.n_streams, self.cap, self._nmax, self.device
        i32 = lambda *s: torch.zeros(s, device=dev, dtype=torch.int32)
        f32 = lambda *s: torch.zeros(s, device=dev, dtype=torch.float32)
        self._scr = dict(ndet=i32(S), frame_id=torch.zeros(S, device=dev, dtype=torch.int64), flags=i32(S),
                         m1=i32(S), row1=i32(S, cap), m2=i32(S), row2=i32(S, cap), n2=i32(S), ud=i32(S, Nm),
                         freelist=i32(S, cap), e2=f32(S, Nm, D), b2=f32(S, Nm, 4), c2=f32(S, Nm),
                         ap_n=i32(S), ap_slot=i32(S, Nm), ap_det=i32(S, Nm), ap_kind=i32(S, Nm), ap_cost=f32(S, Nm),
                         lsap_status=i32(2, S))
        self._stride = int(lib().trk_step_result_stride(cap, Nm))
        self._scr["result"] = torch.zeros(S * self._stride, device=dev, dtype=torch.int64)
        km = min(cap, Nm)
        self._lsap = [dict(rows=torch.empty((S, km), device=dev, dtype=torch.int64),
                           cols=torch.empty((S, km), device=dev, dtype=torch.int64),
                           count=torch.empty(S, device=dev, dtype=torch.int32),
                           assign=torch.empty((S, cap), device=dev, dtype=torch.int32)) for _ in range(2)]
        self._C = [torch.empty(S * cap * Nm, device=dev, dtype=torch.float32) for _ in range(2)]
        self._cost_work = torch.empty(int(lib().trk_cost_work_bytes(S, Nm)), device=dev, dtype=torch.uint8)
        self._pool = []  # result buffers of the old layout
        t = self.table
        self._state = StepState(*[_ptr(getattr(t, n)) if hasattr(t, n) and n not in self._scr else
                                  _ptr(self._scr[n]) for n in _STEP_PTRS])
        self._conf = StepConfig(S, cap, Nm, self.T, int(self.cfg["lost_reid_after"]), int(self.cfg["max_age"]),
                                float(self.cfg["init_conf_min"]), float(self.cfg["conf_update_min"]),
                                float(self.cfg["cost_update_max"]), float(self.cfg["reid_only_cost_max"]),
                                float(self.cfg["maha_thr"]), float(self.cfg["ema_alpha"]))
        # the launch arguments that only change with the scratch / table: converted once
        # (a frame's ~60 pointer conversions were host time the pipeline waited for)
        P = _ptr
        t, l1, l2 = self.table, self._lsap[0], self._lsap[1]
        self._fp = dict(
            st=ctypes.byref(self._state), cf=ctypes.byref(self._conf), prm=ctypes.byref(self.params),
            prm_ng=ctypes.byref(self.params_nogate), m1=P(self._scr["m1"]), ndet=P(self._scr["ndet"]),
            row1=P(self._scr["row1"]), m2=P(self._scr["m2"]), n2=P(self._scr["n2"]), row2=P(self._scr["row2"]),
            e2=P(self._scr["e2"]), b2=P(self._scr["b2"]), c2=P(self._scr["c2"]),
            ls0=P(self._scr["lsap_status"][0]), ls1=P(self._scr["lsap_status"][1]),
            bank=P(t.bank), bank_len=P(t.bank_len), pbox=P(t.pbox), last_conf=P(t.last_conf), gmean=P(t.gmean),
            gsinv=P(t.gsinv), gate_on=P(t.gate_on), C1=P(self._C[0]), C2=P(self._C[1]), work=P(self._cost_work),
            r1=P(l1["rows"]), c1=P(l1["cols"]), n1=P(l1["count"]), a1=P(l1["assign"]),
            r2=P(l2["rows"]), cc2=P(l2["cols"]), nn2=P(l2["count"]), a2=P(l2["assign"]))

    _scr_cap = -1

    def _result_buf(self) -> torch.Tensor:
        if self._pool:
            return self._pool.pop()
        return torch.empty(self.n_streams * self._stride, dtype=torch.int64, pin_memory=True)

    # ------------------------------------------------------- consumption --
    def _consume_through(self, h: StepHandle):
        t0 = time.perf_counter()
        while self._pending:
            q = self._pending.pop(0)
            live = q._parse()
            self._live_exact = live
            self._cum_at_exact = q._after
            if q._buf.numel() == self.n_streams * self._stride:
                self._pool.append(q._buf)
            if q is h:
                break
        self.sync_wait_s += time.perf_counter() - t0

    def drain(self):
        """Wait for every frame in flight (their results stay readable)."""
        if self._pending:
            self._consume_through(self._pending[-1])

    def _live_ub(self) -> np.ndarray:
        """upper bound of each stream's live tracks now: the last read count plus
        every detection launched since (each can at most start a track)"""
        return self._live_exact + (self._cum_N - self._cum_at_exact)

    def _grow(self, need: int):
        cap = self.cap
        while cap < need:
            cap *= 2
        self.drain()
        self.table = self.table.grown(cap)
        self._nmax = 0
        self._scratch(max(1, self._last_nmax))

    # --------------------------------------------------------------- step --
    def step_async(self, det_emb: torch.Tensor, dbox: torch.Tensor, dconf: torch.Tensor, N: Sequence[int],
                   frame_ids: Optional[Sequence[int]] = None, dconf64: Optional[torch.Tensor] = None,
                   after_launch: Optional[Any] = None) -> StepHandle:
        S = self.n_streams
        if det_emb.dim() != 3 or det_emb.shape[0] != S or det_emb.shape[2] != D:
            raise ValueError(f"det_embs must be [S, Nmax, {D}], got {tuple(det_emb.shape)}")
        Nmax = det_emb.shape[1]
        N = np.asarray([int(n) for n in N], np.int64)
        if len(N) != S or (N < 0).any() or (N > Nmax).any():
            raise ValueError("N must hold one count in [0, Nmax] per stream")
        if Nmax == 0:  # pad to one (never read) detection row
            det_emb = torch.zeros((S, 1, D), device=self.device)
            dbox = torch.zeros((S, 1, 4), device=self.device)
            dconf = torch.zeros((S, 1), device=self.device)
            dconf64 = None
            Nmax = 1
        det_emb = det_emb.to(self.device, torch.float32).contiguous()
        dbox = dbox.to(self.device, torch.float32).contiguous()
        dconf = dconf.to(self.device, torch.float32).contiguous()
        if dconf64 is not None:
            dconf64 = dconf64.to(self.device, torch.float64).contiguous()
        self._last_nmax = Nmax
        # a frame can add at most N[s] tracks: grow the table before it could overflow
        if (self._live_ub() + N > self.cap).any():
            self.drain()
            need = int((self._live_exact + N).max())
            if need > self.cap:
                self._grow(need)
        self._scratch(Nmax)
        if Nmax > self._nmax:
            raise AssertionError("scratch sizing")
        if len(self._pending) >= self.max_inflight:
            self._consume_through(self._pending[0])
        if self._live_ub().max() > TRK_LSAP_MAX_DIM:  # the bound counts frames in flight: read them
            self.drain()
        Mb = int(min(self.cap, max(1, self._live_ub().max())))
        self.last_Mb = Mb  # row stride of this frame's stage cost matrices (tools, tests)
        if Mb > TRK_LSAP_MAX_DIM:
            raise NotImplementedError(f"more than {TRK_LSAP_MAX_DIM} live tracks in one stream")
        fid = np.asarray(list(frame_ids) if frame_ids is not None else [0] * S, np.int64)
        st, cf, t, sc = self._state, self._conf, self.table, self._scr
        Nm = self._nmax
        if Nm != Nmax:  # detections laid out with the scratch's stride
            pad = lambda x, *tail: torch.nn.functional.pad(x, (0, 0) * len(tail) + (0, Nm - Nmax))
            det_emb, dbox, dconf = pad(det_emb, D), pad(dbox, 4), pad(dconf)
            if dconf64 is not None:
                dconf64 = pad(dconf64)
        stream = _stream(self.device)
        if self._last_stream is not None and stream.value != self._last_stream:
            # the caller switched streams: frame k+1 reads the table frame k writes, so
            # order it behind everything enqueued on the previous frame's stream
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(self._last_stream, device=self.device))
            _current_stream(self.device).wait_event(ev)
        self._last_stream = stream.value
        L = lib()
        hN = (ctypes.c_int32 * S)(*N.tolist())
        hF = (ctypes.c_int64 * S)(*fid.tolist())
        fp = self._fp
        pe, pb, pc, pc64 = _ptr(det_emb), _ptr(dbox), _ptr(dconf), _ptr(dconf64)
        check(L.trk_step_begin(fp["st"], fp["cf"], hN, hF, Mb, stream), "step_begin")
        kmax = min(self.cap, Nm)
        check(L.trk_build_cost_dev(S, Mb, Nm, fp["m1"], fp["ndet"], fp["row1"], self.cap, self.T, fp["bank"],
                                   fp["bank_len"], fp["pbox"], fp["last_conf"], fp["gmean"], fp["gsinv"],
                                   fp["gate_on"], pe, pb, pc, fp["prm"], fp["C1"], None, fp["work"], stream),
              "build_cost (stage 1)")
        check(L.trk_lsap_dev(S, fp["C1"], TRK_F32, Nm, Mb * Nm, fp["m1"], fp["ndet"], Mb, Nm, kmax, fp["r1"], fp["c1"],
                             fp["n1"], fp["ls0"], fp["a1"], Mb, self._cost_max, stream), "lsap (stage 1)")
        check(L.trk_step_mid(fp["st"], fp["cf"], Mb, fp["C1"], fp["a1"], pe, pb, pc, stream), "step_mid")
        check(L.trk_build_cost_dev(S, Mb, Nm, fp["m2"], fp["n2"], fp["row2"], self.cap, self.T, fp["bank"],
                                   fp["bank_len"], fp["pbox"], fp["last_conf"], None, None, None, fp["e2"], fp["b2"],
                                   fp["c2"], fp["prm_ng"], None, fp["C2"], fp["work"], stream), "build_cost (stage 2)")
        check(L.trk_lsap_dev(S, fp["C2"], TRK_F32, Nm, Mb * Nm, fp["m2"], fp["n2"], Mb, Nm, kmax, fp["r2"], fp["cc2"],
                             fp["nn2"], fp["ls1"], fp["a2"], Mb, self._reid_max, stream), "lsap (stage 2)")
        check(L.trk_step_end(fp["st"], fp["cf"], Mb, fp["C2"], fp["a2"], pc64, pc, stream), "step_end")
        buf = self._result_buf()
        buf.copy_(sc["result"], non_blocking=True)
        ev = torch.cuda.Event()
        cur = _current_stream(self.device)
        ev.record(cur)
        check(L.trk_step_apply(fp["st"], fp["cf"], pe, pb, pc, pc64, stream), "step_apply")
        # the caller's detection tensors must outlive the frame's kernels
        for x in (det_emb, dbox, dconf, dconf64):
            if x is not None:
                x.record_stream(cur)
        self._cum_N = self._cum_N + N
        self._seq += 1
        h = StepHandle(self, self._seq, buf, ev, S, Nm, self.cap, self._stride, self._cum_N.copy())
        self._pending.append(h)
        if after_launch is not None:
            after_launch()
        return h

    def step(self, det_emb: torch.Tensor, dbox: torch.Tensor, dconf: torch.Tensor,
             N: Sequence[int], confs_host: Optional[Sequence[Sequence[float]]] = None,
             frame_ids: Optional[Sequence[int]] = None,
             after_launch: Optional[Any] = None) -> List[FrameResult]:
        """Synchronous step.  confs_host: optional host copies of the confidences
        (the caller's floats: the creation and appearance gates compare them in
        double like the reference, mainTracking.py:365,416); otherwise dconf is
        used.  after_launch: optional callable run once the frame is enqueued and
        before the host waits for its results."""
        dconf64 = None
        if confs_host is not None:
            Nmax = det_emb.shape[1]
            h = np.zeros((self.n_streams, max(Nmax, 1)), np.float64)
            for s, c in enumerate(confs_host):
                c = np.asarray(c, np.float64).reshape(-1)
                h[s, :len(c)] = c
            dconf64 = torch.from_numpy(h[:, :Nmax] if Nmax else h).to(self.device)
        return self.step_async(det_emb, dbox, dconf, N, frame_ids, dconf64, after_launch).result()

    # ------------------------------------------------------ device views --
    def live_slots(self, s: int) -> np.ndarray:
        """global slots of stream s's live tracks in ascending track id (syncs)"""
        self.drain()
        n = int(self.table.n_live[s].item())
        return s * self.cap + self.table.order[s, :n].cpu().numpy().astype(np.int64)

    def _predict(self, slots: np.ndarray):
        if len(slots) == 0:
            return
        t = self.table
        sl = torch.as_tensor(np.ascontiguousarray(slots, np.int32)).to(self.device)
        check(lib().trk_kf_predict(len(slots), _ptr(sl), _ptr(t.x), _ptr(t.P), _ptr(t.pbox), _ptr(t.gmean),
                                   _ptr(t.gsinv), _stream(self.device)), "kf_predict")


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
        self._mst.drain()
        return int(self._mst.table.next_id[0].item())

    def _i32(self, a) -> torch.Tensor:
        return torch.as_tensor(np.ascontiguousarray(a, np.int32)).to(self.device)

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
        live = self._mst.live_slots(0)
        tids = self._mst.table.tid[torch.as_tensor(live, device=self.device)].cpu().numpy()
        lut = {int(t): int(g) for t, g in zip(tids, live)}
        try:
            return np.asarray([lut[int(t)] for t in row_to_tid], np.int32)
        except KeyError as k:
            raise KeyError(k.args[0]) from None

    def predict_all(self):
        """mainTracking.py:340-345 on the device table."""
        self._mst._predict(self._mst.live_slots(0))

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
                         det_emb=e, dbox=b, conf_cur=c, params=p, row_slot=self._i32(rows[None]),
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
                         row_slot=self._i32(rows[None]),
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
        idx = self._i32(rows).long()
        # the kernel's own gate decision (d2 > maha_thr): all weights 0 on a zero C_app, and a
        # gated pair's "cost" 1 -- so the mask is exactly the gate, whatever C_total holds
        p = default_cost_params(dict(w_app=0.0, w_bbox=0.0, w_conf=0.0, maha_thr=maha_thr), gate=True)
        p.inf_cost = 1.0
        out = cost_combine(torch.zeros((M, N), device=dev), t.pbox.index_select(0, idx),
                           t.last_conf.index_select(0, idx),
                           torch.as_tensor(np.asarray(det_boxes, np.float32).reshape(N, 4)).to(dev),
                           torch.ones(N, device=dev), p, t.gmean.index_select(0, idx),
                           t.gsinv.index_select(0, idx), torch.ones(M, device=dev, dtype=torch.int32))
        gated = out["C_total"].cpu().numpy() == np.float32(1.0)
        C_total_np[gated] = INF
        return C_total_np

    # ----------------------------------------------------------------- views --
    @property
    def tracks(self) -> Dict[int, TrackState]:
        """Snapshot of the live tracks (device -> host copy), keyed by track id
        in creation order, like the reference's self.tracks dict."""
        t = self._mst.table
        live = self._mst.live_slots(0)
        if len(live) == 0:
            return {}
        g = torch.as_tensor(live).to(self.device)
        x = t.x.index_select(0, g).cpu().numpy()
        P = t.P.index_select(0, g).cpu().numpy().reshape(-1, 8, 8)
        pb = t.pbox.index_select(0, g).cpu().numpy()
        lc = t.last_conf.index_select(0, g).cpu().numpy()
        enc = t.enc.index_select(0, g).cpu().numpy()
        bank = t.bank.index_select(0, g).cpu().numpy()
        bl = t.bank_len.index_select(0, g).cpu().numpy()
        bh = t.bank_head.index_select(0, g).cpu().numpy()
        tid = t.tid.index_select(0, g).cpu().numpy()
        age = t.age.index_select(0, g).cpu().numpy()
        miss = t.miss.index_select(0, g).cpu().numpy()
        lf = t.last_frame.index_select(0, g).cpu().numpy()
        out = {}
        for q in range(len(live)):
            n, h = int(bl[q]), int(bh[q])
            order = [(h - n + k) % self._mst.T for k in range(n)]  # oldest first
            mem = TrackMemory(encoder_feat=enc[q], feat_historical=[bank[q, k] for k in order],
                              last_conf=float(lc[q]), last_update_frame=int(lf[q]),
                              last_bbox=tuple(float(v) for v in pb[q]), age=int(age[q]),
                              misss_count=int(miss[q]),
                              state="ACTIVE" if miss[q] == 0 else "LOST")
            out[int(tid[q])] = TrackState(int(tid[q]), x[q], P[q], mem, age=int(age[q]),
                                          miss_count=int(miss[q]), state=mem.state)
        return out
