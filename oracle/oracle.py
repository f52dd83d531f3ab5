"""CPU oracle for the tracker hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It is the checker, never the thing measured or shipped.

Contents
  roi_align(...)          ctypes -> oracle/build/liboracle.so ora_roi_align
                          (torchvision 0.20.1 CPU semantics, SURVEY A.1;
                          reference call tracking.py:214-221).  torchvision is
                          absent here: parity pinned by analytic KATs only.
  cost_build(...)         ora_cost_build: build_C_app_topk + costCard.cal_cost
                          + apply_kalman_gating (mainTracking.py:141-338,
                          costCard.py:109-268, KalmanFilter.py:105-116).
                          Pinned against tests/golden/track_golden_*.npz.
  lsap(C)                 ora_lsap: scipy linear_sum_assignment restated
                          (hung.py:28).  Pinned against tests/golden/lsap_golden.npz.
  hungarian_assign(C,cm)  restates hung.py:5-45 over ora_lsap.
  encoder_forward(sd, x)  plain-torch fp32 restatement of the encoder eval graph
                          (encoderAndHead.py:21-26, card.py:48-169), pinned
                          against tests/golden/encoder_golden.npz.
  det_nms(pred, ...)      ora_det_nms: YOLOv7 non_max_suppression defaults +
                          torchvision CPU nms + scale_coords/xyxy2xywh
                          (general.py:255-341,608-700; yoloDetects2.py:111-160).
                          torchvision absent: pinned by KATs in tests/test_detect.py.
  train_rois(...)         PreProcess._preprocess_roi box preparation
                          (trainingCard.py:24-69) in numpy f32; unpinned by a
                          reference run (torchvision/cv2 imports), KATs only.
  KalmanFilterRestated    filterpy 1.4.5 KalmanFilter predict/update restated
                          (third-party, absent from reference + image; used
                          via KalmanFilter.py:57-101).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i = ctypes.c_int
        L.ora_roi_align.argtypes = [P, i, i, i, i, P, i, ctypes.c_float, i, i, i, i, P]
        L.ora_roi_align.restype = None
        L.ora_cost_build.argtypes = [P, P, i, i, P, i, i, P, P, P, P, P, P, P, P,
                                     P, P, P, P, P]
        L.ora_cost_build.restype = None
        L.ora_cost_combine.argtypes = [P, i, i, P, P, P, P, P, P, P, P, P, P, P, P]
        L.ora_cost_combine.restype = None
        L.ora_det_nms.argtypes = [P, ctypes.c_int64, i, ctypes.c_float, ctypes.c_double, i, i, i, i,
                                  P, P, P, P]
        L.ora_det_nms.restype = i
        L.ora_lsap.argtypes = [P, ctypes.c_int64, ctypes.c_int64, P, P]
        L.ora_lsap.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------
def roi_align(inp: np.ndarray, rois: np.ndarray, output_size, spatial_scale: float,
              sampling_ratio: int = 2, aligned: bool = True) -> np.ndarray:
    inp = np.ascontiguousarray(inp, dtype=np.float32)
    rois = np.ascontiguousarray(rois, dtype=np.float32).reshape(-1, 5)
    B, C, H, W = inp.shape
    PH, PW = (output_size, output_size) if isinstance(output_size, int) else output_size
    K = rois.shape[0]
    out = np.zeros((K, C, PH, PW), dtype=np.float32)
    if K:
        lib().ora_roi_align(_p(inp), B, C, H, W, _p(rois), K, float(np.float32(spatial_scale)),
                            PH, PW, int(sampling_ratio), int(bool(aligned)), _p(out))
    return out


class _CostParams(ctypes.Structure):
    _fields_ = [("w_app", ctypes.c_float), ("w_bbox", ctypes.c_float),
                ("w_conf", ctypes.c_float), ("alpha", ctypes.c_float),
                ("beta", ctypes.c_float), ("maha_thr", ctypes.c_double),
                ("inf_cost", ctypes.c_float), ("topk", ctypes.c_int)]


def cost_build(bank, bank_len, det, pbox, dbox, conf_prev, conf_cur,
               gmean=None, gsinv=None, gate_mask=None, *, w_app=1.0, w_bbox=0.3,
               w_conf=0.2, alpha=1.0, beta=0.5, maha_thr=9.49, inf_cost=1e9, topk=5):
    bank = np.ascontiguousarray(bank, dtype=np.float32)
    M, Tmax, D = bank.shape
    det = np.ascontiguousarray(det, dtype=np.float32).reshape(-1, D)
    N = det.shape[0]
    bank_len = np.ascontiguousarray(bank_len, dtype=np.int32)
    pbox = np.ascontiguousarray(pbox, dtype=np.float32).reshape(M, 4)
    dbox = np.ascontiguousarray(dbox, dtype=np.float32).reshape(N, 4)
    conf_prev = np.ascontiguousarray(conf_prev, dtype=np.float32).reshape(M)
    conf_cur = np.ascontiguousarray(conf_cur, dtype=np.float32).reshape(N)
    if gmean is None:
        gmean = np.zeros((M, 4)); gsinv = np.zeros((M, 16)); gate_mask = np.zeros(M, np.int32)
    gmean = np.ascontiguousarray(gmean, dtype=np.float64).reshape(M, 4)
    gsinv = np.ascontiguousarray(gsinv, dtype=np.float64).reshape(M, 16)
    gate_mask = np.ascontiguousarray(gate_mask, dtype=np.int32).reshape(M)
    prm = _CostParams(w_app, w_bbox, w_conf, alpha, beta, maha_thr, inf_cost, topk)
    outs = {k: np.zeros((M, N), np.float32) for k in ("C_total", "C_app", "C_center", "C_scale", "C_conf")}
    if M and N:
        lib().ora_cost_build(_p(bank), _p(bank_len), M, Tmax, _p(det), N, D, _p(pbox), _p(dbox),
                             _p(conf_prev), _p(conf_cur), _p(gmean), _p(gsinv), _p(gate_mask),
                             ctypes.byref(prm), _p(outs["C_total"]), _p(outs["C_app"]),
                             _p(outs["C_center"]), _p(outs["C_scale"]), _p(outs["C_conf"]))
    outs["C_bbox"] = (np.float32(alpha) * outs["C_center"] + np.float32(beta) * outs["C_scale"]).astype(np.float32)
    return outs


def cost_combine(C_app, pbox, dbox, conf_prev, conf_cur, gmean=None, gsinv=None,
                 gate_mask=None, *, w_app=1.0, w_bbox=0.3, w_conf=0.2, alpha=1.0, beta=0.5,
                 maha_thr=9.49, inf_cost=1e9):
    """costCard.cal_cost (+ optional Kalman gating) from a given C_app."""
    C_app = np.ascontiguousarray(C_app, dtype=np.float32)
    M, N = C_app.shape
    pbox = np.ascontiguousarray(pbox, dtype=np.float32).reshape(M, 4)
    dbox = np.ascontiguousarray(dbox, dtype=np.float32).reshape(N, 4)
    conf_prev = np.ascontiguousarray(conf_prev, dtype=np.float32).reshape(M)
    conf_cur = np.ascontiguousarray(conf_cur, dtype=np.float32).reshape(N)
    if gmean is None:
        gmean = np.zeros((M, 4)); gsinv = np.zeros((M, 16)); gate_mask = np.zeros(M, np.int32)
    gmean = np.ascontiguousarray(gmean, dtype=np.float64).reshape(M, 4)
    gsinv = np.ascontiguousarray(gsinv, dtype=np.float64).reshape(M, 16)
    gate_mask = np.ascontiguousarray(gate_mask, dtype=np.int32).reshape(M)
    prm = _CostParams(w_app, w_bbox, w_conf, alpha, beta, maha_thr, inf_cost, 0)
    outs = {k: np.zeros((M, N), np.float32) for k in ("C_total", "C_center", "C_scale", "C_conf")}
    if M and N:
        lib().ora_cost_combine(_p(C_app), M, N, _p(pbox), _p(dbox), _p(conf_prev), _p(conf_cur),
                               _p(gmean), _p(gsinv), _p(gate_mask), ctypes.byref(prm),
                               _p(outs["C_total"]), _p(outs["C_center"]), _p(outs["C_scale"]),
                               _p(outs["C_conf"]))
    outs["C_bbox"] = (np.float32(alpha) * outs["C_center"] + np.float32(beta) * outs["C_scale"]).astype(np.float32)
    return outs


def gate_params(kf_x, kf_P):
    """Per-track gate inputs: H x and (H P H^T + R + 1e-9 I)^-1 in float64
    (KalmanFilter.gating_distance_maha, KalmanFilter.py:105-116; R = I4)."""
    kf_x = np.asarray(kf_x, np.float64).reshape(-1, 8)
    kf_P = np.asarray(kf_P, np.float64).reshape(-1, 8, 8)
    mean = kf_x[:, :4].copy()
    S = kf_P[:, :4, :4] + np.eye(4)[None] + 1e-9 * np.eye(4)[None]
    return mean, np.linalg.inv(S).reshape(-1, 16)


def lsap(C) -> Tuple[np.ndarray, np.ndarray]:
    C = np.asarray(C)
    if C.ndim != 2:
        raise ValueError("expected a matrix (2-d array), got a %r array" % (C.shape,))
    C = np.ascontiguousarray(C, dtype=np.float64)
    nr, nc = C.shape
    k = min(nr, nc)
    rows = np.zeros(k, np.int64)
    cols = np.zeros(k, np.int64)
    st = lib().ora_lsap(_p(C), nr, nc, _p(rows), _p(cols))
    if st == -1:
        raise ValueError("matrix contains invalid numeric entries")
    if st == -2:
        raise ValueError("cost matrix is infeasible")
    return rows, cols


def hungarian_assign(C_total: np.ndarray, cost_max: float = 1e9):
    M, N = C_total.shape
    if M == 0 and N == 0:
        return [], [], []
    if M == 0:
        return [], [], list(range(N))
    if N == 0:
        return [], list(range(M)), []
    r, c = lsap(C_total)
    matches, mt, md = [], set(), set()
    for i, j in zip(r.tolist(), c.tolist()):
        if float(C_total[i, j]) <= float(cost_max):
            matches.append((i, j)); mt.add(i); md.add(j)
    return matches, [i for i in range(M) if i not in mt], [j for j in range(N) if j not in md]


# --------------------------------------------------------------------------
def encoder_forward(sd, x):
    """fp32 plain-torch restatement of the reference encoder eval graph.

    card.DSC.forward (card.py:48-57), SEBlock (:73-78), RMB.forward (:128-148,
    eval: alpha = 0.5, Shake2 -> 0.5/0.5), Model.forward GAP (encoderAndHead.py
    :26-31), ProjectionHead.forward (card.py:166-169)."""
    import torch
    import torch.nn.functional as F

    def dsc(pfx, x, reinforce):
        def branch(b):
            y = F.conv2d(x, sd[f"{pfx}.{b}.0.weight"])
            y = F.conv2d(y, sd[f"{pfx}.{b}.1.weight"], padding=2, groups=y.shape[1])
            return F.conv2d(y, sd[f"{pfx}.{b}.2.weight"])
        out = branch("depth") + branch("point")
        out = F.batch_norm(out, sd[f"{pfx}.bn.running_mean"], sd[f"{pfx}.bn.running_var"],
                           sd[f"{pfx}.bn.weight"], sd[f"{pfx}.bn.bias"], False, 0.0, 1e-5)
        return F.silu(out) if reinforce else F.hardswish(out)

    x_f = dsc("rmb.dsc_reinforce", x, True)
    x_n = dsc("rmb.dsc_normal", x, False)
    s = x_f.mean(dim=(2, 3))
    s = F.relu(F.linear(s, sd["rmb.se.excitation.0.weight"], sd["rmb.se.excitation.0.bias"]))
    s = F.hardsigmoid(F.linear(s, sd["rmb.se.excitation.2.weight"], sd["rmb.se.excitation.2.bias"]))
    x_f = x_f * s[:, :, None, None]
    x_cat = F.silu(F.conv2d(torch.cat([x_f, x_n], 1), sd["rmb.transition.0.weight"],
                            sd["rmb.transition.0.bias"]))
    fuse = 0.5 * x_f + (1 - 0.5) * x_n
    out = 0.5 * x_cat + 0.5 * fuse
    g = out.mean(dim=(2, 3))
    z = F.linear(g, sd["head.net.0.weight"])
    z = F.layer_norm(z, (z.shape[1],), sd["head.net.1.weight"], sd["head.net.1.bias"], 1e-5)
    z = F.linear(F.silu(z), sd["head.net.4.weight"], sd["head.net.4.bias"])
    return F.normalize(z, dim=1)


# --------------------------------------------------------------------------
class KalmanFilterRestated:
    """filterpy 1.4.5 ``KalmanFilter`` (predict / update, Joseph form) restated.

    dtype behaviour follows numpy promotion exactly as filterpy does it: the
    float32 matrices set by KalmanFilter.init_kf_from_bbox (KalmanFilter.py:
    57-99) stay float32 until update() forms ``I - KH`` with filterpy's float64
    identity."""

    def __init__(self, dim_x: int, dim_z: int, dim_u: int = 0):
        self.dim_x, self.dim_z = dim_x, dim_z
        self.x = np.zeros((dim_x, 1))
        self.P = np.eye(dim_x)
        self.Q = np.eye(dim_x)
        self.B = None
        self.F = np.eye(dim_x)
        self.H = np.zeros((dim_z, dim_x))
        self.R = np.eye(dim_z)
        self._alpha_sq = 1.0
        self.z = np.array([[None] * dim_z]).T
        self.K = np.zeros((dim_x, dim_z))
        self.y = np.zeros((dim_z, 1))
        self.S = np.zeros((dim_z, dim_z))
        self.SI = np.zeros((dim_z, dim_z))
        self._I = np.eye(dim_x)
        self.inv = np.linalg.inv

    def predict(self, u=None, B=None, F=None, Q=None):
        F = self.F if F is None else F
        Q = self.Q if Q is None else Q
        self.x = np.dot(F, self.x)
        self.P = self._alpha_sq * np.dot(np.dot(F, self.P), F.T) + Q
        self.x_prior = self.x.copy()
        self.P_prior = self.P.copy()

    def update(self, z, R=None, H=None):
        if z is None:
            return
        z = np.atleast_2d(np.asarray(z))
        if z.shape[1] == self.dim_z:
            z = z.T
        R = self.R if R is None else R
        H = self.H if H is None else H
        self.y = z - np.dot(H, self.x)
        PHT = np.dot(self.P, H.T)
        self.S = np.dot(H, PHT) + R
        self.SI = self.inv(self.S)
        self.K = np.dot(PHT, self.SI)
        self.x = self.x + np.dot(self.K, self.y)
        I_KH = self._I - np.dot(self.K, H)
        self.P = np.dot(np.dot(I_KH, self.P), I_KH.T) + np.dot(np.dot(self.K, R), self.K.T)
        self.z = z.copy()
        self.x_post = self.x.copy()
        self.P_post = self.P.copy()


def det_nms(pred: np.ndarray, conf_thres: float = 0.4, iou_thres: float = 0.45, *, max_det: int = 300,
            max_nms: int = 30000, agnostic: bool = False, cand_gate: int = 0, scale=None):
    """One image: pred [A, no] f32 -> (det [k, 6], xywh [k, 4] or None, cand_count)."""
    pred = np.ascontiguousarray(pred, dtype=np.float32)
    A, no = pred.shape
    det = np.zeros((max_det, 6), np.float32)
    xywh = np.zeros((max_det, 4), np.float32) if scale is not None else None
    sc = np.asarray(scale, np.float32) if scale is not None else None
    cand = ctypes.c_int(0)
    k = lib().ora_det_nms(_p(pred), A, no, float(conf_thres), float(iou_thres), max_det, max_nms,
                          int(agnostic), cand_gate, _p(sc) if sc is not None else None, _p(det),
                          _p(xywh) if xywh is not None else None, ctypes.byref(cand))
    return det[:k], (xywh[:k] if xywh is not None else None), cand.value


def train_rois(boxes: np.ndarray, Hf: int, Wf: int, img_hw, enforce_min_size: float = 1.0) -> np.ndarray:
    """PreProcess._preprocess_roi (trainingCard.py:36-69) box preparation, f32 numpy ops in the
    reference's order: [N, 4] image xyxy -> [N, 5] rois in feature pixels."""
    b = np.asarray(boxes, np.float32).reshape(-1, 4)
    img_h, img_w = img_hw
    f = np.float32
    with np.errstate(invalid="ignore"):
        x1 = np.minimum(b[:, 0], b[:, 2]); y1 = np.minimum(b[:, 1], b[:, 3])
        x2 = np.maximum(b[:, 0], b[:, 2]); y2 = np.maximum(b[:, 1], b[:, 3])
        sx, sy = f(Wf / float(img_w)), f(Hf / float(img_h))
        x1, x2, y1, y2 = x1 * sx, x2 * sx, y1 * sy, y2 * sy
        cl = lambda v, hi: np.where(np.isnan(v), v, np.minimum(np.maximum(v, f(0)), f(hi)))
        x1, x2, y1, y2 = cl(x1, Wf - 1), cl(x2, Wf - 1), cl(y1, Hf - 1), cl(y2, Hf - 1)
        if enforce_min_size > 0:
            ms = f(enforce_min_size)
            x2 = cl(np.maximum(x2, x1 + ms), Wf - 1)
            y2 = cl(np.maximum(y2, y1 + ms), Hf - 1)
    return np.stack([np.zeros_like(x1), x1, y1, x2, y2], 1).astype(np.float32)
