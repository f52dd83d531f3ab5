"""CPU baseline, "reference-literal" mode: the association
cost computed the way the reference's Python does it, loop for loop.  TEST /
BASELINE INFRASTRUCTURE ONLY -- used by bench.py's cpu_baseline leg to time
the reference's CPU path; never imported by the product package.

  build_c_app_topk_literal   Tracking.build_C_app_topk (reference
                             model/mainTracking.py:141-211): a Python loop over
                             tracks, each stacking and renormalising its bank,
                             one [T,128] x [128,N] product, torch.topk + mean
  kalman_gating_literal      Tracking.apply_kalman_gating (:306-338) with
                             KalmanFilter.gating_distance_maha
                             (model/utils/costTool/KalmanFilter.py:105-116): a
                             Python loop over every (track, detection) pair, each
                             with its own 4x4 np.linalg.inv
The bbox / conf terms of costCard.cal_cost are torch-vectorised in the reference
(model/utils/costTool/costCard.py:109-268), so both modes share them.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch


def build_c_app_topk_literal(banks: Sequence[Sequence[np.ndarray]], det_embs: Sequence[np.ndarray],
                             topk: int = 5) -> np.ndarray:
    N = len(det_embs)
    det = np.stack([np.asarray(e, dtype=np.float32).reshape(-1) for e in det_embs], axis=0)
    det = det / (np.linalg.norm(det, axis=1, keepdims=True) + 1e-12)
    F_det = torch.from_numpy(det)
    rows: List[torch.Tensor] = []
    for bank_list in banks:
        if bank_list is None or len(bank_list) == 0:
            rows.append(torch.ones((N,)))
            continue
        bank = np.stack([np.asarray(f, dtype=np.float32).reshape(-1) for f in bank_list], axis=0)
        bank = bank / (np.linalg.norm(bank, axis=1, keepdims=True) + 1e-12)
        sim_TN = torch.from_numpy(bank) @ F_det.T
        k = min(int(topk), sim_TN.shape[0])
        topv, _ = torch.topk(sim_TN, k=k, dim=0)
        rows.append(1.0 - topv.mean(dim=0))
    return torch.stack(rows, dim=0).numpy()


def _bbox_xyxy_to_z(b) -> np.ndarray:
    """KalmanFilter.bbox_xyxy_to_z (KalmanFilter.py:5-16)"""
    x1, y1, x2, y2 = [float(v) for v in b]
    w = max(1.0, x2 - x1)
    h = max(1.0, y2 - y1)
    return np.array([x1 + 0.5 * w, y1 + 0.5 * h, w / h, h], dtype=np.float32).reshape(4, 1)


_H = np.concatenate([np.eye(4), np.zeros((4, 4))], 1)
_R = np.eye(4)


def kalman_gating_literal(C: np.ndarray, kf_x: Sequence[np.ndarray], kf_P: Sequence[np.ndarray],
                          det_boxes: Sequence[Sequence[float]], maha_thr: float = 9.49,
                          INF: float = 1e9) -> np.ndarray:
    M, N = C.shape
    for i in range(M):
        x = np.asarray(kf_x[i], np.float64).reshape(8, 1)
        P = np.asarray(kf_P[i], np.float64).reshape(8, 8)
        for j in range(N):
            z = _bbox_xyxy_to_z(det_boxes[j])
            y = z - (_H @ x)
            S = _H @ P @ _H.T + _R
            Sinv = np.linalg.inv(S + 1e-9 * np.eye(4, dtype=np.float32))
            d2 = float((y.T @ Sinv @ y)[0, 0])
            if d2 > float(maha_thr):
                C[i, j] = float(INF)
    return C
