"""costCard API mirror -- drop-in for reference model/utils/costTool/costCard.py.

bbox_cost / conf_cost / cal_cost keep the reference signatures and return
dicts of [M, N] device tensors; the arithmetic runs in the fused gfx950
kernel (trk_cost_combine), with the same float32 rounding as the reference
CPU path.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import torch

from .ops import _device, cost_combine, default_cost_params


def _tensor(x, dev, shape) -> torch.Tensor:
    return torch.as_tensor(x, dtype=torch.float32).reshape(shape).to(dev).contiguous()


def _combine(C_app, boxes_prev, boxes_cur, conf_prev, conf_cur, *, w_app, w_bbox, w_conf,
             alpha, beta):
    dev = C_app.device if isinstance(C_app, torch.Tensor) and C_app.is_cuda else _device()
    M, N = len(boxes_prev), len(boxes_cur)
    if C_app is None:
        C_app = torch.zeros((M, N), device=dev)
    C_app = C_app.to(dev, torch.float32)
    p = default_cost_params(dict(w_app=w_app, w_bbox=w_bbox, w_conf=w_conf, alpha=alpha, beta=beta),
                            gate=False)
    cp = conf_prev if conf_prev is not None else [1.0] * M
    cc = conf_cur if conf_cur is not None else [1.0] * N
    return cost_combine(C_app, _tensor(boxes_prev, dev, (M, 4)), _tensor(cp, dev, (M,)),
                        _tensor(boxes_cur, dev, (N, 4)), _tensor(cc, dev, (N,)), p), dev


def bbox_cost(boxes_prev: List[List[float]], boxes_cur: List[List[float]], input_hw: Tuple[int, int],
              alpha: float = 1.0, beta: float = 1.0) -> Dict[str, torch.Tensor]:
    """costCard.py:109-174 (input_hw is accepted for API parity; the reference
    normalises by the previous box's diagonal, not the image's)."""
    M, N = len(boxes_prev), len(boxes_cur)
    if M == 0 or N == 0:
        z = torch.zeros((M, N), device=_device())
        return {"C_center": z, "C_scale": z, "C_bbox": z}
    out, _ = _combine(None, boxes_prev, boxes_cur, None, None, w_app=0.0, w_bbox=1.0, w_conf=0.0,
                      alpha=alpha, beta=beta)
    C_bbox = alpha * out["C_center"] + beta * out["C_scale"]
    return {"C_center": out["C_center"], "C_scale": out["C_scale"], "C_bbox": C_bbox}


def conf_cost(conf_prev: List[float], conf_cur: List[float], eps: float = 1e-6) -> torch.Tensor:
    """costCard.py:178-203 (eps fixed at the reference's 1e-6)."""
    M, N = len(conf_prev), len(conf_cur)
    if M == 0 or N == 0:
        return torch.zeros((M, N), device=_device())
    out, _ = _combine(None, [[0.0, 0.0, 1.0, 1.0]] * M, [[0.0, 0.0, 1.0, 1.0]] * N, conf_prev, conf_cur,
                      w_app=0.0, w_bbox=0.0, w_conf=1.0, alpha=1.0, beta=1.0)
    return out["C_conf"]


def cal_cost(*, C_app: torch.Tensor, boxes_prev: List[List[float]], boxes_cur: List[List[float]],
             input_hw: Tuple[int, int], conf_prev: List[float], conf_cur: List[float],
             w_app: float = 1.0, w_bbox: float = 0.3, w_conf: float = 0.2, alpha: float = 1.0,
             beta: float = 0.5, assign: Optional[List[int]] = None,
             unmatch_cost: float = 10.0) -> Dict[str, Any]:
    """costCard.cal_cost (costCard.py:206-300)."""
    M, N = C_app.shape
    if M == 0 or N == 0:
        dev = C_app.device
        z = torch.zeros((M, N), device=dev)
        out = {"C_total": z + 0, "C_app": C_app, "C_bbox": z, "C_center": z, "C_scale": z, "C_conf": z}
    else:
        res, dev = _combine(C_app, boxes_prev, boxes_cur, conf_prev, conf_cur, w_app=w_app,
                            w_bbox=w_bbox, w_conf=w_conf, alpha=alpha, beta=beta)
        out = {"C_total": res["C_total"], "C_app": C_app,
               "C_bbox": alpha * res["C_center"] + beta * res["C_scale"],
               "C_center": res["C_center"], "C_scale": res["C_scale"], "C_conf": res["C_conf"]}
    if assign is not None:  # PSO scalar fitness (costCard.py:282-298)
        C_np = out["C_total"].detach().cpu().numpy()
        cost, used = 0.0, set()
        for i, j in enumerate(assign):
            if j == -1:
                cost += unmatch_cost
            elif j in used:
                cost += 1e6
            else:
                cost += C_np[i, j]
                used.add(j)
        out["total_cost"] = float(cost)
    return out
