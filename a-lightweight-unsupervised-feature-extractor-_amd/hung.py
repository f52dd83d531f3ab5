"""hungarian_assign -- drop-in for reference model/utils/costTool/hung.py:5-45.

The assignment is solved by the gfx950 LSAP kernel (trk_lsap), which is
index-for-index identical to scipy.optimize.linear_sum_assignment; the
``C <= cost_max`` gate of hung.py:35-40 is applied inside the kernel.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from .ops import _device, lsap_batched, lsap_check_status


def hungarian_assign(C_total, cost_max: float = 1e9
                     ) -> Tuple[List[Tuple[int, int]], List[int], List[int]]:
    """Returns (matches [(i, j)] in ascending row order, unmatched_tracks,
    unmatched_dets), exactly as the reference does.  C_total may be a numpy
    array or a (device) torch tensor [M, N]."""
    if isinstance(C_total, torch.Tensor):
        t = C_total
    else:
        a = np.asarray(C_total)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if t.dim() != 2:
        raise ValueError("expected a matrix (2-D array), got a %r array" % (tuple(t.shape),))
    M, N = t.shape
    if M == 0 and N == 0:
        return [], [], []
    if M == 0:
        return [], [], list(range(N))
    if N == 0:
        return [], list(range(M)), []
    if not t.is_cuda:
        t = t.to(_device())
    res = lsap_batched(t.reshape(1, M, N), [M], [N], cost_max=float(cost_max))
    lsap_check_status(int(res["status"][0].item()), "hungarian_assign")
    assign = res["assign"][0, :M].cpu().numpy()
    matches = [(i, int(assign[i])) for i in range(M) if assign[i] >= 0]
    matched_dets = {j for _, j in matches}
    unmatched_tracks = [i for i in range(M) if assign[i] < 0]
    unmatched_dets = [j for j in range(N) if j not in matched_dets]
    return matches, unmatched_tracks, unmatched_dets
