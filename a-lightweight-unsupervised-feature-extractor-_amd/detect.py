"""Detector-side boundary of the ROI path, on gfx950.

The YOLOv7 network itself is out of scope (weights absent, `.MISSING_LARGE_BLOBS`);
what the tracker consumes from it is (i) the SPPCSPC feature map, captured by a
forward hook (reference model/yolov7/yoloDetects2.py:27-34: ``SPPCSPCHook``
registers it on a loaded model; the ``feat`` tensor otherwise comes from the
caller) and (ii) the post-processed detections.  This module mirrors the
post-processing the reference runs on the head output:

  letterbox_geometry      utils/datasets.py:984-1014 (ratio and padding only;
                          the image resize itself is the caller's)
  non_max_suppression     utils/general.py:608-700 (defaults), trk_det_nms
  scale_coords_params     utils/general.py:320-333 (gain, pad of ratio_pad=None)
  YoloPostprocess         YoloDetects.run_with_tensor after the forward
                          (yoloDetects2.py:111-160): cand_gate, NMS,
                          scale_coords(...).round(), xyxy2xywh, result dicts
  preprocess_roi          PreProcess._preprocess_roi (trainingScr/trainingCard.py:24-79):
                          trk_train_rois + trk_roi_align_fwd (spatial_scale 1)

Every device step runs the hand-written kernels of csrc/detect.hip; there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import check, lib
from .ops import _need_gpu, _ptr, _stream, roi_align

__all__ = ["letterbox_geometry", "scale_coords_params", "non_max_suppression", "det_nms_batched",
           "YoloPostprocess", "preprocess_roi", "train_rois", "SPPCSPCHook"]

_P, _i32, _i64, _f32, _f64, _sz = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                   ctypes.c_double, ctypes.c_size_t)
_lib.register({
    "trk_det_workspace_bytes": ([_i64, _i64], _sz),
    "trk_det_nms": ([_P, _i64, _i64, _i64, _f32, _f64, _i32, _i32, _i32, _i32, _P, _P, _P, _P, _P, _P,
                     _sz, _P], _i32),
    "trk_train_rois": ([_P, _i64, _i64, _i64, _f64, _f64, _f32, _P, _P], _i32),
})

MAX_WH, MAX_DET, MAX_NMS = 4096, 300, 30000   # general.py:621-623


class SPPCSPCHook:
    """The backbone-feature capture of YoloDetects.__init__ (yoloDetects2.py:27-34): a
    forward hook on the model's first module whose class is named ``SPPCSPC`` keeps
    that module's output (the [B, C, Hf, Wf] map roi_align reads) in ``.feat`` after
    every forward.  ``remove()`` detaches it.  Raises ValueError when the model has no
    such module (the reference silently leaves ``backbone_feat`` None; a missing
    map would only surface later as a roi_align input error)."""

    def __init__(self, model: torch.nn.Module, class_name: str = "SPPCSPC"):
        self.feat: Optional[torch.Tensor] = None
        self._handle = None
        for m in model.modules():
            if m.__class__.__name__ == class_name:
                self._handle = m.register_forward_hook(self._hook)
                break
        if self._handle is None:
            raise ValueError(f"model has no {class_name} module to hook")

    def _hook(self, module, inputs, output):
        self.feat = output

    def remove(self):
        if self._handle is not None:
            self._handle.remove()
            self._handle = None


def letterbox_geometry(shape_hw: Tuple[int, int], new_shape=1280, auto: bool = False,
                       scaleFill: bool = False, scaleup: bool = True, stride: int = 32):
    """(ratio, (dw, dh), (H_in, W_in)) of utils/datasets.py letterbox (:984-1014) for an
    image of shape_hw; YoloDetects._preprocess calls it with auto=False (:99)."""
    h, w = shape_hw[:2]
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / h, new_shape[1] / w)
    if not scaleup:
        r = min(r, 1.0)
    ratio = r, r
    new_unpad = int(round(w * r)), int(round(h * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = dw % stride, dh % stride
    elif scaleFill:
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
        ratio = new_shape[1] / w, new_shape[0] / h
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return ratio, (dw, dh), (new_unpad[1] + top + bottom, new_unpad[0] + left + right)


def scale_coords_params(img1_shape, img0_shape):
    """gain and pad of scale_coords with ratio_pad=None (general.py:322-324), Python doubles."""
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    pad = (img1_shape[1] - img0_shape[1] * gain) / 2, (img1_shape[0] - img0_shape[0] * gain) / 2
    return gain, pad


def det_nms_batched(prediction: torch.Tensor, conf_thres: float = 0.25, iou_thres: float = 0.45, *,
                    agnostic: bool = False, max_det: int = MAX_DET, max_nms: int = MAX_NMS,
                    cand_gate: int = 0, img1_shape=None, img0_shape=None):
    """Device-side result of trk_det_nms for prediction [B, A, 5+nc] f32:
    (det [B, max_det, 6], det_count [B] i32, cand_count [B] i32, xywh [B, max_det, 4] or None).
    xywh (original-frame x, y, w, h after scale_coords(...).round()) needs both shapes."""
    _need_gpu(prediction, "non_max_suppression")
    if prediction.dim() != 3 or prediction.shape[2] < 6:
        raise ValueError(f"non_max_suppression: expected [B, A, 5 + nc] with nc >= 1, got {tuple(prediction.shape)}")
    if prediction.dtype != torch.float32:
        raise TypeError("non_max_suppression: f32 head output required (the reference CPU path)")
    pred = prediction.contiguous()
    B, A, no = pred.shape
    dev = pred.device
    det = torch.zeros((B, max_det, 6), device=dev, dtype=torch.float32)
    cnt = torch.zeros((B,), device=dev, dtype=torch.int32)
    cand = torch.zeros((B,), device=dev, dtype=torch.int32)
    xywh, hs = None, None
    if img1_shape is not None and img0_shape is not None:
        gain, pad = scale_coords_params(img1_shape, img0_shape)
        hs = (ctypes.c_float * 5)(gain, pad[0], pad[1], img0_shape[1], img0_shape[0])
        xywh = torch.zeros((B, max_det, 4), device=dev, dtype=torch.float32)
    nb = lib().trk_det_workspace_bytes(B, A)
    ws = torch.empty(max(nb, 16), device=dev, dtype=torch.uint8) if nb else None
    check(lib().trk_det_nms(_ptr(pred), B, A, no, float(conf_thres), float(iou_thres), max_det, max_nms,
                            int(bool(agnostic)), int(cand_gate), _ptr(det), _ptr(cnt), _ptr(cand), hs,
                            _ptr(xywh), _ptr(ws), nb, _stream(dev)), "non_max_suppression")
    return det, cnt, cand, xywh


def non_max_suppression(prediction: torch.Tensor, conf_thres: float = 0.25, iou_thres: float = 0.45,
                        classes=None, agnostic: bool = False, multi_label: bool = False, labels=()):
    """utils/general.py:608-700 on gfx950: list of [n, 6] (xyxy, conf, cls) per image."""
    if classes is not None or multi_label and prediction.shape[2] > 6 or len(labels):
        raise NotImplementedError("non_max_suppression: only the defaults YoloDetects uses "
                                  "(classes=None, multi_label=False, labels=())")
    det, cnt, _, _ = det_nms_batched(prediction, conf_thres, iou_thres, agnostic=agnostic)
    counts = cnt.cpu().tolist()
    return [det[b, :k] for b, k in enumerate(counts)]


class YoloPostprocess:
    """YoloDetects.run_with_tensor (yoloDetects2.py:111-160) from the network output on:
    ``run_with_tensor(pred_raw, frame_shape, feat)`` -> (result, pred_raw[, feat]) with the
    same result dicts (x, y, w, h, conf in original pixels; xyxy_in, input_hw, ratio, pad)."""

    def __init__(self, conf_thres: float = 0.4, iou_thres: float = 0.45, img_size: int = 1280,
                 stride: int = 32):
        self.conf_thres = conf_thres
        self.iou_thres = iou_thres
        self.stride = stride
        self.img_size = math.ceil(img_size / stride) * stride   # check_img_size

    def run_with_tensor(self, pred_raw: torch.Tensor, frame_shape, feat: Optional[torch.Tensor] = None,
                        return_img_tensor: bool = False, cand_gate: int = 5):
        ratio, pad, input_hw = letterbox_geometry(frame_shape[:2], self.img_size, auto=False)
        det, cnt, cand, xywh = det_nms_batched(pred_raw[:1], self.conf_thres, self.iou_thres,
                                               cand_gate=cand_gate, img1_shape=input_hw,
                                               img0_shape=frame_shape)
        k, nc = (int(v) for v in torch.stack([cnt[0], cand[0]]).cpu())   # the reference's host syncs
        result = []
        if nc < cand_gate:
            feat = None                           # cand_gate (:127-129): no NMS, no ROI features
        if k:
            d, q = det[0, :k].cpu(), xywh[0, :k].cpu()
            for j in range(k - 1, -1, -1):        # reversed(pred_nms)
                cx, cy, w, h = q[j].tolist()
                result.append({"x": cx, "y": cy, "w": w, "h": h, "conf": float(d[j, 4]),
                               "xyxy_in": d[j, :4].tolist(), "input_hw": input_hw,
                               "ratio": ratio, "pad": pad})
        if return_img_tensor:
            return result, pred_raw, feat
        return result, pred_raw


def train_rois(bboxes_xyxy: torch.Tensor, feat_hw: Tuple[int, int], img_hw: Tuple[float, float],
               enforce_min_size: float = 1.0) -> torch.Tensor:
    """[N, 4] image xyxy -> [N, 5] feature-pixel rois (trainingCard.py:36-69) via trk_train_rois."""
    _need_gpu(bboxes_xyxy, "train_rois")
    b = bboxes_xyxy.to(torch.float32).contiguous().reshape(-1, 4)
    N = b.shape[0]
    rois = torch.empty((N, 5), device=b.device, dtype=torch.float32)
    Hf, Wf = feat_hw
    check(lib().trk_train_rois(_ptr(b), N, Hf, Wf, float(img_hw[0]), float(img_hw[1]),
                               float(enforce_min_size), _ptr(rois), _stream(b.device)), "train_rois")
    return rois


def preprocess_roi(feat: torch.Tensor, bboxes_xyxy: torch.Tensor, img_hw: tuple, output_size=(10, 10),
                   sampling_ratio: int = 2, aligned: bool = True, enforce_min_size: float = 1.0,
                   **kw) -> torch.Tensor:
    """PreProcess._preprocess_roi (trainingCard.py:24-79): [1, C, Hf, Wf] feature map and
    image-pixel boxes -> [N, C, oh, ow] ROI features (roi_align with spatial_scale 1)."""
    if feat.dim() != 4 or feat.size(0) != 1:
        raise AssertionError(f"feat shape expected [1,C,H,W], got {feat.shape}")
    _, _, Hf, Wf = feat.shape
    rois = train_rois(bboxes_xyxy.to(feat.device), (Hf, Wf), img_hw, enforce_min_size)
    return roi_align(feat, rois, output_size, spatial_scale=1.0, sampling_ratio=sampling_ratio,
                     aligned=aligned, **kw)
