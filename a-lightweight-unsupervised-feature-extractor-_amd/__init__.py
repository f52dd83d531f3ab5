"""MI355X-native tracker hot path (ROI Align -> encoder -> cost -> assignment).

Drop-in for the per-frame path of ImChouOWO/A-lightweight-Unsupervised-
Feature-Extractor- (reference tracking.py:193-329, model/mainTracking.py):

  roi_align / roi_align_from_input_boxes   torchvision.ops.roi_align (HIP)
  Model                                    encoderAndHead.Model (PyTorch-ROCm)
  cal_cost / bbox_cost / conf_cost         costCard (HIP fused cost)
  hungarian_assign / linear_sum_assignment hung.py / scipy LSAP (HIP SAP)
  Tracking                                 mainTracking.Tracking
  MultiStreamTracker                       device-resident multi-stream tracker
  non_max_suppression / YoloPostprocess    YOLOv7 post-processing (HIP NMS)
  preprocess_roi                           PreProcess._preprocess_roi (training ROIs)

Import with importlib (the directory name is not an identifier):
    trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
"""
from ._lib import TrkError, lib, header_symbols
from .ops import (roi_align, roi_align_from_input_boxes, nchw_to_nhwc, build_cost, cost_combine, lsap_batched,
                  linear_sum_assignment, default_cost_params, CostParams)
from .hung import hungarian_assign
from .costcard import cal_cost, bbox_cost, conf_cost
from .encoder import Model
from .tracking import Tracking, MultiStreamTracker, TrackTable, tracker_conf, load_conf
from .detect import (letterbox_geometry, scale_coords_params, non_max_suppression, det_nms_batched,
                     YoloPostprocess, preprocess_roi, train_rois, SPPCSPCHook)

__all__ = ["TrkError", "lib", "header_symbols", "roi_align", "roi_align_from_input_boxes", "nchw_to_nhwc",
           "build_cost", "cost_combine", "lsap_batched", "linear_sum_assignment",
           "default_cost_params", "CostParams", "hungarian_assign", "cal_cost", "bbox_cost",
           "conf_cost", "Model", "Tracking", "MultiStreamTracker", "TrackTable", "tracker_conf",
           "load_conf", "letterbox_geometry", "scale_coords_params", "non_max_suppression",
           "det_nms_batched", "YoloPostprocess", "preprocess_roi", "train_rois", "SPPCSPCHook"]
