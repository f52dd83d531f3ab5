"""Detector-side boundary: YOLOv7 post-processing
(non_max_suppression / scale_coords / run_with_tensor, reference
model/yolov7/utils/general.py:255-341,608-700, yoloDetects2.py:111-160) and the
training-side ROI boxes (trainingCard.py:24-79).

Parity: torchvision (nms, roi_align) and cv2 are absent from the reference tree
and this image, so neither path can be run from the reference here: the oracle
restatements (oracle/trk_oracle.c ora_det_nms, oracle.py train_rois) are pinned
by the known-answer tests below, and the HIP kernels must equal the oracle
bit for bit (tolerance 0: every output is a copy, a comparison or f32 arithmetic
done in the reference's order)."""
import numpy as np
import pytest


# ----------------------------------------------------------------- inputs --
def synth_pred(seed, A=6000, nc=3, nobj=40, per=24, quant=None):
    """Head output [A, 5 + nc]: background anchors with low objectness plus
    clusters of jittered boxes around nobj objects (what NMS has to thin out)."""
    rng = np.random.default_rng(seed)
    p = np.zeros((A, 5 + nc), np.float32)
    p[:, 0] = rng.uniform(0, 1280, A); p[:, 1] = rng.uniform(280, 1000, A)
    p[:, 2] = rng.uniform(8, 200, A); p[:, 3] = rng.uniform(8, 200, A)
    p[:, 4] = rng.uniform(0, 0.5, A) ** 2
    p[:, 5:] = rng.uniform(0, 1, (A, nc))
    idx = rng.permutation(A)[: nobj * per].reshape(nobj, per)
    for o in range(nobj):
        cx, cy = rng.uniform(40, 1240), rng.uniform(300, 980)
        w, h = rng.uniform(20, 300), rng.uniform(20, 300)
        cls = rng.integers(nc)
        for a in idx[o]:
            p[a, :4] = [cx + rng.normal(0, w * 0.08), cy + rng.normal(0, h * 0.08),
                        w * rng.uniform(0.8, 1.2), h * rng.uniform(0.8, 1.2)]
            p[a, 4] = rng.uniform(0.35, 1.0)
            p[a, 5:] = rng.uniform(0, 0.3, nc)
            p[a, 5 + cls] = rng.uniform(0.5, 1.0)
    if quant:  # many exactly tied scores: the stable-sort tie order matters
        p[:, 4:] = np.round(p[:, 4:] * quant) / quant
    return p


SCALE_1080P = (1280 / 1920, 0.0, 280.0, 1920.0, 1080.0)  # gain, pad_w, pad_h, img0_w, img0_h


# --------------------------------------------------------- oracle KATs (CPU) --
def _row(cx, cy, w, h, obj, cls):
    return [cx, cy, w, h, obj] + list(cls)


def test_oracle_nms_suppresses_same_class_only(oracle):
    p = np.array([_row(100, 100, 50, 50, 0.9, [0.9, 0.1]),
                  _row(105, 100, 50, 50, 0.8, [0.9, 0.1]),     # IoU 0.82 with row 0, same class
                  _row(105, 100, 50, 50, 0.8, [0.1, 0.9]),     # same box, other class: survives
                  _row(400, 400, 30, 30, 0.95, [0.2, 0.95])], np.float32)
    det, _, cand = oracle.det_nms(p, 0.4, 0.45)
    assert cand == 4
    np.testing.assert_array_equal(det[:, 5], [1, 0, 1])
    np.testing.assert_array_equal(det[:, 4], np.float32([0.95 * np.float32(0.95), 0.9 * np.float32(0.9),
                                                         np.float32(0.8) * np.float32(0.9)]))
    # agnostic: the other-class duplicate is suppressed too
    det, _, _ = oracle.det_nms(p, 0.4, 0.45, agnostic=True)
    assert len(det) == 2


def test_oracle_nms_threshold_is_strict_and_double(oracle):
    # inter 50*50, union 2*2500 - inter ... choose boxes whose f32 IoU is exactly 0.5
    p = np.array([_row(25, 25, 50, 50, 0.9, [1.0]), _row(25, 50, 50, 100, 0.8, [1.0])], np.float32)
    # IoU = 2500 / (2500 + 5000 - 2500) = 0.5 exactly
    assert len(oracle.det_nms(p, 0.4, 0.5)[0]) == 2          # 0.5 > 0.5 is false: kept
    assert len(oracle.det_nms(p, 0.4, 0.4999999)[0]) == 1
    # nc == 1: conf is the objectness itself (x[:, 5:] = x[:, 4:5])
    np.testing.assert_array_equal(oracle.det_nms(p, 0.4, 0.5)[0][:, 4], np.float32([0.9, 0.8]))


def test_oracle_nms_ties_keep_anchor_order_and_filters(oracle):
    p = np.array([_row(100, 100, 40, 40, 0.8, [1.0]),
                  _row(102, 100, 40, 40, 0.8, [1.0]),           # exact tie, later anchor: suppressed
                  _row(600, 600, 40, 40, 0.8, [1.0]),
                  _row(900, 600, 40, 40, 0.3, [1.0]),           # below conf_thres
                  _row(700, 700, 40, 40, np.nan, [1.0]),        # NaN objectness: not a candidate
                  _row(800, 700, 40, 40, 0.9, [np.nan])], np.float32)  # nc == 1: class ignored
    det, _, cand = oracle.det_nms(p, 0.4, 0.45)
    assert cand == 4
    np.testing.assert_array_equal(det[:, 0], np.float32([780, 80, 580]))
    # cand_gate: fewer candidates than the gate -> nothing
    assert len(oracle.det_nms(p, 0.4, 0.45, cand_gate=5)[0]) == 0
    # max_det truncation keeps the best-scored boxes
    det, _, _ = oracle.det_nms(p, 0.4, 0.45, max_det=2)
    np.testing.assert_array_equal(det[:, 0], np.float32([780, 80]))
    # nc > 1: a NaN class score makes the row's max NaN, which fails the conf gate
    q = np.array([_row(100, 100, 40, 40, 0.9, [0.9, np.nan]), _row(500, 100, 40, 40, 0.9, [0.9, 0.1])],
                 np.float32)
    np.testing.assert_array_equal(oracle.det_nms(q, 0.4, 0.45)[0][:, 0], np.float32([480]))


def test_oracle_scale_coords_round_half_even(oracle):
    # gain 0.5, pad (0, 140): x = (v - pad) / gain, clipped to the frame, rounded half to even
    p = np.array([_row(100.25, 300.5, 50.5, 40.0, 0.9, [1.0])], np.float32)
    det, q, _ = oracle.det_nms(p, 0.4, 0.45, scale=(0.5, 0.0, 140.0, 1920.0, 1080.0))
    x1, y1, x2, y2 = det[0, :4]
    c = [np.float32(np.rint((x1 - 0) / np.float32(0.5))), np.float32(np.rint((y1 - 140) / np.float32(0.5))),
         np.float32(np.rint((x2 - 0) / np.float32(0.5))), np.float32(np.rint((y2 - 140) / np.float32(0.5)))]
    np.testing.assert_array_equal(q[0], np.float32([(c[0] + c[2]) / 2, (c[1] + c[3]) / 2, c[2] - c[0], c[3] - c[1]]))
    assert np.rint(np.float32(150.5)) == 150  # half to even, as torch.round


def test_oracle_train_rois(oracle):
    b = np.array([[300, 200, 100, 50],        # reversed corners -> sorted
                  [-20, 10, 2000, 20],        # clamped to [0, W-1]
                  [500, 500, 500.5, 500.5]],  # enforced minimum size
                 np.float32)
    r = oracle.train_rois(b, 40, 40, (1280, 1280), 1.0)
    s = np.float32(40 / 1280)
    np.testing.assert_array_equal(r[0], np.float32([0, 100 * s, 50 * s, 300 * s, 200 * s]))
    np.testing.assert_array_equal(r[1, 1:], np.float32([0, 10 * s, 39, 10 * s + 1]))  # 20s < 10s + 1
    np.testing.assert_array_equal(r[2, 3:], np.float32([500 * s + 1, 500 * s + 1]))


def test_letterbox_and_scale_params(trk):
    ratio, pad, hw = trk.letterbox_geometry((1080, 1920), 1280)
    assert ratio == (1280 / 1920, 1280 / 1920) and pad == (0.0, 280.0) and hw == (1280, 1280)
    ratio, pad, hw = trk.letterbox_geometry((720, 1280), 1280)
    assert ratio == (1.0, 1.0) and pad == (0.0, 280.0) and hw == (1280, 1280)
    gain, pad = trk.scale_coords_params((1280, 1280), (1080, 1920))
    assert gain == 1280 / 1920 and pad == (0.0, 280.0)


def test_sppcspc_hook_captures_backbone_output(trk):
    """SPPCSPCHook = YoloDetects.__init__'s hook (yoloDetects2.py:27-34): the first
    module whose class is named SPPCSPC; its output is kept after each forward."""
    import torch
    from importlib import import_module
    det = import_module(trk.__name__ + ".detect")

    class SPPCSPC(torch.nn.Module):
        def forward(self, x):
            return x * 2

    class Head(torch.nn.Module):
        def forward(self, x):
            return x.sum(1)

    net = torch.nn.Sequential(torch.nn.Identity(), SPPCSPC(), SPPCSPC(), Head())
    h = det.SPPCSPCHook(net)
    x = torch.randn(2, 3, 5, 5)
    y = net(x)
    assert torch.equal(h.feat, x * 2) and y.shape == (2, 5, 5)  # the first SPPCSPC's output
    h.remove()
    h.feat = None
    net(x)
    assert h.feat is None
    with pytest.raises(ValueError, match="no SPPCSPC"):
        det.SPPCSPCHook(torch.nn.Sequential(torch.nn.Identity()))


def test_det_wrappers_reject_host_tensors(trk):
    import torch
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        trk.non_max_suppression(torch.zeros(1, 10, 7))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        trk.train_rois(torch.zeros(2, 4), (40, 40), (1280, 1280))


# -------------------------------------------------------- GPU vs oracle --
@pytest.mark.gpu
@pytest.mark.parametrize("seed,A,nc,nobj,quant,conf", [
    (0, 6000, 3, 40, None, 0.4),
    (1, 25200, 80, 120, None, 0.25),
    (2, 6000, 1, 60, 64, 0.4),            # nc == 1 and exact score ties
    (3, 100800, 3, 400, 16, 0.3),         # > 8192 survivors: sort in the workspace
])
def test_det_nms_matches_oracle(trk, oracle, gpu, seed, A, nc, nobj, quant, conf):
    import torch
    p = synth_pred(seed, A, nc, nobj, quant=quant)
    det, cnt, cand, xywh = trk.det_nms_batched(torch.from_numpy(p)[None].to(gpu), conf, 0.45,
                                               img1_shape=(1280, 1280), img0_shape=(1080, 1920))
    ed, eq, ec = oracle.det_nms(p, conf, 0.45, scale=SCALE_1080P)
    k = int(cnt[0])
    assert int(cand[0]) == ec and k == len(ed) and k > 0
    np.testing.assert_array_equal(det[0, :k].cpu().numpy(), ed)
    np.testing.assert_array_equal(xywh[0, :k].cpu().numpy(), eq)


@pytest.mark.gpu
def test_det_nms_batched_images_limits_and_gate(trk, oracle, gpu):
    import torch
    ps = [synth_pred(10 + b, 8000, 4, 50) for b in range(3)]
    ps[2][:, 4] = 0.01                                          # an image with no candidates
    P = torch.from_numpy(np.stack(ps)).to(gpu)
    for kw in ({}, {"max_det": 7}, {"max_nms": 50}, {"agnostic": True}, {"cand_gate": 10 ** 6}):
        det, cnt, cand, _ = trk.det_nms_batched(P, 0.4, 0.45, **kw)
        for b in range(3):
            ed, _, ec = oracle.det_nms(ps[b], 0.4, 0.45, **kw)
            k = int(cnt[b])
            assert int(cand[b]) == ec and k == len(ed), (kw, b)
            np.testing.assert_array_equal(det[b, :k].cpu().numpy(), ed)
    out = trk.non_max_suppression(P, 0.4, 0.45)
    assert [len(o) for o in out] == [len(oracle.det_nms(q, 0.4, 0.45)[0]) for q in ps]
    # empty anchor set
    det, cnt, cand, _ = trk.det_nms_batched(torch.zeros((2, 0, 8), device=gpu), 0.4, 0.45)
    assert cnt.tolist() == [0, 0]


@pytest.mark.gpu
def test_yolo_postprocess_result_dicts(trk, oracle, gpu):
    import torch
    p = synth_pred(5, 12000, 2, 30)
    feat = torch.zeros(1, 512, 40, 40, device=gpu)
    post = trk.YoloPostprocess(conf_thres=0.4, iou_thres=0.45, img_size=1280)
    res, raw, f = post.run_with_tensor(torch.from_numpy(p)[None].to(gpu), (1080, 1920, 3), feat,
                                       return_img_tensor=True)
    ed, eq, _ = oracle.det_nms(p, 0.4, 0.45, scale=SCALE_1080P)
    assert f is feat and len(res) == len(ed) > 0
    for i, r in enumerate(res):                        # reversed(pred_nms)
        j = len(ed) - 1 - i
        assert [r["x"], r["y"], r["w"], r["h"]] == eq[j].tolist()
        assert r["conf"] == float(ed[j, 4]) and r["xyxy_in"] == ed[j, :4].tolist()
        assert r["input_hw"] == (1280, 1280) and r["pad"] == (0.0, 280.0)
    # below cand_gate: no detections and no feature map
    q = p.copy(); q[:, 4] = 0.0; q[:3, 4] = 0.9
    res, _, f = post.run_with_tensor(torch.from_numpy(q)[None].to(gpu), (1080, 1920, 3), feat,
                                     return_img_tensor=True)
    assert res == [] and f is None


@pytest.mark.gpu
def test_preprocess_roi_matches_oracle(trk, oracle, gpu):
    import torch
    rng = np.random.default_rng(3)
    feat = rng.standard_normal((1, 64, 40, 40)).astype(np.float32)
    b = np.stack([rng.uniform(-50, 1330, 40), rng.uniform(200, 1100, 40),
                  rng.uniform(-50, 1330, 40), rng.uniform(200, 1100, 40)], 1).astype(np.float32)
    b[:5, 2] = b[:5, 0] + 0.2                                    # sub-pixel boxes: min size
    got = trk.preprocess_roi(torch.from_numpy(feat).to(gpu), torch.from_numpy(b).to(gpu), (1280, 1280))
    rois = oracle.train_rois(b, 40, 40, (1280, 1280), 1.0)
    np.testing.assert_array_equal(trk.train_rois(torch.from_numpy(b).to(gpu), (40, 40), (1280, 1280)).cpu().numpy(),
                                  rois)
    exp = oracle.roi_align(feat, rois, (10, 10), 1.0, 2, True)
    np.testing.assert_array_equal(got.cpu().numpy(), exp)
