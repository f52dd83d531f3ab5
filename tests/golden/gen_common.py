"""Deterministic synthetic inputs shared by the golden-fixture generator
(make_golden.py, run in the survey container against /root/reference) and the
tests (run here and on the GPU box, where /root/reference does not exist).

Everything is numpy-seeded so the same arrays are produced on both machines
(same image, same numpy).  Test infrastructure only.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

# encoder parameter table: (key, shape) in reference state_dict order
# (encoderAndHead.Model(in_channels=512, out_channels=512, proj_dim=128)).
C_IN, C_HID, PROJ = 512, 256, 128


def encoder_param_shapes(c=C_IN, proj=PROJ):
    h = c // 2
    shapes = []
    for dsc in ("dsc_reinforce", "dsc_normal"):
        for br in ("depth", "point"):
            shapes.append((f"rmb.{dsc}.{br}.0.weight", (h, c, 1, 1)))
            shapes.append((f"rmb.{dsc}.{br}.1.weight", (h, 1, 5, 5)))
            shapes.append((f"rmb.{dsc}.{br}.2.weight", (c, h, 1, 1)))
        for k in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            shapes.append((f"rmb.{dsc}.bn.{k}", () if k == "num_batches_tracked" else (c,)))
    shapes += [("rmb.se.excitation.0.weight", (c // 4, c)), ("rmb.se.excitation.0.bias", (c // 4,)),
               ("rmb.se.excitation.2.weight", (c, c // 4)), ("rmb.se.excitation.2.bias", (c,)),
               ("rmb.transition.0.weight", (c, 2 * c, 1, 1)), ("rmb.transition.0.bias", (c,)),
               ("head.logit_scale", ()), ("head.logit_bias", ()),
               ("head.net.0.weight", (c, c)), ("head.net.1.weight", (c,)), ("head.net.1.bias", (c,)),
               ("head.net.4.weight", (proj, c)), ("head.net.4.bias", (proj,))]
    return shapes


def seeded_state_dict_np(seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded random encoder weights with non-trivial BN statistics."""
    rng = np.random.default_rng(seed)
    sd = {}
    for key, shape in encoder_param_shapes():
        if key.endswith("num_batches_tracked"):
            sd[key] = np.array(0, dtype=np.int64)
        elif key.endswith("running_mean"):
            sd[key] = rng.uniform(-0.1, 0.1, shape).astype(np.float32)
        elif key.endswith("running_var"):
            sd[key] = rng.uniform(0.5, 1.5, shape).astype(np.float32)
        elif key.endswith("bn.weight") or key == "head.net.1.weight":
            sd[key] = rng.uniform(0.5, 1.5, shape).astype(np.float32)
        elif key.endswith("bias") and key != "head.logit_bias":
            sd[key] = rng.uniform(-0.1, 0.1, shape).astype(np.float32)
        elif key == "head.logit_scale":
            sd[key] = np.array(math.log(10.0), dtype=np.float32)
        elif key == "head.logit_bias":
            sd[key] = np.array(0.0, dtype=np.float32)
        else:
            fan_in = int(np.prod(shape[1:]))
            sd[key] = (rng.standard_normal(shape) / math.sqrt(fan_in)).astype(np.float32)
    return sd


def silu_np(x):
    return x / (1.0 + np.exp(-x))


def encoder_input(seed: int, n: int, s: int, c: int = C_IN) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return silu_np(rng.standard_normal((n, c, s, s)).astype(np.float32)).astype(np.float32)


# --------------------------------------------------------------------------
# synthetic multi-object scene (SURVEY 8(d) "Synthetic inputs")
# --------------------------------------------------------------------------
def make_scene(seed: int, n_obj: int, n_frames: int, *, emb_noise=0.05, img=1280,
               pad_h=280, gaps=(), births=(), low_conf=(), D=128):
    """Returns a list of frames; each frame = dict(embs [N,D] f32, bboxes [N,4]
    (python floats), confs [N], frame_id).  Objects move at constant velocity.

    gaps:   list of (obj, first_frame, n_missing)   -- object not detected
    births: list of (obj, frame)                    -- object appears at frame
    low_conf: list of (obj, frame)                  -- conf forced to 0.45
    """
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n_obj, D)).astype(np.float32)
    base /= np.linalg.norm(base, axis=1, keepdims=True)
    w = rng.uniform(32, 320, n_obj)
    h = rng.uniform(32, 320, n_obj)
    x1 = rng.uniform(-8, img - w + 8)
    y1 = rng.uniform(pad_h - 8, img - pad_h - h + 8)
    vx = rng.uniform(-4, 4, n_obj)
    vy = rng.uniform(-4, 4, n_obj)
    conf = rng.uniform(0.55, 0.99, n_obj)
    birth = {o: f for o, f in births}
    missing = set()
    for o, f0, n in gaps:
        for f in range(f0, f0 + n):
            missing.add((o, f))
    lowc = set(low_conf)
    frames = []
    for f in range(n_frames):
        objs = [o for o in range(n_obj) if birth.get(o, 0) <= f and (o, f) not in missing]
        order = rng.permutation(len(objs))
        objs = [objs[k] for k in order]
        embs, boxes, confs = [], [], []
        for o in objs:
            e = base[o] + emb_noise * rng.standard_normal(D).astype(np.float32)
            e = (e / np.linalg.norm(e)).astype(np.float32)
            bx1 = x1[o] + vx[o] * f + rng.normal(0, 0.3)
            by1 = y1[o] + vy[o] * f + rng.normal(0, 0.3)
            ww = w[o] * (1 + 0.002 * rng.standard_normal())
            hh = h[o] * (1 + 0.002 * rng.standard_normal())
            embs.append(e)
            boxes.append([float(bx1), float(by1), float(bx1 + ww), float(by1 + hh)])
            c = 0.45 if (o, f) in lowc else float(np.clip(conf[o] + rng.normal(0, 0.01), 0.01, 0.999))
            confs.append(c)
        frames.append(dict(embs=np.asarray(embs, np.float32).reshape(-1, D), bboxes=boxes,
                           confs=confs, obj=objs, frame_id=f))
    return frames


SCENES = {
    # name: (seed, n_obj, n_frames, kwargs)
    "s16": (11, 16, 40, dict(gaps=[(3, 10, 3), (7, 20, 2)], births=[(12, 5), (13, 33)],
                             low_conf=[(5, 2), (14, 0), (9, 30)])),
    "s64": (12, 64, 8, dict(gaps=[(1, 3, 2)], births=[(60, 4)], low_conf=[(2, 5)])),
    "reid": (13, 10, 62, dict(gaps=[(2, 4, 53), (6, 5, 55)], births=[(9, 20)])),
    # the metric's size (BASELINE c3: N = 256 per frame): banks fill to T = 30, six tracks
    # lost for 54 frames come back through the ReID-only stage (miss_count > 50), short
    # gaps re-activate in stage 1, births at frames 2 and 60 (none while the six are lost:
    # with cost_max 50 and a loosened gate a lost track takes a newborn detection in stage
    # 1, which the reference does too), low-confidence detections (no track / no update)
    "n256": (14, 256, 64, dict(
        gaps=[(o, 3, 54) for o in range(6)] + [(o, 10, 3) for o in range(10, 22)] +
             [(o, 30, 6) for o in range(40, 46)] + [(o, 45, 1) for o in range(60, 90)],
        births=[(o, 2) for o in range(245, 256)] + [(o, 60) for o in range(240, 245)],
        low_conf=[(100, 0), (101, 5), (102, 20), (103, 40), (241, 60)])),
}

# scenes whose fixture stores only the reference's outputs (plus a digest of the
# inputs): the inputs are regenerated here from the seed (8 MB of embeddings)
OUTPUT_ONLY = {"n256"}


def scene_digest(frames) -> str:
    """sha256 over every frame's embs / boxes / confs, as fixtures record it"""
    import hashlib
    h = hashlib.sha256()
    for fr in frames:
        h.update(np.ascontiguousarray(fr["embs"], np.float32).tobytes())
        h.update(np.asarray(fr["bboxes"], np.float64).reshape(-1, 4).tobytes())
        h.update(np.asarray(fr["confs"], np.float64).tobytes())
    return h.hexdigest()


def scene(name: str):
    seed, n_obj, n_frames, kw = SCENES[name]
    return make_scene(seed, n_obj, n_frames, **kw)


# --------------------------------------------------------------------------
# LSAP stress matrices
# --------------------------------------------------------------------------
def lsap_cases(seed: int = 5) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    cases = []
    shapes = [(1, 1), (1, 5), (5, 1), (2, 2), (3, 7), (7, 3), (8, 8), (16, 16), (13, 29),
              (29, 13), (32, 32), (64, 64), (40, 64), (64, 40), (63, 65)]
    for (r, c) in shapes:
        cases.append(rng.random((r, c)).astype(np.float32))                    # uniform
        cases.append(rng.integers(0, 3, (r, c)).astype(np.float32))            # ties 0..2
        cases.append(np.ones((r, c), np.float32))                              # all equal
        g = rng.random((r, c)).astype(np.float32)
        g[rng.random((r, c)) < 0.7] = 1e9                                      # gated
        cases.append(g)
        cases.append((rng.integers(0, 5, (r, c)) * 0.25).astype(np.float32))   # quarter ties
        t = np.full((r, c), 1e9, np.float32)                                   # tracking-like
        k = min(r, c)
        perm = rng.permutation(c)[:k]
        t[np.arange(k), perm] = rng.uniform(0.1, 0.5, k)
        near = rng.random((r, c)) < 0.1
        t[near] = rng.uniform(0.6, 2.0, near.sum())
        cases.append(t)
    for _ in range(60):
        r, c = int(rng.integers(1, 48)), int(rng.integers(1, 48))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            cases.append(rng.integers(0, 2, (r, c)).astype(np.float32))
        elif kind == 1:
            cases.append(rng.standard_normal((r, c)).astype(np.float32))
        else:
            cases.append((rng.random((r, c)) * 1e4).round().astype(np.float32))
    for _ in range(4):
        cases.append(rng.random((256, 256)).astype(np.float32))
    return cases
