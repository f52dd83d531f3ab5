"""Pin the CPU oracle against the reference's golden vectors (CPU-only)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
import gen_common as G


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


# ---------------------------------------------------------------- LSAP ----
def _lsap_cases():
    d = _load("lsap_golden.npz")
    shapes, data, offs = d["shapes"], d["data"], d["offs"]
    pos = 0
    for q, (r, c) in enumerate(shapes):
        C = data[pos:pos + r * c].reshape(r, c)
        pos += r * c
        yield q, C, d["rows"][offs[q]:offs[q + 1]], d["cols"][offs[q]:offs[q + 1]], int(d["status"][q])


def test_lsap_matches_scipy_golden(oracle):
    n = 0
    for q, C, rows, cols, st in _lsap_cases():
        if st == 0:
            r, c = oracle.lsap(C)
            assert np.array_equal(r, rows) and np.array_equal(c, cols), f"case {q} {C.shape}"
        else:
            with pytest.raises(ValueError, match="invalid" if st == -1 else "infeasible"):
                oracle.lsap(C)
        n += 1
    assert n >= 150


def test_hungarian_assign_golden(oracle):
    d = _load("lsap_golden.npz")
    cases = [C for _, C, _, _, _ in _lsap_cases()]
    for k, (q, cm) in enumerate(zip(d["hm_q"], d["hm_cost_max"])):
        m, _, _ = oracle.hungarian_assign(cases[q], cost_max=float(cm))
        exp = d["hm_match"][d["hm_moff"][k]:d["hm_moff"][k + 1]]
        assert np.array_equal(np.asarray(m, np.int64).reshape(-1, 2), exp)


def test_lsap_empty_and_errors(oracle):
    r, c = oracle.lsap(np.zeros((0, 5)))
    assert r.shape == (0,) and c.dtype == np.int64
    with pytest.raises(ValueError):
        oracle.lsap(np.array([[1.0, -np.inf]]))


# ---------------------------------------------------------------- cost ----
@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_costcard_formula_bit_exact(oracle, tag):
    d = _load("costcard_golden.npz")
    out = oracle.cost_combine(d[f"{tag}_capp"], d[f"{tag}_bp"], d[f"{tag}_bc"],
                              d[f"{tag}_cp"], d[f"{tag}_cu"])
    for k in ("C_center", "C_scale", "C_conf", "C_bbox", "C_total"):
        exp = d[f"{tag}_{k}"]
        got = out[k]
        # bit-exact except transcendental ulps (torch CPU log is SLEEF, C logf is glibc)
        assert np.max(np.abs(got - exp)) <= 2e-6 * max(1.0, np.abs(exp).max()), k
    assert np.array_equal(out["C_center"], d[f"{tag}_C_center"])


@pytest.mark.parametrize("name", ["s16", "s64", "reid"])
def test_cost_and_gate_vs_reference_tracker(oracle, name):
    d = _load(f"track_golden_{name}.npz")
    det_off = d["det_off"]
    checked = 0
    for f in d["dump_frames"]:
        if f"f{f}_rows_main" not in d.files or f"f{f}_state_tids" not in d.files:
            continue
        tids = d[f"f{f}_state_tids"]
        rows = d[f"f{f}_rows_main"]
        sel = np.searchsorted(tids, rows)
        a, b = det_off[f], det_off[f + 1]
        st = {k: d[f"f{f}_state_{k}"][sel] for k in ("bank", "bank_len", "pbox", "last_conf", "kf_x", "kf_P")}
        gm, gs = oracle.gate_params(st["kf_x"], st["kf_P"])
        out = oracle.cost_build(st["bank"], st["bank_len"], d["embs"][a:b], st["pbox"], d["boxes"][a:b],
                                st["last_conf"], d["confs"][a:b], gm, gs, np.ones(len(rows), np.int32))
        assert np.max(np.abs(out["C_app"] - d[f"f{f}_C_app"])) < 1e-5
        pre = oracle.cost_build(st["bank"], st["bank_len"], d["embs"][a:b], st["pbox"], d["boxes"][a:b],
                                st["last_conf"], d["confs"][a:b])
        assert np.max(np.abs(pre["C_total"] - d[f"f{f}_C_total"])) < 1e-5
        for k in ("C_center", "C_scale", "C_conf"):
            assert np.max(np.abs(pre[k] - d[f"f{f}_{k}"])) < 1e-5, k
        gated = d[f"f{f}_C_gated"]
        assert np.array_equal(out["C_total"] >= 1e9, gated >= 1e9)
        assert np.max(np.abs(out["C_total"] - gated)) < 1e-5
        checked += 1
    assert checked >= 2


@pytest.mark.parametrize("name", ["s16", "s64", "reid"])
def test_stage1_assignment_on_reference_costs(oracle, name):
    """hungarian_assign on the reference's own gated cost reproduces the
    reference's stage-1 matches for every frame (mainTracking.py:514-534)."""
    d = _load(f"track_golden_{name}.npz")
    n = 0
    for f in range(int(d["n_frames"])):
        if f"f{f}_C_gated" not in d.files:
            continue
        rows = d[f"f{f}_rows_main"]
        m, _, _ = oracle.hungarian_assign(d[f"f{f}_C_gated"], cost_max=50.0)
        exp = d["matches"][d["m_off"][f]:d["m_off"][f + 1]]
        got = np.array([(rows[i], j) for i, j in m], np.int64).reshape(-1, 2)
        assert np.array_equal(got, exp[:len(got)])
        n += 1
    assert n > 5


# ---------------------------------------------------------- ROI Align ----
def test_roi_align_constant_map(oracle):
    x = np.full((1, 3, 12, 12), 2.5, np.float32)
    rois = np.array([[0, 1.5, 2.0, 8.0, 9.5], [0, 0.0, 0.0, 11.0, 11.0]], np.float32)
    out = oracle.roi_align(x, rois, (7, 7), 1.0)
    assert np.allclose(out, 2.5, atol=1e-6)


def test_roi_align_affine_ramp_exact(oracle):
    """f(y,x) = 3x + 2y + 1 is reproduced exactly by bilinear sampling inside
    the map: each bin = value at the mean sample position."""
    H = W = 16
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    x = (3 * xx + 2 * yy + 1)[None, None].astype(np.float32)
    x1, y1, x2, y2 = 2.25, 3.0, 10.75, 12.5
    out = oracle.roi_align(x, np.array([[0, x1, y1, x2, y2]], np.float32), (4, 4), 1.0, 2, True)
    sw, sh = x1 - 0.5, y1 - 0.5
    bw, bh = (x2 - x1) / 4, (y2 - y1) / 4
    for ph in range(4):
        for pw in range(4):
            cy = sh + (ph + 0.5) * bh
            cx = sw + (pw + 0.5) * bw
            assert abs(out[0, 0, ph, pw] - (3 * cx + 2 * cy + 1)) < 1e-4


def test_roi_align_out_of_bounds_zero(oracle):
    x = np.random.default_rng(0).standard_normal((1, 2, 8, 8)).astype(np.float32)
    out = oracle.roi_align(x, np.array([[0, 100, 100, 140, 150]], np.float32), (3, 3), 1.0)
    assert np.all(out == 0)


def test_roi_align_batch_index_and_scale(oracle):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 4, 10, 10)).astype(np.float32)
    r = np.array([[1, 40, 48, 200, 260]], np.float32)
    a = oracle.roi_align(x, r, (5, 5), 1 / 32)
    r0 = r.copy(); r0[0, 0] = 0
    b = oracle.roi_align(x[1:], r0, (5, 5), 1 / 32)
    assert np.array_equal(a, b)


# ------------------------------------------------------------ encoder ----
@pytest.mark.parametrize("s", [7, 10])
def test_encoder_restatement_vs_reference(oracle, s):
    import torch
    d = _load("encoder_golden.npz")
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    x = torch.from_numpy(G.encoder_input(int(d[f"seed_s{s}"]), 16, s))
    with torch.no_grad():
        z = oracle.encoder_forward(sd, x).numpy()
    assert np.max(np.abs(z - d[f"z_s{s}"])) < 1e-5


def test_cost_nan_semantics_follow_torch(oracle):
    """NaN inputs: the oracle ranks a NaN similarity first (torch.topk puts NaN above
    every number) and keeps NaN through the clamps (torch clamp(min=)), as the
    reference's build_C_app_topk / bbox_cost / conf_cost do (mainTracking.py:191-203,
    costCard.py:150-201).  Checked against the same torch ops, literally."""
    import torch
    rng = np.random.default_rng(4)
    M, N, T = 6, 7, 9
    bank = rng.standard_normal((M, T, 128)).astype(np.float32)
    bank /= np.linalg.norm(bank, axis=-1, keepdims=True)
    det = rng.standard_normal((N, 128)).astype(np.float32)
    det[2, 0] = np.nan
    bank[4, 7, 3] = np.nan
    blen = np.full(M, T, np.int32)
    blen[1] = 3
    pbox = np.tile(np.float32([[100, 300, 180, 420]]), (M, 1)) + rng.uniform(0, 20, (M, 4)).astype(np.float32)
    dbox = np.tile(np.float32([[100, 300, 180, 420]]), (N, 1)) + rng.uniform(0, 20, (N, 4)).astype(np.float32)
    dbox[5, 3] = np.nan
    lc = rng.uniform(0.5, 1, M).astype(np.float32)
    dc = rng.uniform(0.5, 1, N).astype(np.float32)
    dc[6] = np.nan
    with np.errstate(invalid="ignore"):
        got = oracle.cost_build(bank, blen, det, pbox, dbox, lc, dc)
    # the reference's torch ops
    F_det = torch.from_numpy(det / (np.linalg.norm(det, axis=1, keepdims=True) + 1e-12))
    capp = []
    for i in range(M):
        b = bank[i, :blen[i]]
        F_bank = torch.from_numpy(b / (np.linalg.norm(b, axis=1, keepdims=True) + 1e-12))
        sim = F_bank @ F_det.T
        capp.append(1.0 - torch.topk(sim, k=min(5, sim.shape[0]), dim=0)[0].mean(0))
    capp = torch.stack(capp).numpy()
    bp, bc = torch.from_numpy(pbox), torch.from_numpy(dbox)
    wp, hp = (bp[:, 2] - bp[:, 0]).clamp(min=1.0), (bp[:, 3] - bp[:, 1]).clamp(min=1.0)
    wc, hc = (bc[:, 2] - bc[:, 0]).clamp(min=1.0), (bc[:, 3] - bc[:, 1]).clamp(min=1.0)
    scl = torch.abs(torch.log(((wc * hc)[None, :] / (wp * hp)[:, None]).clamp(min=1e-6))).numpy()
    cf = torch.abs(torch.log(torch.from_numpy(dc).clamp(min=1e-6)[None, :] /
                             torch.from_numpy(lc).clamp(min=1e-6)[:, None])).numpy()
    assert np.array_equal(np.isnan(got["C_app"]), np.isnan(capp))
    assert np.array_equal(np.isnan(got["C_scale"]), np.isnan(scl))
    assert np.array_equal(np.isnan(got["C_conf"]), np.isnan(cf))
    assert np.isnan(got["C_app"][:, 2]).all() and np.isnan(got["C_app"][4]).all()
    tot_nan = np.isnan(capp) | np.isnan(scl) | np.isnan(cf) | np.isnan(dbox).any(1)[None, :]
    assert np.array_equal(np.isnan(got["C_total"]), tot_nan)
    f = ~np.isnan(capp)
    assert np.max(np.abs(got["C_app"][f] - capp[f])) <= 2e-6


@pytest.mark.parametrize("name", ["s16", "s64", "reid", "n256"])
def test_tracker_restatement_vs_reference_golden(oracle, name):
    """oracle/tracker_ref.TrackerRef (Tracking.update restated over the oracle's cost,
    LSAP and filterpy restatements) reproduces the reference's own per-frame outputs,
    including the N = 256 scene (inputs regenerated from its seed, digest-checked)."""
    import tracker_ref as TR
    d = _load(f"track_golden_{name}.npz")
    if name in G.OUTPUT_ONLY:
        frames = G.scene(name)
        assert G.scene_digest(frames) == str(d["digest"])
        inputs = [(list(fr["embs"]), fr["bboxes"], fr["confs"]) for fr in frames]
    else:
        off = d["det_off"]
        inputs = [(list(d["embs"][off[f]:off[f + 1]]), d["boxes"][off[f]:off[f + 1]].tolist(),
                   d["confs"][off[f]:off[f + 1]].tolist()) for f in range(int(d["n_frames"]))]
    t = TR.TrackerRef()
    for f, (e, bx, cf) in enumerate(inputs):
        got = t.update(e, bx, cf)
        m = d["matches"][d["m_off"][f]:d["m_off"][f + 1]]
        ut = d["um_tracks"][d["um_t_off"][f]:d["um_t_off"][f + 1]]
        ud = d["um_dets"][d["um_d_off"][f]:d["um_d_off"][f + 1]]
        exp = ([tuple(map(int, x)) for x in m], [int(x) for x in ut], [int(x) for x in ud])
        assert got == exp, f"{name} frame {f}"


# ROI Align boundary branches of SURVEY A.1 (torchvision's CPU kernel): a sample at
# exactly y == -1 or y == H is valid and clamps, one past them contributes 0; a sample
# in (H-1, H) has yl >= H-1 and reads row H-1 with ly = 0; aligned=False widens a ROI
# narrower than one cell to rw = 1.  Same for x.  The map is f = 3x + 2y + 1, which
# bilinear sampling reproduces exactly at the clamped positions.
def _affine_map(H=8, W=8, C=2):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    f = (3 * xx + 2 * yy + 1).astype(np.float32)
    return np.stack([f, -f])[None, :C].astype(np.float32)


def _a1_expected(roi, H, W, PH, PW, sr=2, aligned=True):
    """A.1 in float64 on f = 3x + 2y + 1 (channel 0)"""
    off = 0.5 if aligned else 0.0
    sw, sh, ew, eh = roi[1] - off, roi[2] - off, roi[3] - off, roi[4] - off
    rw, rh = ew - sw, eh - sh
    if not aligned:
        rw, rh = max(rw, 1.0), max(rh, 1.0)
    bh, bw = rh / PH, rw / PW
    out = np.zeros((PH, PW))
    for ph in range(PH):
        for pw in range(PW):
            acc = 0.0
            for iy in range(sr):
                for ix in range(sr):
                    y = sh + ph * bh + (iy + 0.5) * bh / sr
                    x = sw + pw * bw + (ix + 0.5) * bw / sr
                    if y < -1 or y > H or x < -1 or x > W:
                        continue
                    y, x = max(y, 0.0), max(x, 0.0)
                    y = float(H - 1) if int(y) >= H - 1 else y
                    x = float(W - 1) if int(x) >= W - 1 else x
                    acc += 3 * x + 2 * y + 1
            out[ph, pw] = acc / (sr * sr)
    return out


A1_BOUNDARY_ROIS = [
    # (roi, PH, PW, aligned, what)
    ((0, 2.0, -0.75, 5.0, 0.25), 1, 1, True, "y samples at exactly -1 (valid, clamps to 0) and -0.5"),
    ((0, 2.0, -1.0, 5.0, 0.0), 1, 1, True, "y samples at -1.25 (outside: 0) and -0.75"),
    ((0, 2.0, 8.25, 5.0, 9.25), 1, 1, True, "y samples at exactly H (valid, row H-1) and H + 0.5 (outside)"),
    ((0, 2.0, 7.0, 5.0, 8.0), 1, 1, True, "y samples in (H-1, H): yl >= H-1, row H-1, ly = 0"),
    ((0, -0.75, 2.0, 0.25, 5.0), 1, 1, True, "x samples at exactly -1 and -0.5"),
    ((0, 8.25, 2.0, 9.25, 5.0), 1, 1, True, "x samples at exactly W and W + 0.5"),
    ((0, 3.0, 3.0, 3.3, 3.2), 2, 2, False, "aligned=False, rw, rh < 1 -> 1"),
    ((0, 7.6, 7.7, 7.9, 7.95), 3, 3, False, "aligned=False, sub-cell ROI at the far corner"),
]


@pytest.mark.parametrize("k", range(len(A1_BOUNDARY_ROIS)))
def test_roi_align_a1_boundary_branches(oracle, k):
    roi, PH, PW, aligned, what = A1_BOUNDARY_ROIS[k]
    x = _affine_map()
    out = oracle.roi_align(x, np.array([roi], np.float32), (PH, PW), 1.0, 2, aligned)
    exp = _a1_expected(np.float32(roi).astype(np.float64), 8, 8, PH, PW, 2, aligned)
    assert np.max(np.abs(out[0, 0] - exp)) < 1e-4, what
    assert np.array_equal(out[0, 1], -out[0, 0]), what
