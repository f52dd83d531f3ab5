"""Parity of the gfx950 kernels (through the C ABI) against the CPU oracle and
the reference's golden vectors.  Tolerances are written in each test:
  roi_align f32: bit-exact;  bf16 output: == bf16(round-to-nearest of f32) with the exact
    arithmetic (roi_fma=0); the default fused arithmetic (roi_fma=1) within the tolerance
    of test_roi_align_sweep_variants
  cost: |d| <= 2e-6 (f32 dot-order / logf ulp differences), gate decisions equal
  lsap: indices bit-exact (scipy semantics)
  encoder fp32: <= 1e-4 (north star);  bf16: |d| <= 1.2e-3, cosine >= 1 - 5e-6 vs fp32 (2x measured)
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
import gen_common as G

pytestmark = pytest.mark.gpu


# ----------------------------------------------------------------- helpers
def _boxes(rng, n, img=1280, pad=280):
    w = rng.uniform(32, 320, n)
    h = rng.uniform(32, 320, n)
    x1 = rng.uniform(-8, img - w + 8)
    y1 = rng.uniform(pad - 8, img - pad - h + 8)
    return np.stack([x1, y1, x1 + w, y1 + h], 1).astype(np.float32)


def _feat(rng, B, C=512, H=40, W=40):
    return G.silu_np(rng.standard_normal((B, C, H, W)).astype(np.float32)).astype(np.float32)


# --------------------------------------------------------------- roi_align
@pytest.mark.parametrize("N", [16, 64, 256])
@pytest.mark.parametrize("S", [7, 10])
def test_roi_align_bit_exact_vs_oracle(trk, oracle, gpu, N, S):
    rng = np.random.default_rng(N * 10 + S)
    feat = _feat(rng, 1)
    boxes = _boxes(rng, N)
    rois = np.concatenate([np.zeros((N, 1), np.float32), boxes], 1)
    exp = oracle.roi_align(feat, rois, (S, S), 40 / 1280.0, 2, True)
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    got = trk.roi_align(x, r, (S, S), 40 / 1280.0, 2, True)
    assert got.shape == (N, 512, S, S) and got.is_contiguous()
    assert np.array_equal(got.cpu().numpy(), exp)
    nhwc = trk.roi_align(x, r, (S, S), 40 / 1280.0, 2, True, channels_last=True)
    assert nhwc.is_contiguous(memory_format=torch.channels_last)
    assert np.array_equal(nhwc.cpu().numpy(), exp)
    L = trk.lib()
    try:  # bf16 output with the exact arithmetic (roi_fma=0) == bf16(f32); roi_fma: test_roi_align_sweep_variants
        assert L.trk_set_tuning(b"roi_fma", 0) == 0
        bf = trk.roi_align(x, r, (S, S), 40 / 1280.0, 2, True, out_dtype=torch.bfloat16, channels_last=True)
    finally:
        L.trk_set_tuning(b"roi_fma", 1)
    assert torch.equal(bf.cpu(), torch.from_numpy(exp).bfloat16())


@pytest.mark.parametrize("out", ["f32", "bf16_nhwc"])
def test_roi_align_full_size_properties(trk, oracle, gpu, out):
    """The bench's c3 launch ([8, 512, 40, 40] NCHW maps, 8 x 256 ROIs, 10 x 10 bins), where the
    CPU oracle is too slow to run, checked through properties exact in the arithmetic of both the
    exact f32 path and the default bf16 channels-last path (fused multiply-adds):
      * homogeneity: 2 x map -> exactly 2 x output (every product and sum scales by a power of 2);
      * channel equivariance: permuting the map's channels permutes the output's channels;
      * frame independence: a ROI on frame b equals the same ROI on a batch whose frame 0 is b;
      * integer translation: boxes moved by exactly one map cell (32 px at scale 1/32) on a map
        moved by one cell give the same output, for ROIs clear of the map's edges whose corners
        are multiples of 1/16 px and sizes of 10/16 px (so every sample coordinate is a short
        dyadic number and moves by exactly 1.0);
    and the 2,048 outputs against the oracle for 32 of them (all frames)."""
    rng = np.random.default_rng(77)
    B, N, C = 8, 256, 512
    feat = torch.from_numpy(_feat(rng, B)).to(gpu)
    boxes = np.stack([_boxes(rng, N) for _ in range(B)])
    rois = np.concatenate([np.repeat(np.arange(B), N).astype(np.float32)[:, None], boxes.reshape(-1, 4)], 1)
    r = torch.from_numpy(rois).to(gpu)
    kw = dict(out_dtype=torch.bfloat16, channels_last=True) if out == "bf16_nhwc" else {}
    ra = lambda f, rr: trk.roi_align(f, rr, (10, 10), 40 / 1280.0, 2, True, **kw).float()
    base = ra(feat, r)
    assert torch.isfinite(base).all()
    assert torch.equal(ra(feat * 2, r), base * 2)
    perm = torch.randperm(C, generator=torch.Generator().manual_seed(5)).to(gpu)
    assert torch.equal(ra(feat[:, perm].contiguous(), r), base[:, perm])
    sel = torch.arange(0, B * N, 61, device=gpu)  # ROIs of every frame
    b_of = r[sel, 0].long()
    r0 = r[sel].clone()
    r0[:, 0] = 0
    one = torch.stack([ra(feat[b:b + 1].contiguous(), r0[k:k + 1]) for k, b in enumerate(b_of.tolist())])
    assert torch.equal(one.squeeze(1), base[sel])
    # translation: boxes inside cells [2, 36] of the 40 x 40 map, moved by +1 cell in x and y
    dy = lambda lo, hi, q: torch.from_numpy((np.round(rng.uniform(lo, hi, B * N) / q) * q).astype(np.float32)).to(gpu)
    x1, y1 = dy(64, 1000, 1 / 16), dy(64, 1000, 1 / 16)
    w, h = dy(32, 120, 10 / 16), dy(32, 120, 10 / 16)
    rt = torch.stack([r[:, 0], x1, y1, x1 + w, y1 + h], 1)
    rs = rt.clone()
    rs[:, 1:] += 32.0
    shifted = torch.zeros_like(feat)
    shifted[:, :, 1:, 1:] = feat[:, :, :-1, :-1]
    assert torch.equal(ra(shifted, rs), ra(feat, rt))
    if out == "f32":
        pick = sel[:32].cpu().numpy()
        exp = oracle.roi_align(feat.cpu().numpy(), rois[pick], (10, 10), 40 / 1280.0, 2, True)
        assert np.array_equal(base[sel[:32]].cpu().numpy(), exp)


@pytest.mark.parametrize("shape", [(8, 512, 40, 40), (2, 36, 13, 12), (1, 70, 9, 7), (3, 4, 1, 4)])
def test_nchw_to_nhwc_transpose(trk, gpu, shape):
    """The map transpose roi_align runs on NCHW input (float4 kernel when C and H*W are
    multiples of 4, else the scalar one): exactly torch's channels_last copy, partial 64 x 64
    tiles at the channel and pixel ends included."""
    x = torch.randn(shape, generator=torch.Generator().manual_seed(sum(shape))).to(gpu)
    got = trk.nchw_to_nhwc(x)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, x.contiguous(memory_format=torch.channels_last))


def test_roi_align_batched_frames_and_edges(trk, oracle, gpu):
    rng = np.random.default_rng(3)
    B, N = 8, 256
    feat = _feat(rng, B)
    boxes = _boxes(rng, B * N)
    bidx = np.repeat(np.arange(B), N).astype(np.float32)[:, None]
    rois = np.concatenate([bidx, boxes], 1)
    # edge cases: fully outside, crossing every border, degenerate, tiny, huge
    rois[0, 1:] = [2000, 2000, 2100, 2100]
    rois[1, 1:] = [-300, -300, 100, 100]
    rois[2, 1:] = [1200, 1200, 1400, 1500]
    rois[3, 1:] = [500, 500, 500, 500]
    rois[4, 1:] = [600, 610, 600.5, 611]
    rois[5, 1:] = [-50, -50, 1330, 1330]
    rois[6, 1:] = [700, 700, 650, 640]  # inverted
    exp = oracle.roi_align(feat, rois, (10, 10), 1 / 32, 2, True)
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    got = trk.roi_align(x, r, (10, 10), 1 / 32, 2, True)
    assert np.array_equal(got.cpu().numpy(), exp)
    # channels_last input skips the transpose, same result
    got2 = trk.roi_align(x.contiguous(memory_format=torch.channels_last), r, (10, 10), 1 / 32, 2, True)
    assert np.array_equal(got2.cpu().numpy(), exp)
    # aligned=False, other sampling ratio, non-square bins
    exp3 = oracle.roi_align(feat, rois[:300], (7, 5), 1 / 32, 3, False)
    got3 = trk.roi_align(x, r[:300], (7, 5), 1 / 32, 3, False)
    assert np.array_equal(got3.cpu().numpy(), exp3)


@pytest.mark.parametrize("sweep", [1, 2, 0])
def test_roi_align_nhwc_out_paths(trk, oracle, gpu, sweep):
    """NHWC output goes through the row-sweep kernel (register column cache);
    roi_sweep=0 selects the per-sample-tap kernel.  Both bit-exact, including
    edge ROIs, sampling ratios 1..4, aligned=False, non-square bins and a
    channel count that leaves a partial chunk."""
    L = trk.lib()
    rng = np.random.default_rng(11)
    B, N = 3, 96
    feat = _feat(rng, B, C=516, H=23, W=31)
    boxes = _boxes(rng, B * N, img=992, pad=100)
    rois = np.concatenate([np.repeat(np.arange(B), N).astype(np.float32)[:, None], boxes], 1)
    rois[0, 1:] = [2000, 2000, 2100, 2100]
    rois[1, 1:] = [-300, -300, 100, 100]
    rois[2, 1:] = [900, 700, 1400, 1500]
    rois[3, 1:] = [500, 500, 500, 500]
    rois[4, 1:] = [700, 700, 650, 640]
    rois[5, 1:] = [-50, -50, 1330, 1330]
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    try:
        L.trk_set_tuning(b"roi_sweep", sweep)
        L.trk_set_tuning(b"roi_fma", 0)  # bf16 == bf16(f32) below: the exact arithmetic
        for (ph, pw), sr, al in (((10, 10), 2, True), ((7, 7), 2, True), ((7, 5), 3, False),
                                 ((4, 6), 1, True), ((5, 3), 4, True)):
            exp = oracle.roi_align(feat, rois, (ph, pw), 1 / 32, sr, al)
            got = trk.roi_align(x, r, (ph, pw), 1 / 32, sr, al, channels_last=True)
            assert np.array_equal(got.cpu().numpy(), exp), (ph, pw, sr, al)
            bf = trk.roi_align(x, r, (ph, pw), 1 / 32, sr, al, out_dtype=torch.bfloat16, channels_last=True)
            assert torch.equal(bf.cpu(), torch.from_numpy(exp).bfloat16()), (ph, pw, sr, al)
    finally:
        L.trk_set_tuning(b"roi_sweep", 1)
        L.trk_set_tuning(b"roi_fma", 1)


@pytest.mark.parametrize("knobs", [dict(roi_asm=0, roi_fma=0), dict(roi_asm=1, roi_fma=0),
                                   dict(roi_asm=0, roi_fma=1), dict(roi_asm=1, roi_fma=1)])
def test_roi_align_sweep_variants(trk, oracle, gpu, knobs):
    """Row-sweep variants (both knobs default to 1).  roi_asm: the bilinear sample as
    one asm block and one column cache for sample rows that share their map rows --
    the same operations in the same order, bit-exact in f32 and bf16.  roi_fma (bf16
    output only): the three additions of each sample fused into their products, so a
    sample moves by at most ~3 f32 roundings of its largest product; tolerance
    written here: |got - f32 oracle| <= 2^-8 |oracle| (bf16 rounding) + 2^-19 max|map|,
    and >= 99.9 % of the outputs identical to bf16(oracle).  f32 output stays exact."""
    L = trk.lib()
    rng = np.random.default_rng(12)
    B, N = 4, 200
    feat = _feat(rng, B)
    boxes = _boxes(rng, B * N)
    rois = np.concatenate([np.repeat(np.arange(B), N).astype(np.float32)[:, None], boxes], 1)
    rois[0, 1:] = [2000, 2000, 2100, 2100]
    rois[1, 1:] = [-300, -300, 100, 100]
    rois[2, 1:] = [1200, 1200, 1400, 1500]
    rois[3, 1:] = [500, 500, 500, 500]
    rois[4, 1:] = [-50, -50, 1330, 1330]
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    fma = bool(knobs.get("roi_fma"))
    try:
        for k, v in knobs.items():
            assert L.trk_set_tuning(k.encode(), v) == 0
        for (ph, pw) in ((10, 10), (7, 7)):
            exp = oracle.roi_align(feat, rois, (ph, pw), 1 / 32, 2, True)
            f32 = trk.roi_align(x, r, (ph, pw), 1 / 32, 2, True, channels_last=True)
            assert np.array_equal(f32.cpu().numpy(), exp), (ph, knobs)
            bf = trk.roi_align(x, r, (ph, pw), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True).cpu()
            want = torch.from_numpy(exp).bfloat16()
            if not fma:
                assert torch.equal(bf, want), (ph, knobs)
                continue
            got = bf.float().numpy()
            tol = np.abs(exp) * 2.0 ** -8 + 2.0 ** -19 * float(np.abs(feat).max())
            assert np.all(np.abs(got - exp) <= tol), (ph, float(np.max(np.abs(got - exp) - tol)))
            same = float((bf.view(torch.int16) == want.view(torch.int16)).float().mean())
            assert same >= 0.999, (ph, same)
    finally:
        for k in knobs:
            L.trk_set_tuning(k.encode(), 1)  # the defaults


@pytest.mark.parametrize("C,sweep,ph", [(256, 1, 10), (128, 1, 7), (512, 2, 10), (1024, 2, 7), (512, 1, 1),
                                        (128, 1, 1), (260, 1, 10)])
def test_roi_align_sweep_one_chunk_and_one_row(trk, oracle, gpu, C, sweep, ph):
    """The row sweep's work-item decomposition divides by the chunk count and by PH with
    magic multipliers; a divisor of 1 (C <= 256 channels per wave, 512 with roi_sweep=2,
    or a single bin row) has no 32-bit multiplier and takes its own branch.  Every
    output written and bit-exact vs the oracle (f32; bf16 with the exact arithmetic)."""
    L = trk.lib()
    rng = np.random.default_rng(C + ph)
    B, N = 2, 40
    feat = _feat(rng, B, C=C)
    boxes = _boxes(rng, B * N)
    rois = np.concatenate([np.repeat(np.arange(B), N).astype(np.float32)[:, None], boxes], 1)
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    try:
        assert L.trk_set_tuning(b"roi_sweep", sweep) == 0
        assert L.trk_set_tuning(b"roi_fma", 0) == 0
        for pw in (10, 7):
            exp = oracle.roi_align(feat, rois, (ph, pw), 1 / 32, 2, True)
            got = trk.roi_align(x, r, (ph, pw), 1 / 32, 2, True, channels_last=True)
            assert np.array_equal(got.cpu().numpy(), exp), (C, sweep, ph, pw)
            bf = trk.roi_align(x, r, (ph, pw), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True)
            assert torch.equal(bf.cpu(), torch.from_numpy(exp).bfloat16()), (C, sweep, ph, pw)
    finally:
        L.trk_set_tuning(b"roi_sweep", 1)
        L.trk_set_tuning(b"roi_fma", 1)


@pytest.mark.parametrize("fma", [0, 1])
def test_roi_align_nan_at_origin(trk, oracle, gpu, fma):
    """torchvision's CPU kernel reads pixel (0,0) with weight 0 for a sample outside the
    map, so a NaN there reaches exactly the bins that have such a sample.  Both the
    exact and the fused (bf16 default) arithmetic keep that read: the NaN positions equal
    the oracle's, and every other output is within the test_roi_align_sweep_variants
    tolerance (bit-exact with the exact arithmetic)."""
    L = trk.lib()
    rng = np.random.default_rng(21)
    B, N = 2, 64
    feat = _feat(rng, B)
    feat[:, :, 0, 0] = np.nan
    boxes = _boxes(rng, B * N)
    rois = np.concatenate([np.repeat(np.arange(B), N).astype(np.float32)[:, None], boxes], 1)
    rois[0, 1:] = [2000, 2000, 2100, 2100]  # all samples outside
    rois[1, 1:] = [-300, -300, 100, 100]    # some outside
    rois[N, 1:] = [1200, 1200, 1400, 1500]
    x = torch.from_numpy(feat).to(gpu)
    r = torch.from_numpy(rois).to(gpu)
    try:
        assert L.trk_set_tuning(b"roi_fma", fma) == 0
        exp = oracle.roi_align(feat, rois, (10, 10), 1 / 32, 2, True)
        assert np.isnan(exp).any() and not np.isnan(exp).all()
        bf = trk.roi_align(x, r, (10, 10), 1 / 32, 2, True, out_dtype=torch.bfloat16, channels_last=True)
        got = bf.cpu().float().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(exp))
        ok = ~np.isnan(exp)
        if fma:
            tol = np.abs(exp[ok]) * 2.0 ** -8 + 2.0 ** -19 * float(np.nanmax(np.abs(feat)))
            assert np.all(np.abs(got[ok] - exp[ok]) <= tol)
        else:
            assert np.array_equal(got[ok], torch.from_numpy(exp).bfloat16().float().numpy()[ok])
    finally:
        L.trk_set_tuning(b"roi_fma", 1)


def test_roi_align_odd_channels_and_empty(trk, oracle, gpu):
    rng = np.random.default_rng(4)
    feat = rng.standard_normal((2, 37, 13, 11)).astype(np.float32)
    rois = np.array([[1, 10, 20, 200, 300], [0, 0, 0, 30, 30]], np.float32)
    exp = oracle.roi_align(feat, rois, (3, 4), 1 / 16, 2, True)
    got = trk.roi_align(torch.from_numpy(feat).to(gpu), torch.from_numpy(rois).to(gpu), (3, 4), 1 / 16, 2, True)
    assert np.array_equal(got.cpu().numpy(), exp)
    e = trk.roi_align(torch.from_numpy(feat).to(gpu), torch.zeros((0, 5), device=gpu), (7, 7), 1.0, 2, True)
    assert e.shape == (0, 37, 7, 7)


def test_roi_align_from_input_boxes_reference_contract(trk, oracle, gpu):
    rng = np.random.default_rng(5)
    feat = _feat(rng, 1)
    boxes = _boxes(rng, 33).astype(np.float64).tolist()
    got = trk.roi_align_from_input_boxes(torch.from_numpy(feat).to(gpu), boxes, (1280, 1280), out_size=(7, 7))
    rois = np.array([[0.0] + b for b in boxes], np.float32)
    exp = oracle.roi_align(feat, rois, (7, 7), 40 / 1280.0, 2, True)
    assert np.array_equal(got.cpu().numpy(), exp)


# -------------------------------------------------------------------- cost
def _state_from_golden(d, f):
    tids = d[f"f{f}_state_tids"]
    rows = d[f"f{f}_rows_main"]
    sel = np.searchsorted(tids, rows)
    return {k: d[f"f{f}_state_{k}"][sel] for k in ("bank", "bank_len", "pbox", "last_conf", "kf_x", "kf_P")}


def _renorm(x):
    x = np.asarray(x, np.float32)
    n = np.sqrt((x.astype(np.float64) ** 2).sum(-1, keepdims=True)).astype(np.float32) + np.float32(1e-12)
    return (x / n).astype(np.float32)


def _run_cost(trk, gpu, bank, blen, pbox, lconf, gm, gs, det, dbox, dconf, gate=True):
    M, N = bank.shape[0], det.shape[0]
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)
    out = trk.build_cost(M=[M], N=[N], bank=t(_renorm(bank)), bank_len=t(blen, torch.int32), pbox=t(pbox),
                         conf_prev=t(lconf), det_emb=t(det[None]), dbox=t(dbox[None]),
                         conf_cur=t(dconf[None]), params=trk.default_cost_params(gate=gate),
                         gmean=t(gm, torch.float64), gsinv=t(gs, torch.float64),
                         gate_on=t(np.ones(M, np.int32), torch.int32),
                         want=("C_total", "C_app", "C_center", "C_scale", "C_conf"))
    res = {k: v[0].cpu().numpy() for k, v in out.items()}
    # C_total / C_app only: the bank-resident kernel (det_prep + cost3).  Exact f32 products
    # (cost_split 0): bit-identical; the default f16 hi / lo split: within SPLIT_TOL, gate
    # decisions equal
    L = trk.lib()
    for split in (0, 1):
        assert L.trk_set_tuning(b"cost_split", split) == 0
        try:
            out3 = trk.build_cost(M=[M], N=[N], bank=t(_renorm(bank)), bank_len=t(blen, torch.int32), pbox=t(pbox),
                                  conf_prev=t(lconf), det_emb=t(det[None]), dbox=t(dbox[None]),
                                  conf_cur=t(dconf[None]), params=trk.default_cost_params(gate=gate),
                                  gmean=t(gm, torch.float64), gsinv=t(gs, torch.float64),
                                  gate_on=t(np.ones(M, np.int32), torch.int32), want=("C_total", "C_app"))
        finally:
            L.trk_set_tuning(b"cost_split", 1)
        for k in ("C_total", "C_app"):
            got3 = out3[k][0].cpu().numpy()
            if split == 0:
                assert np.array_equal(got3, res[k], equal_nan=True), k
            else:
                assert np.array_equal(np.isnan(got3), np.isnan(res[k])), k
                assert np.array_equal(got3 >= 1e9, res[k] >= 1e9), k
                ok = ~np.isnan(got3)
                assert np.max(np.abs(got3[ok] - res[k][ok]), initial=0.0) <= SPLIT_TOL, k
        res["split_" + "C_total"], res["split_C_app"] = out3["C_total"][0].cpu().numpy(), out3["C_app"][0].cpu().numpy()
    return res


# cost_split (the default cost3 path): the similarity of two unit rows from f16 hi / lo splits is
# within 1.1e-6 of the exact f32 products (cost.hip split16: the dropped lo*lo term, lo's two f16
# roundings and its subnormal floor); C_app = 1 - mean of top-k similarities moves by no more, and
# C_total by w_app (0.6) times that
SPLIT_TOL = 1.1e-6


@pytest.mark.parametrize("name", ["s16", "s64", "reid"])
def test_cost_kernel_vs_reference_golden(trk, oracle, gpu, name):
    d = np.load(os.path.join(GOLDEN, f"track_golden_{name}.npz"))
    n = 0
    for f in d["dump_frames"]:
        if f"f{f}_rows_main" not in d.files or f"f{f}_state_tids" not in d.files:
            continue
        st = _state_from_golden(d, f)
        a, b = d["det_off"][f], d["det_off"][f + 1]
        gm, gs = oracle.gate_params(st["kf_x"], st["kf_P"])
        got = _run_cost(trk, gpu, st["bank"], st["bank_len"], st["pbox"], st["last_conf"], gm, gs,
                        d["embs"][a:b], d["boxes"][a:b].astype(np.float32), d["confs"][a:b].astype(np.float32))
        assert np.max(np.abs(got["C_app"] - d[f"f{f}_C_app"])) <= 2e-6
        for k in ("C_center", "C_scale", "C_conf"):
            assert np.max(np.abs(got[k] - d[f"f{f}_{k}"])) <= 2e-6, k
        gated = d[f"f{f}_C_gated"]
        assert np.array_equal(got["C_total"] >= 1e9, gated >= 1e9)
        assert np.max(np.abs(got["C_total"] - gated)) <= 2e-6
        n += 1
    assert n >= 2


def test_cost_kernel_full_size_vs_oracle(trk, oracle, gpu):
    """N = M = 256, full banks (T = 30) and ragged banks, gate on."""
    rng = np.random.default_rng(21)
    M = N = 256
    base = _renorm(rng.standard_normal((M, 128)))
    bank = _renorm(base[:, None, :] + 0.05 * rng.standard_normal((M, 30, 128)))
    blen = np.full(M, 30, np.int32)
    blen[:40] = rng.integers(0, 30, 40)
    bank[np.arange(30)[None, :] >= blen[:, None]] = 0
    perm = rng.permutation(N)
    det = _renorm(base[perm] + 0.05 * rng.standard_normal((N, 128)))
    pbox = _boxes(rng, M)
    dbox = pbox[perm] + rng.normal(0, 2, (N, 4)).astype(np.float32)
    lconf = rng.uniform(0.55, 0.99, M).astype(np.float32)
    dconf = rng.uniform(0.55, 0.99, N).astype(np.float32)
    x = np.zeros((M, 8)); x[:, :4] = np.stack([(pbox[:, 0] + pbox[:, 2]) / 2, (pbox[:, 1] + pbox[:, 3]) / 2,
                                               (pbox[:, 2] - pbox[:, 0]) / (pbox[:, 3] - pbox[:, 1]),
                                               pbox[:, 3] - pbox[:, 1]], 1)
    P = np.tile(np.diag([10., 10, 10, 10, 1000, 1000, 1000, 1000]), (M, 1, 1))
    gm, gs = oracle.gate_params(x, P)
    got = _run_cost(trk, gpu, bank, blen, pbox, lconf, gm, gs, det, dbox, dconf)
    exp = oracle.cost_build(_renorm(bank), blen, det, pbox, dbox, lconf, dconf, gm, gs, np.ones(M, np.int32))
    assert np.max(np.abs(got["C_app"] - exp["C_app"])) <= 2e-6
    assert np.array_equal(got["C_total"] >= 1e9, exp["C_total"] >= 1e9)
    assert np.max(np.abs(got["C_total"] - exp["C_total"])) <= 2e-6
    assert (exp["C_total"] >= 1e9).mean() > 0.5  # the gate is exercised
    # det-tile kernel (default) and the bank-resident kernel (cost_v2): identical outputs
    L = trk.lib()
    try:
        assert L.trk_set_tuning(b"cost_v2", 1) == 0
        got1 = _run_cost(trk, gpu, bank, blen, pbox, lconf, gm, gs, det, dbox, dconf)
    finally:
        assert L.trk_set_tuning(b"cost_v2", 0) == 0
    for k in got:
        if not k.startswith("split_"):
            assert np.array_equal(got[k], got1[k]), k
    # the default (split) cost3 outputs against the oracle, as the exact ones above
    assert np.max(np.abs(got["split_C_app"] - exp["C_app"])) <= 2e-6
    assert np.array_equal(got["split_C_total"] >= 1e9, exp["C_total"] >= 1e9)
    assert np.max(np.abs(got["split_C_total"] - exp["C_total"])) <= 2e-6


def test_cost_dev_full_size_permutation_properties(trk, gpu):
    """The bench's cost launch (8 frames x 256 tracks x 256 detections, T = 30, gate on, the
    default f16-split cost3 through trk_build_cost_dev with a workspace), beyond the oracle's
    one-frame check: permuting a frame's detections permutes its columns and permuting its row
    slots permutes its rows, bit for bit (each (track, detection) entry is computed the same way
    whichever tile and lane hold it), and the launch is deterministic."""
    import ctypes
    from importlib import import_module
    ops = import_module(trk.__name__ + ".ops")
    rng = np.random.default_rng(41)
    F, M, N, T = 8, 256, 256, 30
    S = F * M
    bank = _renorm(rng.standard_normal((S, T, 128)))
    blen = np.full(S, T, np.int32)
    blen[::9] = rng.integers(0, T, len(blen[::9]))
    bank[np.arange(T)[None, :] >= blen[:, None]] = 0
    pbox = _boxes(rng, S)
    lconf = rng.uniform(0.3, 1, S).astype(np.float32)
    gm = np.concatenate([(pbox[:, :2] + pbox[:, 2:]) / 2, pbox[:, 2:] - pbox[:, :2]], 1).astype(np.float64)
    gs = np.tile(np.eye(4).reshape(1, 16) * 1e-4, (S, 1))  # gated beyond ~300 px: both outcomes occur
    det = rng.standard_normal((F, N, 128)).astype(np.float32)
    dbox = np.stack([_boxes(rng, N) for _ in range(F)])
    dconf = rng.uniform(0.3, 1, (F, N)).astype(np.float32)
    slots = np.arange(S, dtype=np.int32).reshape(F, M)
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)
    L = trk.lib()
    params = trk.default_cost_params(gate=True)
    P = ops._ptr
    work = torch.empty(int(L.trk_cost_work_bytes(F, N)), device=gpu, dtype=torch.uint8)
    dev = dict(bank=t(bank), blen=t(blen, torch.int32), pbox=t(pbox), lconf=t(lconf), gm=t(gm, torch.float64),
               gs=t(gs, torch.float64), gon=t(np.ones(S, np.int32), torch.int32),
               M=t(np.full(F, M, np.int32), torch.int32), N=t(np.full(F, N, np.int32), torch.int32))

    def run(det_, dbox_, dconf_, slots_):
        Ct = torch.full((F, M, N), -7.0, device=gpu)
        Ca = torch.full((F, M, N), -7.0, device=gpu)
        d, b, c, sl = t(det_), t(dbox_), t(dconf_), t(slots_, torch.int32)
        rc = L.trk_build_cost_dev(F, M, N, P(dev["M"]), P(dev["N"]), P(sl), M, T, P(dev["bank"]), P(dev["blen"]),
                                  P(dev["pbox"]), P(dev["lconf"]), P(dev["gm"]), P(dev["gs"]), P(dev["gon"]), P(d),
                                  P(b), P(c), ctypes.byref(params), P(Ct), P(Ca), P(work), ops._stream(gpu))
        assert rc == 0
        torch.cuda.synchronize()
        return Ct.cpu().numpy(), Ca.cpu().numpy()

    Ct, Ca = run(det, dbox, dconf, slots)
    Ct2, Ca2 = run(det, dbox, dconf, slots)
    assert np.array_equal(Ct, Ct2) and np.array_equal(Ca, Ca2)
    assert 0.05 < (Ct >= 1e9).mean() < 0.95  # the gate is exercised both ways
    dp = np.stack([rng.permutation(N) for _ in range(F)])
    rp = np.stack([rng.permutation(M) for _ in range(F)])
    fi = np.arange(F)[:, None]
    Ctp, Cap = run(det[fi, dp], dbox[fi, dp], dconf[fi, dp], slots[fi, rp])
    assert np.array_equal(Ctp, Ct[fi[:, :, None], rp[:, :, None], dp[:, None, :]])
    assert np.array_equal(Cap, Ca[fi[:, :, None], rp[:, :, None], dp[:, None, :]])


def test_cost_batched_frames_with_row_slots(trk, oracle, gpu):
    rng = np.random.default_rng(22)
    F, Mmax, Nmax, S = 3, 40, 48, 200
    bank = _renorm(rng.standard_normal((S, 30, 128)))
    blen = rng.integers(1, 31, S).astype(np.int32)
    pbox = _boxes(rng, S)
    lconf = rng.uniform(0.3, 1, S).astype(np.float32)
    Ms, Ns = [40, 17, 0], [48, 5, 9]
    slots = np.stack([rng.permutation(S)[:Mmax] for _ in range(F)]).astype(np.int32)
    det = _renorm(rng.standard_normal((F, Nmax, 128)))
    dbox = np.stack([_boxes(rng, Nmax) for _ in range(F)])
    dconf = rng.uniform(0.3, 1, (F, Nmax)).astype(np.float32)
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)
    out = trk.build_cost(M=Ms, N=Ns, bank=t(bank), bank_len=t(blen, torch.int32), pbox=t(pbox),
                         conf_prev=t(lconf), det_emb=t(det), dbox=t(dbox), conf_cur=t(dconf),
                         params=trk.default_cost_params(gate=False), row_slot=t(slots, torch.int32),
                         want=("C_total", "C_app"))
    for f in range(F):
        M, N = Ms[f], Ns[f]
        if M == 0:
            continue
        s = slots[f, :M]
        exp = oracle.cost_build(bank[s], blen[s], det[f, :N], pbox[s], dbox[f, :N], lconf[s], dconf[f, :N])
        assert np.max(np.abs(out["C_total"][f, :M, :N].cpu().numpy() - exp["C_total"])) <= 2e-6


def test_cost_dev_bank_resident_vs_det_tile(trk, oracle, gpu):
    """trk_build_cost_dev with a workspace (det_prep + cost3: the bank read once
    per launch) against the same call without one (cost_kernel): bit-identical,
    and against the oracle; ragged N (not a multiple of 32), row slots, gate on,
    device-side sizes, an empty frame."""
    import ctypes
    from importlib import import_module
    ops = import_module(trk.__name__ + ".ops")
    rng = np.random.default_rng(23)
    F, Mmax, Nmax, S, T = 3, 40, 70, 200, 30
    bank = _renorm(rng.standard_normal((S, T, 128)))
    bank[::7, 1:] = bank[::7, :1]  # ties: every row of these banks the same
    blen = rng.integers(0, 31, S).astype(np.int32)
    bank[np.arange(T)[None, :] >= blen[:, None]] = 0
    pbox = _boxes(rng, S)
    lconf = rng.uniform(0.3, 1, S).astype(np.float32)
    x = np.zeros((S, 8)); x[:, :4] = np.stack([(pbox[:, 0] + pbox[:, 2]) / 2, (pbox[:, 1] + pbox[:, 3]) / 2,
                                               (pbox[:, 2] - pbox[:, 0]) / (pbox[:, 3] - pbox[:, 1]),
                                               pbox[:, 3] - pbox[:, 1]], 1)
    gm, gs = oracle.gate_params(x, np.tile(np.diag([10., 10, 10, 10, 1000, 1000, 1000, 1000]), (S, 1, 1)))
    gate_on = (rng.random(S) < 0.8).astype(np.int32)
    Ms, Ns = np.array([40, 17, 0], np.int32), np.array([70, 5, 9], np.int32)
    slots = np.stack([rng.permutation(S)[:Mmax] for _ in range(F)]).astype(np.int32)
    det = rng.standard_normal((F, Nmax, 128)).astype(np.float32)   # not normalised: the kernel renormalises
    dbox = np.stack([_boxes(rng, Nmax) for _ in range(F)])
    dconf = rng.uniform(0.3, 1, (F, Nmax)).astype(np.float32)
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)
    dev = dict(bank=t(bank), blen=t(blen, torch.int32), pbox=t(pbox), lconf=t(lconf), gm=t(gm, torch.float64),
               gs=t(gs, torch.float64), gon=t(gate_on, torch.int32), det=t(det), dbox=t(dbox), dconf=t(dconf),
               M=t(Ms, torch.int32), N=t(Ns, torch.int32), slots=t(slots, torch.int32))
    L = trk.lib()
    params = trk.default_cost_params(gate=True)
    P = ops._ptr

    def run(work):
        Ct = torch.full((F, Mmax, Nmax), -7.0, device=gpu)
        Ca = torch.full((F, Mmax, Nmax), -7.0, device=gpu)
        rc = L.trk_build_cost_dev(F, Mmax, Nmax, P(dev["M"]), P(dev["N"]), P(dev["slots"]), Mmax, T, P(dev["bank"]),
                                  P(dev["blen"]), P(dev["pbox"]), P(dev["lconf"]), P(dev["gm"]), P(dev["gs"]),
                                  P(dev["gon"]), P(dev["det"]), P(dev["dbox"]), P(dev["dconf"]), ctypes.byref(params),
                                  P(Ct), P(Ca), P(work), ops._stream(gpu))
        assert rc == 0
        torch.cuda.synchronize()
        return Ct.cpu().numpy(), Ca.cpu().numpy()

    work = torch.empty(int(L.trk_cost_work_bytes(F, Nmax)), device=gpu, dtype=torch.uint8)
    # cost3's top-k: a sorting network for topk <= 5 (two tiles per step, lane halves swapping the
    # partial lists), insertion for 6..8; both must give cost_kernel's sums bit for bit, with banks
    # shorter than topk (blen 0..30) and exact ties (a few banks repeat one row)
    for topk in (1, 3, 8):
        params.topk = topk
        Ct1, Ca1 = run(None)
        assert L.trk_set_tuning(b"cost_split", 0) == 0
        try:
            Ct3e, Ca3e = run(work)
        finally:
            L.trk_set_tuning(b"cost_split", 1)
        assert np.array_equal(Ct3e, Ct1) and np.array_equal(Ca3e, Ca1), topk
    params.topk = 5
    Ct1, Ca1 = run(None)
    assert L.trk_set_tuning(b"cost_split", 0) == 0
    try:
        Ct3e, Ca3e = run(work)
    finally:
        L.trk_set_tuning(b"cost_split", 1)
    assert np.array_equal(Ct3e, Ct1) and np.array_equal(Ca3e, Ca1)  # exact f32 products: bit-identical
    Ct3, Ca3 = run(work)  # the default f16 split
    assert np.array_equal(Ct3 >= 1e9, Ct1 >= 1e9)
    assert np.max(np.abs(Ca3 - Ca1)) <= SPLIT_TOL and np.max(np.abs(Ct3 - Ct1)) <= SPLIT_TOL
    for f in range(F):
        M, N = int(Ms[f]), int(Ns[f])
        assert (Ct3[f, M:] == -7.0).all() and (Ct3[f, :, N:] == -7.0).all()  # nothing written outside M x N
        if M == 0:
            continue
        s = slots[f, :M]
        exp = oracle.cost_build(bank[s], blen[s], det[f, :N], pbox[s], dbox[f, :N], lconf[s], dconf[f, :N],
                                gm[s], gs[s], gate_on[s])
        assert np.max(np.abs(Ca3[f, :M, :N] - exp["C_app"])) <= 2e-6
        assert np.array_equal(Ct3[f, :M, :N] >= 1e9, exp["C_total"] >= 1e9)
        assert np.max(np.abs(Ct3[f, :M, :N] - exp["C_total"])) <= 2e-6


def test_cost_nan_inputs_propagate_like_torch(trk, oracle, gpu):
    """A NaN embedding, bank row, box or confidence reaches C_total as NaN where the
    reference's torch ops put it (torch.topk ranks NaN largest, clamp(min=) keeps
    NaN: mainTracking.py:201-203, costCard.py:150-201), so hungarian_assign raises
    scipy's ValueError instead of assigning around it; all other entries are
    unchanged (vs the oracle, which restates the same rules)."""
    rng = np.random.default_rng(31)
    M, N = 20, 24
    base = _renorm(rng.standard_normal((M, 128)))
    bank = _renorm(base[:, None, :] + 0.05 * rng.standard_normal((M, 30, 128)))
    blen = np.full(M, 30, np.int32)
    blen[:4] = [0, 1, 3, 7]
    bank[np.arange(30)[None, :] >= blen[:, None]] = 0
    det = rng.standard_normal((N, 128)).astype(np.float32)
    pbox, dbox = _boxes(rng, M), _boxes(rng, N)
    lconf = rng.uniform(0.55, 0.99, M).astype(np.float32)
    dconf = rng.uniform(0.55, 0.99, N).astype(np.float32)
    det[3, 17] = np.nan          # one embedding
    bank[9, 2, 5] = np.nan       # one stored bank row of a full bank
    bank[1, 0, 0] = np.nan       # a bank with one entry
    dbox[7, 2] = np.nan          # a detection box
    dconf[11] = np.nan           # a detection confidence
    pbox[13, 1] = np.nan         # a predicted track box
    lconf[15] = np.nan           # a track's last confidence
    # ungated (a gated pair's 1e9 replaces whatever C_total held, NaN included, as in the
    # reference's apply_kalman_gating; the gate itself is unchanged by this rule)
    gm, gs = np.zeros((M, 4)), np.tile(np.eye(4).reshape(1, 16), (M, 1))
    got = _run_cost(trk, gpu, bank, blen, pbox, lconf, gm, gs, det, dbox, dconf, gate=False)
    with np.errstate(invalid="ignore"):
        exp = oracle.cost_build(_renorm(bank), blen, det, pbox, dbox, lconf, dconf)
    for k in ("C_app", "C_total"):
        g, e = got[k], exp[k]
        assert np.array_equal(np.isnan(g), np.isnan(e)), k
        assert np.isnan(g).any(), k
        f = ~np.isnan(e)
        assert np.max(np.abs(g[f] - e[f])) <= 2e-6, k
    nanc = np.isnan(got["C_total"])
    assert nanc[1:, 3].all() and nanc[9].all() and nanc[1].all() and nanc[:, 7].all() and nanc[:, 11].all()
    assert nanc[13].all() and nanc[15].all()
    assert not nanc[0, 3] and not np.isnan(got["C_app"][0]).any()  # row 0: empty bank, C_app = 1 (no sims)
    with pytest.raises(ValueError, match="invalid numeric entries"):
        trk.hungarian_assign(torch.from_numpy(got["C_total"]).to(gpu), cost_max=50.0)


@pytest.mark.parametrize("Tmax", [33, 50, 96])
def test_cost_bank_longer_than_32(trk, oracle, gpu, Tmax):
    """hist_max > 32 (any YAML value, reference mainTracking.py:56): the bank is walked
    in 32-row MFMA chunks with one running top-k; equal to the oracle, with ragged and
    empty banks, through both entry points (all five outputs / C_total + C_app)."""
    rng = np.random.default_rng(Tmax)
    M, N = 40, 45
    base = _renorm(rng.standard_normal((M, 128)))
    bank = _renorm(base[:, None, :] + 0.1 * rng.standard_normal((M, Tmax, 128)))
    blen = rng.integers(0, Tmax + 1, M).astype(np.int32)
    blen[:3] = [0, Tmax, 31]
    bank[np.arange(Tmax)[None, :] >= blen[:, None]] = 0
    det = rng.standard_normal((N, 128)).astype(np.float32)
    pbox = _boxes(rng, M)
    dbox = _boxes(rng, N)
    lconf = rng.uniform(0.55, 0.99, M).astype(np.float32)
    dconf = rng.uniform(0.55, 0.99, N).astype(np.float32)
    x = np.zeros((M, 8)); x[:, :4] = np.stack([(pbox[:, 0] + pbox[:, 2]) / 2, (pbox[:, 1] + pbox[:, 3]) / 2,
                                               (pbox[:, 2] - pbox[:, 0]) / (pbox[:, 3] - pbox[:, 1]),
                                               pbox[:, 3] - pbox[:, 1]], 1)
    gm, gs = oracle.gate_params(x, np.tile(np.diag([10., 10, 10, 10, 1000, 1000, 1000, 1000]), (M, 1, 1)))
    got = _run_cost(trk, gpu, bank, blen, pbox, lconf, gm, gs, det, dbox, dconf)  # also checks the 2-output path
    exp = oracle.cost_build(_renorm(bank), blen, det, pbox, dbox, lconf, dconf, gm, gs, np.ones(M, np.int32))
    assert np.max(np.abs(got["C_app"] - exp["C_app"])) <= 2e-6
    assert np.array_equal(got["C_total"] >= 1e9, exp["C_total"] >= 1e9)
    assert np.max(np.abs(got["C_total"] - exp["C_total"])) <= 2e-6


def test_costcard_api_vs_reference_golden(trk, gpu):
    d = np.load(os.path.join(GOLDEN, "costcard_golden.npz"))
    for tag in "abc":
        out = trk.cal_cost(C_app=torch.from_numpy(d[f"{tag}_capp"]).to(gpu), boxes_prev=d[f"{tag}_bp"].tolist(),
                           boxes_cur=d[f"{tag}_bc"].tolist(), input_hw=(1280, 1280),
                           conf_prev=d[f"{tag}_cp"].tolist(), conf_cur=d[f"{tag}_cu"].tolist())
        for k in ("C_total", "C_center", "C_scale", "C_conf", "C_bbox"):
            assert np.max(np.abs(out[k].cpu().numpy() - d[f"{tag}_{k}"])) <= 2e-6, k


# -------------------------------------------------------------------- LSAP
def _lsap_cases():
    d = np.load(os.path.join(GOLDEN, "lsap_golden.npz"))
    pos = 0
    for q, (r, c) in enumerate(d["shapes"]):
        C = d["data"][pos:pos + r * c].reshape(r, c)
        pos += r * c
        yield q, C, d["rows"][d["offs"][q]:d["offs"][q + 1]], d["cols"][d["offs"][q]:d["offs"][q + 1]], int(d["status"][q])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_lsap_vs_scipy_golden(trk, gpu, dtype):
    for q, C, rows, cols, st in _lsap_cases():
        if st == 0:
            r, c = trk.linear_sum_assignment(C.astype(dtype))
            assert np.array_equal(r, rows) and np.array_equal(c, cols), f"case {q} {C.shape}"
        else:
            with pytest.raises(ValueError, match="invalid" if st == -1 else "infeasible"):
                trk.linear_sum_assignment(C.astype(dtype))


def test_lsap_batched_one_launch(trk, gpu):
    cases = [(C, r, c) for _, C, r, c, st in _lsap_cases() if st == 0]
    R = max(C.shape[0] for C, _, _ in cases)
    L = max(C.shape[1] for C, _, _ in cases)
    buf = np.zeros((len(cases), R, L), np.float32)
    for k, (C, _, _) in enumerate(cases):
        buf[k, :C.shape[0], :C.shape[1]] = C
    res = trk.lsap_batched(torch.from_numpy(buf).to(gpu), [C.shape[0] for C, _, _ in cases],
                           [C.shape[1] for C, _, _ in cases], cost_max=50.0)
    rows, cols, cnt = res["rows"].cpu().numpy(), res["cols"].cpu().numpy(), res["count"].cpu().numpy()
    assert (res["status"].cpu().numpy() == 0).all()
    for k, (C, r, c) in enumerate(cases):
        assert np.array_equal(rows[k, :cnt[k]], r) and np.array_equal(cols[k, :cnt[k]], c), k


def test_hungarian_assign_vs_reference_golden(trk, gpu):
    d = np.load(os.path.join(GOLDEN, "lsap_golden.npz"))
    cases = [C for _, C, _, _, _ in _lsap_cases()]
    for k, (q, cm) in enumerate(zip(d["hm_q"], d["hm_cost_max"])):
        m, ut, ud = trk.hungarian_assign(cases[q], cost_max=float(cm))
        exp = d["hm_match"][d["hm_moff"][k]:d["hm_moff"][k + 1]]
        assert np.array_equal(np.asarray(m, np.int64).reshape(-1, 2), exp)
        M, N = cases[q].shape
        assert sorted(ut + [i for i, _ in m]) == list(range(M))
        assert sorted(ud + [j for _, j in m]) == list(range(N))
    assert trk.hungarian_assign(np.zeros((0, 3))) == ([], [], [0, 1, 2])
    assert trk.hungarian_assign(np.zeros((2, 0))) == ([], [0, 1], [])


def test_lsap_full_size_vs_oracle(trk, oracle, gpu):
    rng = np.random.default_rng(30)
    mats = [rng.random((256, 256)).astype(np.float32),
            rng.integers(0, 3, (256, 256)).astype(np.float32),
            np.where(rng.random((256, 256)) < 0.9, np.float32(1e9), rng.random((256, 256)).astype(np.float32)),
            rng.random((300, 256)).astype(np.float32), rng.random((200, 512)).astype(np.float32),
            rng.random((1024, 1024)).astype(np.float32)]
    for C in mats:
        r, c = trk.linear_sum_assignment(C)
        er, ec = oracle.lsap(C)
        assert np.array_equal(r, er) and np.array_equal(c, ec), C.shape


def test_lsap_widest_body_vs_oracle(trk, oracle, gpu):
    """Matrices wider than 1024 columns run the 32-slot body (444 VGPRs per wave, the only
    instantiation past 256): index-identical to the oracle, f32 and f64, wide and tall (the
    solver transposes a tall matrix)."""
    rng = np.random.default_rng(31)
    for shape in ((300, 1500), (1100, 400)):
        C = rng.random(shape)
        er, ec = oracle.lsap(C)
        for dt in (np.float32, np.float64):
            Cd = C.astype(dt)
            er2, ec2 = (er, ec) if dt == np.float64 else oracle.lsap(Cd)
            r, c = trk.linear_sum_assignment(Cd)
            assert np.array_equal(r, er2) and np.array_equal(c, ec2), (shape, dt)


# ----------------------------------------------------------------- encoder
@pytest.mark.parametrize("s", [7, 10])
def test_encoder_gpu_vs_reference_golden(trk, gpu, s):
    d = np.load(os.path.join(GOLDEN, "encoder_golden.npz"))
    m = trk.Model(512, 512, 10, 128).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
    m = m.to(gpu)
    x = torch.from_numpy(G.encoder_input(int(d[f"seed_s{s}"]), 16, s)).to(gpu)
    with torch.no_grad():
        z = m(x).cpu().numpy()
        zb = m(x.bfloat16().contiguous(memory_format=torch.channels_last)).float().cpu().numpy()
    exp = d[f"z_s{s}"]
    assert np.max(np.abs(z - exp)) <= 1e-4
    print(f"\nbf16 encoder vs golden s={s}: max |d| {np.max(np.abs(zb - exp)):.3e}, "
          f"min cosine {(zb * exp).sum(1).min():.7f}")
    # measured on MI355X (r04, gpurun_out/r4k_chain.log): s=7 max |d| 5.51e-4, min cosine
    # 1 - 2.2e-6; s=10 4.94e-4, 1 - 1.8e-6.  Bounds: about 2x
    assert np.max(np.abs(zb - exp)) <= 1.2e-3
    assert (zb * exp).sum(1).min() >= 1.0 - 5e-6
    # bf16: fused trk GEMMs vs the hipBLASLt + separate-pass graph (same bf16 rounding points
    # except the means, which the fused epilogues take in f32 before rounding)
    try:
        m.fused_gemm = False
        with torch.no_grad():
            zu = m(x.bfloat16().contiguous(memory_format=torch.channels_last)).float().cpu().numpy()
    finally:
        m.fused_gemm = True
    assert (zb * zu).sum(1).min() >= 0.9999


def _bf16_ref_rows(Y2, W2, b2):
    """fp32 reference of the DSC pair on bf16 operands"""
    Kg = W2.shape[2]
    xr = Y2[:, :Kg].float() @ W2[0].float().t() + b2[:W2.shape[1]]
    xn = Y2[:, Kg:].float() @ W2[1].float().t() + b2[W2.shape[1]:]
    return xr, xn


@pytest.mark.parametrize("P,R", [(100, 37), (49, 29)])
def test_enc_fused_gemms_vs_torch_fp32(trk, gpu, P, R):
    """trk_enc_dsc_gemm / trk_enc_transition_gemm vs a torch fp32 reference on the same
    bf16 operands (tol: bf16 output rounding for stored values; 2e-3 relative for sums).
    M = R*P is not a multiple of the 128-row tile and ROIs straddle tiles."""
    import torch.nn.functional as F
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(P)
    M, Kg, Ng = R * P, 512, 512
    Y2 = torch.randn(M, 2 * Kg, generator=g).to(gpu).bfloat16()
    W2 = (torch.randn(2, Ng, Kg, generator=g) / 24).to(gpu).bfloat16()
    b2 = (torch.randn(2 * Ng, generator=g) / 4).to(gpu)
    XRN, sr, sn = ops.enc_dsc_gemm(Y2, P, W2, b2)
    xr, xn = _bf16_ref_rows(Y2, W2, b2)
    hn = F.hardswish(xn)
    sr_ = F.silu(xr)
    assert (XRN[:, :Ng].float() - sr_).abs().max().item() <= 1e-2 * max(1.0, sr_.abs().max().item())
    assert (XRN[:, Ng:].float() - hn).abs().max().item() <= 1e-2 * max(1.0, hn.abs().max().item())
    ref_sr = F.silu(xr).view(R, P, Ng).sum(1)
    ref_sn = hn.view(R, P, Ng).sum(1)
    assert (sr - ref_sr).abs().max().item() <= 2e-3 * ref_sr.abs().max().item()
    assert (sn - ref_sn).abs().max().item() <= 2e-3 * ref_sn.abs().max().item()
    # deterministic: a second run gives the same bits
    XRN2, sr2, sn2 = ops.enc_dsc_gemm(Y2, P, W2, b2)
    assert torch.equal(XRN, XRN2) and torch.equal(sr, sr2) and torch.equal(sn, sn2)
    # transition with the SE scale applied in the prologue
    s = torch.rand(R, Ng, generator=g).to(gpu)
    Wt = (torch.randn(Ng, 2 * Ng, generator=g) / 32).to(gpu).bfloat16()
    bt = (torch.randn(Ng, generator=g) / 4).to(gpu)
    st = ops.enc_transition_gemm(XRN, P, s, Wt, bt)
    xs = (XRN[:, :Ng].float().view(R, P, Ng) * s[:, None, :]).bfloat16().float().view(M, Ng)
    A = torch.cat([xs, XRN[:, Ng:].float()], 1)
    ref_t = F.silu(A @ Wt.float().t() + bt).view(R, P, Ng).sum(1)
    assert (st - ref_t).abs().max().item() <= 2e-3 * ref_t.abs().max().item()
    st2 = ops.enc_transition_gemm(XRN, P, s, Wt, bt)
    assert torch.equal(st, st2)
    if P == 100:
        # first GEMM + depthwise 5x5 fused (g1dw4) against the fp32 GEMM rounded to bf16 +
        # dwconv5_nhwc, odd ROI count (a half-filled last tile): Y1 sums its products in another
        # order, so a Y1 value can round to the neighbouring bf16 (2^-8 relative), which moves the
        # Y2 outputs it feeds by |w| times that; deterministic run to run
        W1 = (torch.randn(1024, 512, generator=g) / 24).to(gpu).bfloat16()
        X = Y2[:, :512].contiguous()
        wdw = (torch.randn(25, 1024, generator=g) / 5).to(gpu)
        Y1 = (X.float() @ W1.float().t()).bfloat16()
        Yu = ops.dwconv5_nhwc(Y1.view(R, 10, 10, 1024), wdw).view(M, 1024)
        Y7 = ops.enc_g1_dwconv(X, W1, wdw)
        Y7b = ops.enc_g1_dwconv(X, W1, wdw)
        assert torch.equal(Y7, Y7b)
        d = (Y7.float() - Yu.float()).abs()
        assert d.max().item() <= 2e-2 * Yu.float().abs().max().item()
        assert (d == 0).float().mean().item() >= 0.9


@pytest.mark.parametrize("P,R", [(100, 1), (100, 37), (100, 2048), (200, 23), (49, 29)])
def test_enc_transition_trans4_vs_gemm4(trk, gpu, P, R):
    """trans4 (enc_trans 1: the weights straight into VGPRs from the packed fragments,
    4 waves x 64 columns x 128 rows) vs gemm4 (weights through LDS, 2 x 2 waves): the same
    MFMA operands and K order, the same SE-scaled bf16 rows and the same per-64-row-block
    MFMA sums, so the reduced ROI sums must be bit-identical; deterministic run to run."""
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(2000 + R + P)
    M, Ng = R * P, 512
    XRN = torch.randn(M, 2 * Ng, generator=g).to(gpu).bfloat16()
    s = torch.rand(R, Ng, generator=g).to(gpu)
    Wt = (torch.randn(Ng, 2 * Ng, generator=g) / 32).to(gpu).bfloat16()
    bt = (torch.randn(Ng, generator=g) / 4).to(gpu)
    Wtp = ops.enc_pack_fragments_k(Wt)
    assert Wtp[3, 5, 2, 7, 4].item() == Wt[16 * 5 + 7, 32 * 3 + 8 * 2 + 4].item()
    ref = ops.enc_transition_gemm(XRN, P, s, Wt, bt)  # no fragments: gemm4 whatever the knob
    L = trk.lib()
    try:
        assert L.trk_set_tuning(b"enc_trans", 1) == 0
        got = ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
        got2 = ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
        assert L.trk_set_tuning(b"enc_trans", 0) == 0
        nopk = ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)  # knob 0: gemm4 with the fragments given
    finally:
        L.trk_set_tuning(b"enc_trans", 1)
    assert torch.equal(got, ref) and torch.equal(got2, ref) and torch.equal(nopk, ref)
    with pytest.raises(ValueError, match="enc_pack_fragments_k"):
        ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp[:-1])


@pytest.mark.parametrize("N", [768, 1024])
def test_enc_transition_packed_weights_need_n512(trk, gpu, N):
    """trans4 steps one K step of its packed fragments as 32 column tiles (N = 512): packed
    weights of another N are refused by the wrapper and by the C ABI (never read in the wrong
    order); without them gemm4 handles any N % 256 == 0 and matches the fp32 reference."""
    import torch.nn.functional as F
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(N)
    P, R = 100, 5
    M = R * P
    XRN = torch.randn(M, 1024, generator=g).to(gpu).bfloat16()
    s = torch.rand(R, 512, generator=g).to(gpu)
    Wt = (torch.randn(N, 1024, generator=g) / 32).to(gpu).bfloat16()
    bt = (torch.randn(N, generator=g) / 4).to(gpu)
    Wtp = ops.enc_pack_fragments_k(Wt)
    with pytest.raises(ValueError, match="enc_pack_fragments_k"):
        ops.enc_transition_gemm(XRN, P, s, Wt, bt, Wtp=Wtp)
    sums = torch.empty((R, 3, N), device=gpu, dtype=torch.int64)
    c = lambda t: ctypes.c_void_p(t.data_ptr())
    L = trk.lib()
    assert L.trk_enc_transition_gemm2(c(XRN), M, P, 1024, c(s), 512, c(Wt), c(Wtp), c(bt), N, c(sums), None) == -1
    assert b"N = 512" in L.trk_last_error()
    st = ops.enc_transition_gemm(XRN, P, s, Wt, bt)
    xs = (XRN[:, :512].float().view(R, P, 512) * s[:, None, :]).bfloat16().float().view(M, 512)
    ref = F.silu(torch.cat([xs, XRN[:, 512:].float()], 1) @ Wt.float().t() + bt).view(R, P, N).sum(1)
    assert (st - ref).abs().max().item() <= 2e-3 * ref.abs().max().item()


def _front_operands(gpu, R, seed):
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(R * 100, 512, generator=g).to(gpu).bfloat16()
    W1 = (torch.randn(1024, 512, generator=g) / 24).to(gpu).bfloat16()
    wdw = (torch.randn(25, 1024, generator=g) / 5).to(gpu)
    W2 = (torch.randn(2, 512, 512, generator=g) / 24).to(gpu).bfloat16()
    b2 = (torch.randn(1024, generator=g) / 10).to(gpu)
    se = [(torch.randn(128, 512, generator=g) / 20).to(gpu), (torch.randn(128, generator=g) / 10).to(gpu),
          (torch.randn(512, 128, generator=g) / 10).to(gpu), (torch.randn(512, generator=g) / 10).to(gpu)]
    return ops, X, W1, wdw, W2, b2, se


@pytest.mark.parametrize("groups,chunks", [(0, 1), (1, 1), (14, 1), (16, 1), (64, 1), (16, 4), (1, 7), (0, 64)])
@pytest.mark.parametrize("R", [1, 37, 2048])
def test_enc_rmb_front_vs_two_kernel_path(trk, gpu, R, groups, chunks):
    """trk_enc_rmb_front_means (first 1x1 convs + depthwise + DSC GEMMs in one kernel, Y2 in
    LDS, the squeeze means written by the kernel) vs enc_g1_dwconv -> enc_dsc_gemm -> enc_se:
    the same MFMA shape, K order and bf16 roundings, so XRN must be bit-identical; the means add
    the same f32 activations in another order (tol 1e-5 of the largest mean).  R = 2048 is the
    bench's c3 launch.  groups: rf3_groups, the persistent grid's workgroup pairs per XCD (0 =
    CUs / 16 - 2, the default; 1 pair: 256 ROIs per workgroup at R = 2048, the LDS counters
    counting on across all of them; 64: more pairs than ROIs); chunks: rf3_chunks, the grid as
    that many generations of workgroups, each running one chunk of its pair's ROIs (more
    chunks than a pair has ROIs: capped, or empty workgroups exit)."""
    ops, X, W1, wdw, W2, b2, se = _front_operands(gpu, R, R)
    L = trk.lib()
    P = 100
    Y2 = ops.enc_g1_dwconv(X, W1, wdw)
    XRN2, sums2 = ops.enc_dsc_gemm(Y2, P, W2, b2, raw=True)
    m_r2, m_n2, s2 = ops.enc_se(sums2, P, *se)
    W1p, W2p = ops.enc_pack_fragments(W1), ops.enc_pack_fragments(W2)
    # the packing is a permutation: fragment (g, s, n, lane) holds W[g*512+16n+lane%16][32s+8(lane//16)+j]
    assert W1p[1, 3, 5, 2, 7, 4].item() == W1[512 + 16 * 5 + 7, 32 * 3 + 8 * 2 + 4].item()
    assert L.trk_set_tuning(b"rf3_groups", groups) == 0 and L.trk_set_tuning(b"rf3_chunks", chunks) == 0
    try:
        XRN1, m_r1, m_n1 = ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
        XRN1b, m_r1b, m_n1b = ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)  # deterministic
        torch.cuda.synchronize()
    finally:
        L.trk_set_tuning(b"rf3_groups", 0)
        L.trk_set_tuning(b"rf3_chunks", 1)
    assert torch.equal(XRN1, XRN2)
    for a, b in ((m_r1, m_r2), (m_n1, m_n2)):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()
    assert torch.equal(XRN1, XRN1b) and torch.equal(m_r1, m_r1b) and torch.equal(m_n1, m_n1b)
    # the SE from given means is enc_se's arithmetic: the same s for the same m_r
    assert torch.equal(ops.enc_se_means(m_r2, *se), s2)
    # unpacked weights (same numel) are refused, not read in the wrong order
    with pytest.raises(ValueError, match="enc_pack_fragments"):
        ops.enc_rmb_front_means(X, W1, wdw, W2p, b2)
    with pytest.raises(ValueError, match="enc_pack_fragments"):
        ops.enc_rmb_front_means(X, W1p, wdw, W2.reshape(1024, 512), b2)


@pytest.mark.parametrize("chunks", [1, 4])
def test_enc_front_progress_and_stream_gate(trk, gpu, chunks):
    """enc_rmb_front_means' `progress` argument: a launch adds one per finished ROI (R = 37 and
    300, the persistent grid and 4 generations) to the caller's counter and leaves the results
    unchanged; a launch without it leaves the counter alone (the library keeps no pointer).
    trk_stream_gate: returns at once once the count is reached, after its bound otherwise, and
    the work queued behind it then runs.  The counter starts at 0xFFFFFF00, so the fronts carry
    it across the u32 wrap: the gate's comparison is wrap-safe (a reached target past the wrap
    opens at once, one not yet reached before the wrap waits for its bound)."""
    import time
    ops, X, W1, wdw, W2, b2, se = _front_operands(gpu, 300, 300)
    L = trk.lib()
    W1p, W2p = ops.enc_pack_fragments(W1), ops.enc_pack_fragments(W2)
    ref = ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
    start = 0xFFFFFF00
    cnt = torch.tensor([start - (1 << 32)], dtype=torch.int32, device=gpu)
    u32 = lambda: int(cnt.item()) & 0xFFFFFFFF
    assert L.trk_set_tuning(b"rf3_chunks", chunks) == 0
    try:
        out = ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2, progress=cnt)
        ops.enc_rmb_front_means(X[: 37 * 100], W1p, wdw, W2p, b2, progress=cnt)
        torch.cuda.synchronize()
        assert u32() == (start + 337) & 0xFFFFFFFF == 81
        ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2)
        torch.cuda.synchronize()
        assert u32() == 81
    finally:
        L.trk_set_tuning(b"rf3_chunks", 1)
    assert all(torch.equal(a, b) for a, b in zip(out, ref))
    with pytest.raises(TypeError, match="progress"):
        ops.enc_rmb_front_means(X, W1p, wdw, W2p, b2, progress=cnt.to(torch.int64))
    side = torch.cuda.Stream(device=gpu)
    # targets as a caller computes them from the start: before the wrap, just past it (both
    # reached: open at once), and one ROI beyond the count (waits for its bound)
    for target, bound_us, slow in ((start + 200, 500000, False), ((start + 300) & 0xFFFFFFFF, 500000, False),
                                   ((start + 338) & 0xFFFFFFFF, 20000, True)):
        flag = torch.zeros(1, dtype=torch.int32, device=gpu)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(side):
            ops.stream_gate(cnt, target, bound_us)
            flag.fill_(1)  # queued behind the gate
        side.synchronize()
        dt = time.perf_counter() - t0
        assert flag.item() == 1
        assert (dt >= 0.015) if slow else (dt < 0.25), (target, dt)
    with pytest.raises(Exception):
        ops.stream_gate(cnt, 1, 2_000_000)  # the bound is capped at 1 s


def _partials(total, P, parts=3):
    """split int64 per-ROI totals [R, ld] into the GEMMs' partial layout
    [R, parts, ld] (one entry per 128-row tile covering the ROI; the rest junk)"""
    R, ld = total.shape
    out = torch.full((R, parts, ld), -(2 ** 40), dtype=torch.int64)  # never read
    g = torch.Generator().manual_seed(R)
    for r in range(R):
        cnt = (r * P + P - 1) // 128 - (r * P) // 128 + 1
        left = total[r].clone()
        for j in range(cnt - 1):
            x = torch.randint(-2 ** 30, 2 ** 30, (ld,), generator=g, dtype=torch.int64)
            out[r, j] = x
            left -= x
        out[r, cnt - 1] = left
    return out


@pytest.mark.parametrize("hw", [16, 8])
@pytest.mark.parametrize("R", [1, 37, 2048])
def test_enc_se_head_vs_torch_fp32(trk, gpu, R, hw):
    """trk_enc_se / trk_enc_head vs the same math in torch fp32 (the encoder's own
    _se / _head on the reference weights).  Means: bit-identical (same ops);
    s: 2e-6; embeddings (unit rows): 2e-5 -- the f32 MFMA sums in another order.
    R = 1 / 37: partial 16-ROI workgroups; 16- and 8-wave head workgroups."""
    L = trk.lib()
    assert L.trk_set_tuning(b"head_waves", hw) == 0
    try:
        _se_head_case(trk, gpu, R)
    finally:
        L.trk_set_tuning(b"head_waves", 16)


def _se_head_case(trk, gpu, R):
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    m = trk.Model(512, 512, 10, 128).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
    m = m.to(gpu)
    W = m._fused_weights(torch.bfloat16, gpu)
    g = torch.Generator().manual_seed(R)
    P = 100
    sums = (torch.randn(R, 1024, generator=g) * 40 * 2 ** 24).to(torch.int64)
    m_r, m_n, s = ops.enc_se(_partials(sums, P).to(gpu), P, W["se_w1"], W["se_b1"], W["se_w2"], W["se_b2"])
    f = (sums.double() * 2.0 ** -24).float().to(gpu)
    # correctly rounded f32 division by P (torch's GPU tensor / scalar multiplies by 1/P: <= 1 ulp apart)
    assert torch.allclose(m_r, f[:, :512] / P, rtol=1.2e-7, atol=0)
    assert torch.allclose(m_n, f[:, 512:] / P, rtol=1.2e-7, atol=0)
    with torch.no_grad():
        s_ref = m._se(m_r)
    assert (s - s_ref).abs().max().item() <= 2e-6
    tsums = (torch.randn(R, 512, generator=g) * 30 * 2 ** 24).to(torch.int64)
    tpart = _partials(tsums, P).to(gpu)
    assert torch.equal(ops.enc_sums_reduce(tpart, P), (tsums.double() * 2.0 ** -24).float().to(gpu))
    for a in (0.5, 0.3141592653589793):
        z = ops.enc_head(tpart, P, s, m_r, m_n, a, W["h0"], W["ln_w"], W["ln_b"], m.head.net[1].eps,
                         W["h4"], W["h4b"])
        m_cat = (tsums.double() * 2.0 ** -24).float().to(gpu) / P
        with torch.no_grad():
            z_ref = m._head(0.5 * m_cat + 0.5 * (a * (s * m_r) + (1 - a) * m_n))
        assert z.shape == (R, 128)
        assert (z - z_ref).abs().max().item() <= 2e-5, a
    # deterministic
    z2 = ops.enc_head(tpart, P, s, m_r, m_n, a, W["h0"], W["ln_w"], W["ln_b"], m.head.net[1].eps,
                      W["h4"], W["h4b"])
    assert torch.equal(z, z2)


def test_encoder_fused_tail_matches_torch_tail(trk, gpu):
    """bf16 encoder with the two tail kernels vs the same graph with the torch
    SE / mix / head ops: identical up to f32 summation order (2e-5)."""
    m = trk.Model(512, 512, 10, 128).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
    m = m.to(gpu)
    x = torch.from_numpy(G.encoder_input(5, 64, 10)).to(gpu).bfloat16().contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        z = m(x)
        try:
            m.fused_tail = False
            zt = m(x)
        finally:
            m.fused_tail = True
    assert (z - zt).abs().max().item() <= 2e-5


def test_encoder_deferred_head_on_another_stream(trk, gpu):
    """defer_head: the encoder returns the projection head unlaunched; launched on
    another stream (as the bench does, on the tracker's) it gives the same embeddings
    bit for bit, with the producing stream already running the next input."""
    m = trk.Model(512, 512, 10, 128).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()})
    m = m.to(gpu)
    x = torch.from_numpy(G.encoder_input(7, 64, 10)).to(gpu).bfloat16().contiguous(
        memory_format=torch.channels_last)
    other = torch.cuda.Stream(device=gpu)
    with torch.no_grad():
        z = m(x)
        try:
            m.defer_head = True
            dh = m(x)
            assert hasattr(dh, "launch")
            z_next = m(x.flip(0))  # the producing stream moves on
        finally:
            m.defer_head = False
        zd = dh.launch(other)
    other.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(z, zd)
    assert torch.equal(z_next.launch(torch.cuda.current_stream()), m(x.flip(0)))


# ----------------------------------------------------- encoder helpers ----
@pytest.mark.parametrize("S", [7, 10])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dwconv5_vs_torch_fp32(trk, gpu, S, dtype):
    """trk dwconv5 vs a plain PyTorch fp32 depthwise conv (tol: 2e-5 f32; bf16: output rounding)."""
    import torch.nn.functional as F
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(S)
    x = torch.randn(37, S, S, 1024, generator=g).to(gpu, dtype)
    w = (torch.randn(1024, 1, 5, 5, generator=g) / 5).to(gpu)
    got = ops.dwconv5_nhwc(x, w).float()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w, padding=2, groups=1024).permute(0, 2, 3, 1)
    tol = 2e-5 if dtype == torch.float32 else 1e-2
    assert (got - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())
    # the fast row-pair kernel and the generic kernel accumulate in the same order: identical
    L = trk.lib()
    try:
        L.trk_set_tuning(b"dw_fast", 0)
        gen = ops.dwconv5_nhwc(x, w).float()
    finally:
        L.trk_set_tuning(b"dw_fast", 1)
    assert torch.equal(got, gen)
    # ragged / odd shapes take the generic kernel (C % 128 != 0, non-square)
    x2 = torch.randn(5, 6, 9, 196, generator=g).to(gpu, dtype)
    w2 = (torch.randn(196, 1, 5, 5, generator=g) / 5).to(gpu)
    got2 = ops.dwconv5_nhwc(x2, w2).float()
    ref2 = F.conv2d(x2.float().permute(0, 3, 1, 2), w2, padding=2, groups=196).permute(0, 2, 3, 1)
    assert (got2 - ref2).abs().max().item() <= tol * max(1.0, ref2.abs().max().item())


@pytest.mark.parametrize("act", ["silu", "hardswish", None])
def test_act_mean_and_scale_rows(trk, gpu, act):
    import torch.nn.functional as F
    from importlib import import_module
    ops = import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(19, 100, 512, generator=g).to(gpu)
    fn = {"silu": F.silu, "hardswish": F.hardswish, None: lambda t: t}[act]
    ref = fn(x)
    y = x.clone()
    m = ops.act_mean(y, act)
    assert (y - ref).abs().max().item() <= 1e-6
    assert (m - ref.mean(1)).abs().max().item() <= 1e-5
    s = torch.rand(19, 512, generator=g).to(gpu)
    y0 = y.clone()
    ops.scale_rows(y, s)
    assert torch.equal(y, y0 * s[:, None, :])
    # fused act + scale == act (as act_mean writes it) then scale, bit for bit
    z = x.clone()
    ops.scale_rows(z, s, act=act)
    assert torch.equal(z, y)
    # mean without write-back leaves x untouched and equals the written mean
    x2 = x.clone()
    m2 = ops.act_mean(x2, act, write=False)
    assert torch.equal(x2, x) and torch.equal(m2, m)
    # a column block of a wider buffer (row stride 1024): only that block changes
    wide = torch.randn(19, 100, 1024, generator=g).to(gpu)
    wide[:, :, 256:768] = x
    w0 = wide.clone()
    blk = wide[:, :, 256:768]
    m3 = ops.act_mean(blk, act)
    assert torch.equal(m3, m) and torch.equal(blk, y0)
    ops.scale_rows(blk, s, act=None)
    assert torch.equal(blk, y) and torch.equal(wide[:, :, :256], w0[:, :, :256])
    assert torch.equal(wide[:, :, 768:], w0[:, :, 768:])


def test_lsap_prefix_shortcut_vs_oracle(trk, oracle, gpu):
    """The solver's exact shortcut (leading rows with a unique finite minimum in a
    column no earlier row's minimum took) against the oracle on matrices where
    the prefix is whole, cut by a duplicated minimum, by a tied row, by an
    all-gated row, on a tall (transposed) problem and in f64."""
    rng = np.random.default_rng(31)

    def perm_like(nr, nc, lo=0.05, hi=5.0):
        C = rng.uniform(1.0, hi, (nr, nc)).astype(np.float32)
        cols = rng.permutation(nc)[:nr]
        C[np.arange(nr), cols] = rng.uniform(0.0, lo, nr).astype(np.float32)
        return C, cols

    cases = []
    C, _ = perm_like(256, 256); cases.append(C)                        # whole prefix
    C, cols = perm_like(256, 256); C[100, cols[40]] = 0.0; cases.append(C)   # row 100 wants row 40's column
    C, cols = perm_like(256, 256); C[50, :] = 2.0; cases.append(C)           # tied row
    C, _ = perm_like(200, 256); C[7, :] = np.float32(1e9); cases.append(C)   # gated row early
    C, _ = perm_like(256, 300); C[255, :] = np.float32(1e9); cases.append(C)  # gated last row
    C, _ = perm_like(180, 256); cases.append(C.T.copy())                      # tall: transposed problem
    C = rng.integers(0, 4, (128, 128)).astype(np.float32); cases.append(C)    # tie-heavy: prefix of ~0
    for C in cases:
        for dt in (np.float32, np.float64):
            r, c = trk.linear_sum_assignment(C.astype(dt))
            er, ec = oracle.lsap(C)
            assert np.array_equal(r, er) and np.array_equal(c, ec), (C.shape, dt)
    # batched: frames with different prefixes in one launch
    F = len(cases[:5])
    buf = np.zeros((F, 256, 300), np.float32)
    for k, C in enumerate(cases[:5]):
        buf[k, :C.shape[0], :C.shape[1]] = C
    res = trk.lsap_batched(torch.from_numpy(buf).to(gpu), [C.shape[0] for C in cases[:5]],
                           [C.shape[1] for C in cases[:5]])
    for k, C in enumerate(cases[:5]):
        er, ec = oracle.lsap(C)
        n = int(res["count"][k])
        assert np.array_equal(res["rows"][k, :n].cpu().numpy(), er)
        assert np.array_equal(res["cols"][k, :n].cpu().numpy(), ec)
    # the cost gate (hungarian_assign, hung.py:35-40) on whole-prefix and cut matrices: a matrix
    # solved whole by the shortcut reads its gate values from the duals (u = the row minimum)
    for cmax in (0.03, 2.5):
        res = trk.lsap_batched(torch.from_numpy(buf).to(gpu), [C.shape[0] for C in cases[:5]],
                               [C.shape[1] for C in cases[:5]], cost_max=cmax)
        for k, C in enumerate(cases[:5]):
            er, ec = oracle.lsap(C)
            exp = np.full(C.shape[0], -1, np.int64)
            ok = C[er, ec].astype(np.float64) <= cmax
            exp[er[ok]] = ec[ok]
            assert np.array_equal(res["assign"][k, :C.shape[0]].cpu().numpy(), exp), (k, cmax)


def test_roi_align_a1_boundary_branches_gpu(trk, oracle, gpu):
    """The A.1 boundary branches on the GPU, bit-exact vs the oracle (which
    tests/test_oracle.py pins to the analytic values): the small-bin cases through the
    generic kernel, and 10x10 / 7x7 ROIs whose samples land exactly on y, x = -1 and
    y, x = H (W) through the row-sweep kernel (NHWC out, f32 and bf16) and NCHW out."""
    import test_oracle as TO
    x = TO._affine_map()
    for roi, PH, PW, aligned, what in TO.A1_BOUNDARY_ROIS:
        r = np.array([roi], np.float32)
        exp = oracle.roi_align(x, r, (PH, PW), 1.0, 2, aligned)
        got = trk.roi_align(torch.from_numpy(x).to(gpu), torch.from_numpy(r).to(gpu), (PH, PW), 1.0, 2, aligned)
        assert np.array_equal(got.cpu().numpy(), exp), what
    rng = np.random.default_rng(40)
    feat = rng.standard_normal((1, 512, 40, 40)).astype(np.float32)
    # bin height 0.5 cell: samples at sh + 0.125 + 0.25 k; sh = -1.125 puts k = 0 at y = -1,
    # sh = 35.125 puts k = 19 at y = 40 = H (and the same along x)
    rois = np.array([[0, -0.625, -0.625, 4.375, 4.375], [0, 35.625, 35.625, 40.625, 40.625],
                     [0, -0.625, 35.625, 4.375, 40.625], [0, 35.625, -0.625, 40.625, 4.375],
                     [0, 38.9, 38.7, 39.6, 39.95], [0, -1.6, -1.7, 0.2, 0.1]], np.float32)
    L = trk.lib()
    for S in (10, 7):
        exp = oracle.roi_align(feat, rois, (S, S), 1.0, 2, True)
        ft, rt = torch.from_numpy(feat).to(gpu), torch.from_numpy(rois).to(gpu)
        assert np.array_equal(trk.roi_align(ft, rt, (S, S), 1.0, 2, True).cpu().numpy(), exp), S
        for od in (torch.float32, torch.bfloat16):
            try:  # bf16 with the exact arithmetic (the fused default: test_roi_align_sweep_variants)
                assert L.trk_set_tuning(b"roi_fma", 0) == 0
                nhwc = trk.roi_align(ft, rt, (S, S), 1.0, 2, True, out_dtype=od, channels_last=True)
            finally:
                L.trk_set_tuning(b"roi_fma", 1)
            assert torch.equal(nhwc.float().cpu(), torch.from_numpy(exp).to(od).float()), (S, od)


def test_lsap_dev_vs_host_sizes(trk, gpu):
    """trk_lsap_dev (shapes in device memory, one bound for the batch, each matrix solved by
    the body its own width needs) vs trk_lsap (host shapes, the kernel sized by the widest
    matrix), with empty and out-of-bound matrices (status -4, assign -1 over the bound's
    rows).  Every output is bit-identical to the host-sized launch."""
    from importlib import import_module
    ops = import_module(trk.__name__ + ".ops")
    L = trk.lib()
    shapes = [(0, 5), (3, 0), (40, 60), (256, 256), (200, 300), (300, 260), (600, 700), (64, 1), (700, 600)]
    B = 720  # nr / nc bound (16 column slots: the bench's c3 bound class)
    rng = np.random.default_rng(11)
    F = len(shapes) + 1  # + one matrix outside the bound
    C = np.full((F, B + 8, B), 1e3, np.float32)
    for k, (r, c) in enumerate(shapes):
        C[k, :r, :c] = rng.uniform(0, 100, (r, c)).astype(np.float32)
    Cg = torch.from_numpy(C).to(gpu)
    nr = shapes + [(B + 8, 10)]
    kmax = B  # trk_lsap_dev: kmax >= min(nr, nc) bound
    ref = {"rows": torch.empty((F, kmax), dtype=torch.int64, device=gpu),
           "cols": torch.empty((F, kmax), dtype=torch.int64, device=gpu),
           "count": torch.empty((F,), dtype=torch.int32, device=gpu),
           "status": torch.empty((F,), dtype=torch.int32, device=gpu),
           "assign": torch.empty((F, B + 8), dtype=torch.int32, device=gpu)}
    trk.lsap_batched(Cg, [r for r, _ in shapes] + [0], [c for _, c in shapes] + [0], cost_max=50.0, out=ref)
    dnr = torch.tensor([r for r, _ in nr], dtype=torch.int32, device=gpu)
    dnc = torch.tensor([c for _, c in nr], dtype=torch.int32, device=gpu)
    out = {k: torch.full_like(v, -7) for k, v in ref.items()}
    rc = L.trk_lsap_dev(F, ops._ptr(Cg), ops._lib.TRK_F32, B, (B + 8) * B, ops._ptr(dnr), ops._ptr(dnc), B, B,
                        kmax, ops._ptr(out["rows"]), ops._ptr(out["cols"]), ops._ptr(out["count"]),
                        ops._ptr(out["status"]), ops._ptr(out["assign"]), B + 8, 50.0, ops._stream(gpu))
    assert rc == 0
    torch.cuda.synchronize()
    cnt = ref["count"].cpu().numpy()
    assert (out["status"][:-1].cpu() == ref["status"][:-1].cpu()).all() and int(out["status"][-1]) == -4
    assert int(out["count"][-1]) == 0 and (out["assign"][-1, :B].cpu() == -1).all()
    for k, (r, c) in enumerate(shapes):
        n = int(cnt[k])
        assert int(out["count"][k]) == n, k
        assert torch.equal(out["rows"][k, :n], ref["rows"][k, :n]) and torch.equal(out["cols"][k, :n], ref["cols"][k, :n]), k
        assert torch.equal(out["assign"][k, :r], ref["assign"][k, :r]), k
