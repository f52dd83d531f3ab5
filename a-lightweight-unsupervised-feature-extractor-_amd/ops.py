"""Torch-facing wrappers over the libtrk_amd C ABI.

Every function here launches the hand-written gfx950 kernels on the current
HIP stream of the input's device.  Host (CPU) tensors are rejected: there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib
from ._lib import CostParams, check, lib

__all__ = ["dwconv5_nhwc", "act_mean", "scale_rows", "roi_align", "nchw_to_nhwc", "roi_align_from_input_boxes", "build_cost", "cost_combine", "lsap_batched",
           "linear_sum_assignment", "CostParams", "default_cost_params"]


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(dev: torch.device):
    """the HIP stream handle of dev's current stream (what every launch goes on).
    torch.cuda.current_stream() builds a Stream object through the device-index
    helpers, ~3-7 us of host time per call on the hot path; the raw accessor is one
    C call"""
    idx = dev.index
    if _raw_stream is not None and idx is not None:
        return ctypes.c_void_p(_raw_stream(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def current_stream(dev: torch.device) -> torch.cuda.Stream:
    """torch.cuda.current_stream(dev), cached per raw handle (Event.record /
    record_stream need the Stream object)"""
    h = _stream(dev).value
    st = _streams.get((dev.index, h))
    if st is None:
        st = torch.cuda.current_stream(dev)
        _streams[(dev.index, h)] = st
    return st


_streams = {}


def _need_gpu(t: torch.Tensor, what: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise RuntimeError(f"{what}: expected a ROCm device tensor (this package has no CPU fallback)")


# -------------------------------------------------------- encoder helpers --
_ACT = {None: 0, "none": 0, "silu": 1, "hardswish": 2}


def _edt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.TRK_F32
    if t.dtype == torch.bfloat16:
        return _lib.TRK_BF16
    raise TypeError(f"expected float32 or bfloat16, got {t.dtype}")


def dwconv5_nhwc(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Depthwise 5x5 / pad 2 on NHWC storage x [N, H, W, C]; weight [C, 1, 5, 5]
    or already tap-major [25, C] f32 (card.DSC depth.1/point.1).  Returns
    [N, H, W, C] in x.dtype."""
    _need_gpu(x, "dwconv5_nhwc")
    N, H, W, C = x.shape
    x = x.contiguous()
    if weight.dim() == 2 and weight.shape == (25, C) and weight.dtype == torch.float32:
        w = weight.contiguous()
    else:
        w = weight.reshape(C, 25).to(torch.float32).t().contiguous()
    out = torch.empty_like(x)
    check(lib().trk_dwconv5_nhwc(_ptr(x), _ptr(w), _ptr(out), N, H, W, C, _edt(x), _stream(x.device)),
          "dwconv5_nhwc")
    return out


def _rows_view(x: torch.Tensor, name: str):
    """x [N, P, C] whose rows (dims 0-1 flattened) have unit channel stride and a
    common row stride ld >= C (a column block of a wider buffer is allowed)."""
    _need_gpu(x, name)
    if x.dim() != 3 or x.stride(2) != 1 or x.stride(0) != x.shape[1] * x.stride(1):
        raise ValueError(f"{name}: x must be [N, P, C] with unit channel stride and uniform row stride")
    return x.shape[0], x.shape[1], x.shape[2], x.stride(1)


def act_mean(x: torch.Tensor, act: Optional[str], *, inplace: bool = True,
             write: bool = True) -> torch.Tensor:
    """x [N, P, C] (row stride may exceed C): x <- act(x) (if write), returns
    mean over P (f32 [N, C])."""
    N, P, C, ld = _rows_view(x, "act_mean")
    mean = torch.empty((N, C), device=x.device, dtype=torch.float32)
    if write and not inplace:
        out = torch.empty_like(x.contiguous())
        if ld != C:
            raise ValueError("act_mean: a strided x needs inplace=True")
    else:
        out = x if write else None
    check(lib().trk_act_mean(_ptr(x), _ptr(out), _ptr(mean), N, P, C, ld, _ACT[act], _edt(x),
                             _stream(x.device)), "act_mean")
    return mean


def scale_rows(x: torch.Tensor, s: torch.Tensor, act: Optional[str] = None) -> torch.Tensor:
    """x [N, P, C] = act(x) * s[N, C] in place (act None: plain scale; row stride may exceed C)."""
    N, P, C, ld = _rows_view(x, "scale_rows")
    s = s.to(torch.float32).contiguous()
    if act is None and ld == C:
        check(lib().trk_scale_rows(_ptr(x), _ptr(s), N, P, C, _edt(x), _stream(x.device)), "scale_rows")
    else:
        check(lib().trk_act_scale_rows(_ptr(x), _ptr(s), N, P, C, ld, _ACT[act], _edt(x), _stream(x.device)),
              "act_scale_rows")
    return x


_FIX = 2.0 ** -24


def enc_g1_dwconv(X: torch.Tensor, W1: torch.Tensor, wdw: torch.Tensor) -> torch.Tensor:
    """bf16: dwconv5(X . W1^T) for 10x10 ROIs: X [R*100, 512] rows, W1 [N, 512],
    wdw tap-major [25, N] f32 -> Y2 [R*100, N] (the four first 1x1 convs of the RMB as one
    GEMM, Y1 rounded to bf16, then the 1024-channel depthwise 5x5)."""
    _need_gpu(X, "enc_g1_dwconv")
    if X.dtype != torch.bfloat16 or W1.dtype != torch.bfloat16:
        raise TypeError("enc_g1_dwconv: bf16 operands required")
    if X.dim() != 2 or not X.is_contiguous() or X.shape[1] != 512 or W1.shape[1] != 512:
        raise ValueError("enc_g1_dwconv: X must be contiguous [M, 512] and W1 [N, 512]")
    M = X.shape[0]
    N = W1.shape[0]
    if wdw.shape != (25, N) or wdw.dtype != torch.float32:
        raise ValueError("enc_g1_dwconv: wdw must be [25, N] f32")
    Y2 = torch.empty((M, N), device=X.device, dtype=torch.bfloat16)
    check(lib().trk_enc_g1_dwconv(_ptr(X), M, _ptr(W1.contiguous()), N, _ptr(wdw.contiguous()), _ptr(Y2),
                                  _stream(X.device)), "enc_g1_dwconv")
    return Y2


def enc_dsc_gemm(Y2: torch.Tensor, P: int, W2: torch.Tensor, bias: torch.Tensor, raw: bool = False):
    """Both DSC 1x1 GEMMs (bf16): Y2 [M, 2*Kg], W2 [2, Ng, Kg], bias [2*Ng] f32 ->
    (XRN [M, 2*Ng] = [SiLU(x_r) | Hardswish(x_n)], sum_silu_r [R, Ng] f32, sum_hsw_n [R, Ng] f32)
    with R = ceil(M / P) ROIs (sums over each ROI's P rows).  raw=True returns
    (XRN, sums [R, 2*Ng] int64 fixed point x 2^24) for enc_se."""
    _need_gpu(Y2, "enc_dsc_gemm")
    if Y2.dtype != torch.bfloat16 or W2.dtype != torch.bfloat16:
        raise TypeError("enc_dsc_gemm: bf16 operands required")
    M, K2 = Y2.shape
    G, Ng, Kg = W2.shape
    if G != 2 or K2 != 2 * Kg or bias.numel() != 2 * Ng:
        raise ValueError("enc_dsc_gemm: shape mismatch")
    Y2, W2, bias = Y2.contiguous(), W2.contiguous(), bias.to(torch.float32).contiguous()
    R = (M + P - 1) // P
    XRN = torch.empty((M, 2 * Ng), device=Y2.device, dtype=torch.bfloat16)
    sums = torch.empty((R, _lib.TRK_ENC_PARTS, 2 * Ng), device=Y2.device, dtype=torch.int64)  # partials
    check(lib().trk_enc_dsc_gemm(_ptr(Y2), M, P, Kg, _ptr(W2), _ptr(bias), Ng, _ptr(XRN), _ptr(sums),
                                 _stream(Y2.device)), "enc_dsc_gemm")
    if raw:
        return XRN, sums
    f = enc_sums_reduce(sums, P)
    return XRN, f[:, :Ng], f[:, Ng:]


def enc_pack_fragments_k(W: torch.Tensor) -> torch.Tensor:
    """[N, K] bf16 weights -> the 16x16x32 MFMA A-fragment order the trans4 transition reads:
    [K/32 k steps][N/16 col tiles][64 lanes][8], element (s, n, l, j) =
    W[16n + l%16][32s + 8(l//16) + j]."""
    N, K = W.shape
    W = W.reshape(N // 16, 16, K // 32, 4, 8)                 # n, fr, s, fc, j
    return W.permute(2, 0, 3, 1, 4).contiguous()               # s, n, fc, fr, j  (lane = 16 fc + fr)


def enc_pack_fragments(W: torch.Tensor) -> torch.Tensor:
    """[2*512, 512] (or [2, 512, 512]) bf16 weights [N][K] -> the 16x16x32 MFMA
    fragment order trk_enc_rmb_front_means reads: [2][16 k steps][32 col tiles][64 lanes][8],
    element (g, s, n, l, j) = W[g*512 + 16n + l%16][32s + 8(l//16) + j]."""
    W = W.reshape(2, 32, 16, 16, 4, 8)                 # g, n, fr, s, fc, j
    return W.permute(0, 3, 1, 4, 2, 5).contiguous()    # g, s, n, fc, fr, j  (lane = 16 fc + fr)


def enc_transition_gemm(XRN: torch.Tensor, P: int, s: torch.Tensor, Wt: torch.Tensor,
                        bias: torch.Tensor, raw: bool = False, Wtp: torch.Tensor = None) -> torch.Tensor:
    """sum over each ROI's P rows of SiLU([x_f * s | x_n] . Wt^T + bias):
    XRN [M, K] bf16 (x_f = first kscale = s.shape[1] columns), s [R, kscale]
    f32, Wt [N, K] bf16 -> [R, N] f32 (raw=True: the int64 x 2^24 sums, for enc_head).
    Wtp: optionally Wt as enc_pack_fragments_k(Wt), which the trans4 kernel
    (set_tuning("enc_trans", 1)) reads straight into registers; same bits either way."""
    _need_gpu(XRN, "enc_transition_gemm")
    if XRN.dtype != torch.bfloat16 or Wt.dtype != torch.bfloat16:
        raise TypeError("enc_transition_gemm: bf16 operands required")
    M, K = XRN.shape
    N, K2 = Wt.shape
    R = (M + P - 1) // P
    if K2 != K or s.shape[0] != R or bias.numel() != N:
        raise ValueError("enc_transition_gemm: shape mismatch")
    if Wtp is not None and (Wtp.dtype != torch.bfloat16 or not Wtp.is_contiguous() or
                            tuple(Wtp.shape) != (K // 32, N // 16, 4, 16, 8) or (N, K) != (512, 1024)):
        raise ValueError("enc_transition_gemm: Wtp must be enc_pack_fragments_k(Wt) of a [512, 1024] Wt")
    XRN, Wt = XRN.contiguous(), Wt.contiguous()
    s, bias = s.to(torch.float32).contiguous(), bias.to(torch.float32).contiguous()
    sums = torch.empty((R, _lib.TRK_ENC_PARTS, N), device=XRN.device, dtype=torch.int64)  # partials
    check(lib().trk_enc_transition_gemm2(_ptr(XRN), M, P, K, _ptr(s), s.shape[1], _ptr(Wt),
                                         _ptr(Wtp) if Wtp is not None else None, _ptr(bias), N,
                                         _ptr(sums), _stream(XRN.device)), "enc_transition_gemm")
    if raw:
        return sums
    return enc_sums_reduce(sums, P)


def enc_sums_reduce(part: torch.Tensor, P: int) -> torch.Tensor:
    """Total per-ROI sums from the GEMMs' int64 partials [R, TRK_ENC_PARTS, ld]
    (one per 128-row tile covering the ROI): [R, ld] f32 = (sum * 2^-24)."""
    _need_gpu(part, "enc_sums_reduce")
    if part.dtype != torch.int64 or part.dim() != 3 or part.shape[1] != _lib.TRK_ENC_PARTS:
        raise TypeError("enc_sums_reduce: part must be [R, TRK_ENC_PARTS, ld] int64")
    part = part.contiguous()
    R, _, ld = part.shape
    out = torch.empty((R, ld), device=part.device, dtype=torch.float32)
    check(lib().trk_enc_sums_reduce(_ptr(part), R, P, ld, _ptr(out), _stream(part.device)), "enc_sums_reduce")
    return out


def enc_rmb_front_means(X: torch.Tensor, W1p: torch.Tensor, wdw: torch.Tensor, W2p: torch.Tensor,
                        bias: torch.Tensor, progress: Optional[torch.Tensor] = None):
    """bf16, 10x10 ROIs of 512 channels: enc_g1_dwconv + enc_dsc_gemm in one kernel
    (trk_enc_rmb_front_means; Y2 stays in LDS).  X [R*100, 512], W1p / W2p from
    enc_pack_fragments, wdw [25, 1024] f32, bias [1024] f32 -> (XRN [R*100, 1024], m_r, m_n
    [R, 512] f32): XRN bit-identical to the two-kernel path, m_r / m_n the squeeze means
    enc_se takes (of the kernel's own f32 column sums).  progress: None, or a one-element
    int32 tensor on X's device that the launch advances by one per finished ROI (the count a
    stream_gate on another stream waits for; it wraps at 2^32)."""
    _need_gpu(X, "enc_rmb_front_means")
    if X.dtype != torch.bfloat16 or W1p.dtype != torch.bfloat16 or W2p.dtype != torch.bfloat16:
        raise TypeError("enc_rmb_front_means: bf16 operands required")
    if X.dim() != 2 or not X.is_contiguous() or X.shape[1] != 512 or X.shape[0] % 100:
        raise ValueError("enc_rmb_front_means: X must be contiguous [R*100, 512]")
    pk = (2, 16, 32, 4, 16, 8)
    if tuple(W1p.shape) != pk or tuple(W2p.shape) != pk or not (W1p.is_contiguous() and W2p.is_contiguous()):
        raise ValueError("enc_rmb_front_means: W1p / W2p must be enc_pack_fragments output [2, 16, 32, 4, 16, 8]")
    if wdw.shape != (25, 1024) or wdw.dtype != torch.float32 or bias.numel() != 1024:
        raise ValueError("enc_rmb_front_means: wdw [25, 1024] f32 and bias [1024] required")
    if progress is not None and (progress.dtype != torch.int32 or progress.numel() < 1 or
                                 progress.device != X.device):
        raise TypeError("enc_rmb_front_means: progress must be a one-element int32 tensor on X's device")
    M = X.shape[0]
    XRN = torch.empty((M, 1024), device=X.device, dtype=torch.bfloat16)
    m = torch.empty((2, M // 100, 512), device=X.device, dtype=torch.float32)
    check(lib().trk_enc_rmb_front_means(_ptr(X), M, _ptr(W1p), _ptr(wdw.contiguous()), _ptr(W2p),
                                        _ptr(bias.to(torch.float32).contiguous()), _ptr(XRN), _ptr(m[0]), _ptr(m[1]),
                                        _ptr(progress), _stream(X.device)), "enc_rmb_front_means")
    return XRN, m[0], m[1]


def stream_gate(counter: torch.Tensor, target: int, max_us: int = 2000) -> None:
    """Enqueue on the current stream a one-wave kernel that returns once the wrapping u32 count
    counter[0] has reached target ((int32)(count - target) >= 0: a target within 2^31 of the
    count; the `progress` counter of enc_rmb_front_means launches on another stream) or after
    max_us: the work queued behind it starts then (trk_stream_gate; a scheduling hint, not an
    ordering)."""
    _need_gpu(counter, "stream_gate")
    if counter.dtype != torch.int32:
        raise TypeError("stream_gate: int32 counter required")
    check(lib().trk_stream_gate(_ptr(counter), ctypes.c_uint32(int(target) & 0xFFFFFFFF), int(max_us),
                                _stream(counter.device)), "stream_gate")


def enc_pack_rows(w: torch.Tensor) -> torch.Tensor:
    """[N, K] f32 weight -> [N/16, K/16, 64, 4], the fragment order the SE / head kernels read
    (rb_linear.h): lane 16 g + r of (column tile t, K block kb) holds W[16 t + r][16 kb + 4 g .. + 3]."""
    if w.dim() != 2 or w.shape[0] % 16 or w.shape[1] % 16:
        raise ValueError("enc_pack_rows: [N, K] with N, K multiples of 16 required")
    N, K = w.shape
    return (_f32c(w).reshape(N // 16, 16, K // 16, 4, 4).permute(0, 2, 3, 1, 4).contiguous()
            .reshape(N // 16, K // 16, 64, 4))


def _rows_packed(w: torch.Tensor, what: str):
    """(packed weight, N, K) from an [N, K] weight (packed here) or an enc_pack_rows result"""
    if w.dim() == 2:
        return enc_pack_rows(w), w.shape[0], w.shape[1]
    if w.dim() == 4 and tuple(w.shape[2:]) == (64, 4) and w.dtype == torch.float32 and w.is_contiguous():
        return w, w.shape[0] * 16, w.shape[1] * 16
    raise ValueError(f"{what}: weights must be [N, K] f32 or enc_pack_rows output [N/16, K/16, 64, 4]")


def enc_se_means(m_r: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor):
    """SE excitation from given squeeze means (trk_enc_se_means): s [R, C] f32, bit-identical
    to enc_se's s for the same m_r (card.py:59-78)."""
    _need_gpu(m_r, "enc_se_means")
    if m_r.dtype != torch.float32 or m_r.dim() != 2:
        raise TypeError("enc_se_means: m_r must be [R, C] f32")
    w1, H, C = _rows_packed(w1, "enc_se_means")
    w2, C2, H2 = _rows_packed(w2, "enc_se_means")
    R = m_r.shape[0]
    if m_r.shape[1] != C or (C2, H2) != (C, H) or b1.numel() != H or b2.numel() != C:
        raise ValueError("enc_se_means: shape mismatch")
    m_r = m_r.contiguous()
    s = torch.empty((R, C), device=m_r.device, dtype=torch.float32)
    b1, b2 = _f32c(b1), _f32c(b2)
    check(lib().trk_enc_se_means(_ptr(m_r), R, C, _ptr(w1), _ptr(b1), H, _ptr(w2), _ptr(b2), _ptr(s),
                                 _stream(m_r.device)), "enc_se_means")
    return s


def _f32c(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous()


def enc_se(sums: torch.Tensor, P: int, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
           b2: torch.Tensor):
    """SE squeeze + excitation from enc_dsc_gemm's raw partial sums
    [R, TRK_ENC_PARTS, 2C] int64: returns (m_r, m_n, s) [R, C] f32 with
    m = (float)(sum * 2^-24) / P and s = hardsigmoid(w2 . relu(w1 . m_r + b1) + b2)
    (card.py:59-78)."""
    _need_gpu(sums, "enc_se")
    if sums.dtype != torch.int64 or sums.dim() != 3 or sums.shape[1] != _lib.TRK_ENC_PARTS:
        raise TypeError("enc_se: sums must be [R, TRK_ENC_PARTS, 2C] int64 partials")
    w1, H, C = _rows_packed(w1, "enc_se")
    w2, C2, H2 = _rows_packed(w2, "enc_se")
    R = sums.shape[0]
    if sums.shape[2] < 2 * C or (C2, H2) != (C, H) or b1.numel() != H or b2.numel() != C:
        raise ValueError("enc_se: shape mismatch")
    sums = sums.contiguous()
    out = torch.empty((3, R, C), device=sums.device, dtype=torch.float32)
    b1, b2 = _f32c(b1), _f32c(b2)
    check(lib().trk_enc_se(_ptr(sums), R, sums.stride(1), P, C, _ptr(w1), _ptr(b1), H, _ptr(w2), _ptr(b2),
                           _ptr(out[0]), _ptr(out[1]), _ptr(out[2]), _stream(sums.device)), "enc_se")
    return out[0], out[1], out[2]


def enc_head(tsums: torch.Tensor, P: int, s: torch.Tensor, m_r: torch.Tensor, m_n: torch.Tensor, alpha: float,
             w0: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, ln_eps: float, w4: torch.Tensor,
             b4: torch.Tensor) -> torch.Tensor:
    """Shake2 eval mix + ProjectionHead from enc_transition_gemm's raw partial
    sums [R, TRK_ENC_PARTS, C] int64 (card.py:83-96, :151-169): [R, D] f32 unit rows."""
    _need_gpu(tsums, "enc_head")
    if tsums.dtype != torch.int64 or tsums.dim() != 3 or tsums.shape[1] != _lib.TRK_ENC_PARTS:
        raise TypeError("enc_head: tsums must be [R, TRK_ENC_PARTS, C] int64 partials")
    R, _, C = tsums.shape
    w0, N0, K0 = _rows_packed(w0, "enc_head")
    w4, D, K4 = _rows_packed(w4, "enc_head")
    if (s.shape != (R, C) or m_r.shape != (R, C) or m_n.shape != (R, C) or (N0, K0) != (C, C) or
            K4 != C or b4.numel() != D or ln_w.numel() != C or ln_b.numel() != C):
        raise ValueError("enc_head: shape mismatch")
    out = torch.empty((R, D), device=tsums.device, dtype=torch.float32)
    tsums, s, m_r, m_n = tsums.contiguous(), _f32c(s), _f32c(m_r), _f32c(m_n)
    ln_w, ln_b, b4 = _f32c(ln_w), _f32c(ln_b), _f32c(b4)
    check(lib().trk_enc_head(_ptr(tsums), R, P, C, _ptr(s), _ptr(m_r), _ptr(m_n), float(alpha), _ptr(w0),
                             _ptr(ln_w), _ptr(ln_b), float(ln_eps), _ptr(w4), _ptr(b4), D, _ptr(out),
                             _stream(tsums.device)), "enc_head")
    return out


# ------------------------------------------------------------- ROI Align --
def _rois_tensor(boxes, device, dtype) -> torch.Tensor:
    if isinstance(boxes, torch.Tensor):
        if boxes.dim() != 2 or boxes.size(1) != 5:
            raise ValueError("boxes must be a Tensor[K, 5] or a list of Tensor[L, 4]")
        return boxes.to(device=device, dtype=dtype).contiguous()
    parts = []
    for b, bb in enumerate(boxes):
        bb = torch.as_tensor(bb, device=device, dtype=dtype).reshape(-1, 4)
        parts.append(torch.cat([torch.full((bb.size(0), 1), float(b), device=device, dtype=dtype), bb], 1))
    if not parts:
        return torch.zeros((0, 5), device=device, dtype=dtype)
    return torch.cat(parts, 0).contiguous()


def roi_align(input: torch.Tensor, boxes: Union[torch.Tensor, List[torch.Tensor]],
              output_size, spatial_scale: float = 1.0, sampling_ratio: int = -1,
              aligned: bool = False, *, out_dtype: Optional[torch.dtype] = None,
              channels_last: bool = False) -> torch.Tensor:
    """``torchvision.ops.roi_align`` on gfx950 (drop-in for the call at reference
    tracking.py:214-221).  Returns [K, C, PH, PW]; with ``channels_last=True`` the
    same logical tensor is stored NHWC (the encoder's GEMM layout).  An input
    already in channels_last memory format skips the per-call NCHW->NHWC copy."""
    _need_gpu(input, "roi_align")
    if input.dim() != 4:
        raise ValueError(f"roi_align: expected input of shape [B, C, H, W], got {tuple(input.shape)}")
    PH, PW = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
    if sampling_ratio <= 0:
        raise NotImplementedError("roi_align: adaptive sampling (sampling_ratio <= 0) is not "
                                  "implemented; the reference always passes sampling_ratio=2")
    in_dtype = input.dtype
    if out_dtype is None:
        out_dtype = in_dtype
    x = input if input.dtype == torch.float32 else input.float()  # fp16/bf16 -> f32 is exact
    rois = _rois_tensor(boxes, x.device, torch.float32)
    B, C, H, W = x.shape
    K = rois.size(0)
    if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        in_layout, src = _lib.TRK_NHWC, x
    else:
        in_layout, src = _lib.TRK_NCHW, x.contiguous()
    kdt = _lib.TRK_BF16 if out_dtype == torch.bfloat16 else _lib.TRK_F32
    tdt = torch.bfloat16 if kdt == _lib.TRK_BF16 else torch.float32
    if channels_last:
        out = torch.empty((K, PH, PW, C), device=x.device, dtype=tdt).permute(0, 3, 1, 2)
    else:
        out = torch.empty((K, C, PH, PW), device=x.device, dtype=tdt)
    if K == 0:
        return out.to(out_dtype)
    ws_bytes = lib().trk_roi_align_workspace_bytes(B, C, H, W, in_layout)
    ws = torch.empty(max(ws_bytes, 1), device=x.device, dtype=torch.uint8) if ws_bytes else None
    rc = lib().trk_roi_align_fwd(_ptr(src), B, C, H, W, in_layout, _ptr(rois), K,
                                 float(spatial_scale), PH, PW, int(sampling_ratio), int(bool(aligned)),
                                 _ptr(out), kdt, _lib.TRK_NHWC if channels_last else _lib.TRK_NCHW,
                                 _ptr(ws), ws_bytes, _stream(x.device))
    check(rc, "roi_align")
    return out if out.dtype == out_dtype else out.to(out_dtype)


def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    """An f32 [B, C, H, W] map in channels_last storage (a [B, H, W, C] copy), by the
    same kernel roi_align uses for NCHW input: passing the result to roi_align skips
    that copy, so a caller can convert a frame's map ahead of its ROI Align."""
    _need_gpu(x, "nchw_to_nhwc")
    if x.dim() != 4 or x.dtype != torch.float32:
        raise ValueError("nchw_to_nhwc: expected an f32 [B, C, H, W] tensor")
    x = x.contiguous()
    B, C, H, W = x.shape
    out = torch.empty((B, H, W, C), device=x.device, dtype=torch.float32)
    check(lib().trk_nchw_to_nhwc(_ptr(x), B, C, H, W, _ptr(out), _stream(x.device)), "nchw_to_nhwc")
    return out.permute(0, 3, 1, 2)


def roi_align_from_input_boxes(feat: torch.Tensor, boxes_in: Sequence[Sequence[float]],
                               input_hw: Tuple[int, int], out_size=(7, 7), aligned: bool = True,
                               sampling_ratio: int = 2, **kw) -> torch.Tensor:
    """MainInfer.roi_align_from_input_boxes (reference tracking.py:193-221):
    rois = [[0, x1, y1, x2, y2]] cast to feat.dtype, spatial_scale = Hf / H_in."""
    H_in, W_in = input_hw
    _, _, Hf, Wf = feat.shape
    spatial_scale = Hf / float(H_in)
    rois = torch.tensor([[0.0, b[0], b[1], b[2], b[3]] for b in boxes_in], dtype=feat.dtype,
                        device=feat.device).reshape(-1, 5)
    return roi_align(feat, rois, out_size, spatial_scale=spatial_scale,
                     sampling_ratio=sampling_ratio, aligned=aligned, **kw)


# ------------------------------------------------------------------ cost --
def default_cost_params(conf: Optional[dict] = None, *, gate: bool = True) -> CostParams:
    """Constants of conf.yaml's tracker section (reference model/conf/conf.yaml:3-24)."""
    c = conf or {}
    return CostParams(float(c.get("w_app", 1.0)), float(c.get("w_bbox", 0.3)),
                      float(c.get("w_conf", 0.2)), float(c.get("alpha", 1.0)),
                      float(c.get("beta", 0.5)), float(c.get("maha_thr", 9.49)), 1e9,
                      int(c.get("emb_top_k", 5)), 1 if gate else 0)


def build_cost(*, M: Sequence[int], N: Sequence[int], bank: torch.Tensor, bank_len: torch.Tensor,
               pbox: torch.Tensor, conf_prev: torch.Tensor, det_emb: torch.Tensor,
               dbox: torch.Tensor, conf_cur: torch.Tensor, params: CostParams,
               gmean: Optional[torch.Tensor] = None, gsinv: Optional[torch.Tensor] = None,
               gate_on: Optional[torch.Tensor] = None, row_slot: Optional[torch.Tensor] = None,
               out: Optional[dict] = None, want=("C_total",)) -> dict:
    """Batched fused cost.  Shapes: det_emb [F, Nmax, 128], dbox [F, Nmax, 4],
    conf_cur [F, Nmax]; track arrays indexed by slot (bank [S, Tmax, 128] ...),
    rows mapped through row_slot [F, Mmax] if given, else slot = f*Mmax + i.
    Returns {name: [F, Mmax, Nmax] f32}.  C_total / C_app only: the bank-resident
    kernel (trk_build_cost_dev with a workspace); any of C_center / C_scale /
    C_conf: the det-tile kernel (trk_build_cost).  Bit-identical outputs."""
    _need_gpu(det_emb, "build_cost")
    F, Nmax, D = det_emb.shape
    if D != 128:
        raise ValueError(f"det_embs must be 128D, got {D}")
    Mmax = row_slot.shape[1] if row_slot is not None else bank.shape[0] // max(F, 1)
    Tmax = bank.shape[1]
    dev = det_emb.device
    if out is None:
        out = {k: torch.empty((F, Mmax, Nmax), device=dev, dtype=torch.float32) for k in want}
    if set(out) <= {"C_total", "C_app"} and F > 0 and Mmax > 0 and Nmax > 0:
        Mi, Ni = [int(m) for m in M], [int(n) for n in N]
        if len(Mi) != F or len(Ni) != F or any(not 0 <= m <= Mmax for m in Mi) or any(not 0 <= n <= Nmax for n in Ni):
            raise ValueError("build_cost: frame M/N outside [0, Mmax/Nmax]")
        if row_slot is None:
            row_slot = torch.arange(F * Mmax, device=dev, dtype=torch.int32).view(F, Mmax)
        dM = torch.tensor(Mi, dtype=torch.int32).to(dev, non_blocking=True)
        dN = torch.tensor(Ni, dtype=torch.int32).to(dev, non_blocking=True)
        work = torch.empty(int(lib().trk_cost_work_bytes(F, Nmax)), device=dev, dtype=torch.uint8)
        rc = lib().trk_build_cost_dev(F, Mmax, Nmax, _ptr(dM), _ptr(dN), _ptr(row_slot), row_slot.shape[1], Tmax,
                                      _ptr(bank), _ptr(bank_len), _ptr(pbox), _ptr(conf_prev), _ptr(gmean),
                                      _ptr(gsinv), _ptr(gate_on), _ptr(det_emb), _ptr(dbox), _ptr(conf_cur),
                                      ctypes.byref(params), _ptr(out.get("C_total")), _ptr(out.get("C_app")),
                                      _ptr(work), _stream(dev))
        check(rc, "build_cost")
        return out
    hM = (ctypes.c_int32 * max(F, 1))(*[int(m) for m in M])
    hN = (ctypes.c_int32 * max(F, 1))(*[int(n) for n in N])
    rc = lib().trk_build_cost(F, Mmax, Nmax, hM, hN, _ptr(row_slot), Tmax, _ptr(bank), _ptr(bank_len),
                              _ptr(pbox), _ptr(conf_prev), _ptr(gmean), _ptr(gsinv), _ptr(gate_on),
                              _ptr(det_emb), _ptr(dbox), _ptr(conf_cur), ctypes.byref(params),
                              _ptr(out.get("C_total")), _ptr(out.get("C_app")), _ptr(out.get("C_center")),
                              _ptr(out.get("C_scale")), _ptr(out.get("C_conf")), _stream(dev))
    check(rc, "build_cost")
    return out


def cost_combine(C_app: torch.Tensor, pbox: torch.Tensor, conf_prev: torch.Tensor,
                 dbox: torch.Tensor, conf_cur: torch.Tensor, params: CostParams,
                 gmean=None, gsinv=None, gate_on=None) -> dict:
    """costCard.cal_cost combine given C_app (trk_cost_combine)."""
    _need_gpu(C_app, "cost_combine")
    M, N = C_app.shape
    dev = C_app.device
    out = {k: torch.empty((M, N), device=dev, dtype=torch.float32)
           for k in ("C_total", "C_center", "C_scale", "C_conf")}
    rc = lib().trk_cost_combine(M, N, _ptr(C_app.contiguous()), _ptr(pbox), _ptr(conf_prev), _ptr(dbox),
                                _ptr(conf_cur), _ptr(gmean), _ptr(gsinv), _ptr(gate_on),
                                ctypes.byref(params), _ptr(out["C_total"]), _ptr(out["C_center"]),
                                _ptr(out["C_scale"]), _ptr(out["C_conf"]), _stream(dev))
    check(rc, "cost_combine")
    return out


# ------------------------------------------------------------------ LSAP --
def lsap_batched(C: torch.Tensor, nr: Sequence[int], nc: Sequence[int], *,
                 cost_max: Optional[float] = None, out: Optional[dict] = None) -> dict:
    """Batched scipy-exact LSAP (trk_lsap).  C: [F, R, ld] f32/f64 device tensor
    (matrix f = C[f, :nr[f], :nc[f]]).  Returns device tensors rows/cols [F, kmax]
    int64, count/status [F] int32 and, if cost_max is given, assign [F, R] int32
    (matched column or -1 after hungarian_assign's cost gate, hung.py:35-40)."""
    _need_gpu(C, "lsap")
    if C.dim() != 3:
        raise ValueError("lsap_batched expects C of shape [F, R, ld]")
    if C.dtype not in (torch.float32, torch.float64):
        C = C.double()
    C = C.contiguous()
    F, R, ld = C.shape
    kmax = max(1, max((min(a, b) for a, b in zip(nr, nc)), default=1))
    dev = C.device
    if out is None:
        out = {"rows": torch.empty((F, kmax), device=dev, dtype=torch.int64),
               "cols": torch.empty((F, kmax), device=dev, dtype=torch.int64),
               "count": torch.empty((F,), device=dev, dtype=torch.int32),
               "status": torch.empty((F,), device=dev, dtype=torch.int32)}
        if cost_max is not None:
            out["assign"] = torch.empty((F, R), device=dev, dtype=torch.int32)
    kmax = out["rows"].shape[1]
    hr = (ctypes.c_int32 * max(F, 1))(*[int(x) for x in nr])
    hc = (ctypes.c_int32 * max(F, 1))(*[int(x) for x in nc])
    dt = _lib.TRK_F32 if C.dtype == torch.float32 else _lib.TRK_F64
    assign = out.get("assign")
    rc = lib().trk_lsap(F, _ptr(C), dt, ld, R * ld, hr, hc, kmax, _ptr(out["rows"]), _ptr(out["cols"]),
                        _ptr(out["count"]), _ptr(out["status"]), _ptr(assign),
                        R if assign is not None else 0,
                        float(cost_max) if cost_max is not None else 0.0, _stream(dev))
    check(rc, "lsap")
    return out


def lsap_check_status(status: int, what: str = "lsap"):
    """Raise like scipy for a trk_lsap status (-1 invalid entries, -2 infeasible);
    -3 (internal solver stall) and -4 (launch bound) are library errors."""
    if status == 0:
        return
    if status == -1:
        raise ValueError("matrix contains invalid numeric entries")
    if status == -2:
        raise ValueError("cost matrix is infeasible")
    if status == -3:
        raise _lib.TrkError(f"{what}: the solver stalled (a bounded wait expired); the result is not valid")
    raise _lib.TrkError(f"{what}: failed with status {status}")


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("linear_sum_assignment: no ROCm device (this package has no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def linear_sum_assignment(cost_matrix, maximize: bool = False):
    """scipy.optimize.linear_sum_assignment drop-in (reference hung.py:28),
    solved on the GPU; returns host int64 (row_ind, col_ind) like scipy."""
    if isinstance(cost_matrix, torch.Tensor):
        t = cost_matrix
        if t.dim() != 2:
            raise ValueError("expected a matrix (2-D array), got a %r array" % (tuple(t.shape),))
    else:
        a = np.asarray(cost_matrix)
        if a.ndim != 2:
            raise ValueError("expected a matrix (2-D array), got a %r array" % (a.shape,))
        if a.dtype == np.bool_:
            a = a.astype(np.float64)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if maximize:
        t = -t.double()
    nr, nc = t.shape
    if nr == 0 or nc == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    t = t.to(_device(), non_blocking=False)
    res = lsap_batched(t.reshape(1, nr, nc), [nr], [nc])
    status = int(res["status"][0].item())
    lsap_check_status(status)
    k = int(res["count"][0].item())
    return res["rows"][0, :k].cpu().numpy(), res["cols"][0, :k].cpu().numpy()
