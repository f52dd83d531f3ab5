"""The lightweight ROI encoder -- drop-in for reference
model/utils/modules/encoderAndHead.py:11-26 (Model) built from card.py's RMB +
ProjectionHead.

The module tree reproduces the reference's 35 state_dict keys so a reference
checkpoint ``ckpt["model"]`` loads with ``strict=True`` (tracking.py:180-182).
The forward is a re-derivation of the eval graph for MI355X,
not a module-by-module replay:

  * the four first 1x1 convs (depth/point x reinforce/normal) read the same
    input, so they are ONE GEMM  [N*S*S, 512] x [512, 1024] on NHWC rows;
  * the four depthwise 5x5 convs are one 1024-group depthwise conv;
  * each DSC's ``depth.2(d) + point.2(p)`` is one GEMM over the concatenated
    [d | p] columns with eval-BN folded into its weights and bias;
  * only the spatial mean of the RMB output feeds the head, so the shake/fuse
    blend and the GAP are applied to per-ROI means:
        mean(0.5*x_cat + 0.5*(0.5*x_f*s + 0.5*x_n))
      = 0.5*mean(SiLU(T)) + 0.25*s*mean(x_f) + 0.25*mean(x_n)
    and the SE scale s is applied to the transition GEMM's input rows.
Input: [N, 512, S, S] ROI features in any memory format; channels_last
(what trk roi_align writes with channels_last=True) makes the first GEMM's
operand a zero-copy view.  Compute dtype = input dtype (fp32 for parity,
bf16 for throughput; fp16 -- the reference's model.half() configuration --
runs the fp32 path on the widened values); reductions, SE and the head run
in fp32.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class DSC(nn.Module):
    """Parameter container matching card.DSC (card.py:8-46)."""

    def __init__(self, in_channels, out_channels, kernel_size=5):
        super().__init__()
        hidden = in_channels // 2

        def branch():
            return nn.Sequential(
                nn.Conv2d(in_channels, hidden, 1, bias=False),
                nn.Conv2d(hidden, hidden, kernel_size, padding=kernel_size // 2, groups=hidden, bias=False),
                nn.Conv2d(hidden, out_channels, 1, bias=False))

        self.depth = branch()
        self.point = branch()
        self.bn = nn.BatchNorm2d(out_channels)


class SEBlock(nn.Module):
    """card.SEBlock (card.py:59-78) parameters."""

    def __init__(self, in_channels, reduction=4):
        super().__init__()
        hid = in_channels // reduction
        self.excitation = nn.Sequential(nn.Linear(in_channels, hid), nn.ReLU(),
                                        nn.Linear(hid, in_channels), nn.Hardsigmoid())


class RMB(nn.Module):
    """card.RMB (card.py:105-148) parameters; warmup/epoch semantics kept."""

    def __init__(self, in_channels, out_channels, stride=1, warmup_epochs=0):
        super().__init__()
        if stride != 1:
            raise NotImplementedError("RMB stride != 1 is not used by the reference")
        self.warmup_epochs = warmup_epochs
        self.current_epoch = 0
        self.dsc_reinforce = DSC(in_channels, out_channels)
        self.dsc_normal = DSC(in_channels, out_channels)
        self.se = SEBlock(out_channels)
        self.transition = nn.Sequential(nn.Conv2d(2 * out_channels, out_channels, 1), nn.SiLU())

    def set_epoch(self, epoch: int):
        self.current_epoch = epoch


class ProjectionHead(nn.Module):
    """card.ProjectionHead (card.py:151-169) parameters."""

    def __init__(self, in_dim, proj_dim=128, dropout=0.2, init_logit_scale=10.0):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(in_dim, in_dim, bias=False), nn.LayerNorm(in_dim), nn.SiLU(),
                                 nn.Dropout(p=dropout), nn.Linear(in_dim, proj_dim))
        self.logit_scale = nn.Parameter(torch.tensor(math.log(init_logit_scale), dtype=torch.float32),
                                        requires_grad=False)
        self.logit_bias = nn.Parameter(torch.tensor(0.0, dtype=torch.float32), requires_grad=False)


class DeferredHead:
    """The fused path's last kernel (enc_head), not yet launched.  `launch(stream)`
    makes `stream` wait for everything enqueued on the producing stream so far and
    launches the head there, returning the [R, 128] embeddings (valid on `stream`)."""

    def __init__(self, fn, inputs):
        self._fn, self._inputs = fn, inputs
        self.ready = torch.cuda.Event()
        self.ready.record()  # after the transition GEMM, on the producing stream

    def launch(self, stream: torch.cuda.Stream) -> torch.Tensor:
        with torch.cuda.stream(stream):
            stream.wait_event(self.ready)
            for t in self._inputs:
                t.record_stream(stream)
            return self._fn()


class Model(nn.Module):
    """encoderAndHead.Model(in_channels, out_channels, warmup_epochs, proj_dim)."""

    def __init__(self, in_channels=None, out_channels=None, warmup_epochs=10, proj_dim=128):
        super().__init__()
        self.rmb = RMB(in_channels, out_channels, stride=1, warmup_epochs=warmup_epochs)
        self.head = ProjectionHead(out_channels, proj_dim=proj_dim, dropout=0.2)
        self._fused = None
        self._fused_key = None
        self._pdicts = None   # every submodule's _parameters / _buffers dict (cache-key walk)

    # -------------------------------------------------------------- weights --
    def _apply(self, fn, *args, **kwargs):  # .to() / .cuda() / .float(): tensors replaced
        self._pdicts = None
        return super()._apply(fn, *args, **kwargs)

    def _fused_weights(self, dtype, device):
        # key: identity and in-place version of every parameter and buffer, read from
        # the submodules' own dicts (a replaced or updated tensor changes it); the dicts
        # are listed once (walking parameters() / buffers() per forward cost ~140 us of
        # host time per frame)
        if self._pdicts is None:
            self._pdicts = [d for m in self.modules() for d in (m._parameters, m._buffers)]
        key = (dtype, device, tuple((id(t), t._version) for d in self._pdicts for t in d.values() if t is not None))
        if self._fused is not None and self._fused_key == key:
            return self._fused
        r = self.rmb
        with torch.no_grad():
            w = {}
            dr, dn = r.dsc_reinforce, r.dsc_normal
            w1 = torch.cat([m[0].weight.flatten(1) for m in (dr.depth, dr.point, dn.depth, dn.point)], 0)
            w["w1t"] = w1.t().contiguous().to(device, dtype)                              # [C, 4h]
            dw = torch.cat([m[1].weight for m in (dr.depth, dr.point, dn.depth, dn.point)], 0)
            w["dw"] = dw.to(device, dtype).contiguous(memory_format=torch.channels_last)  # host path
            w["dw_t"] = dw.reshape(dw.shape[0], 25).t().contiguous().to(device, torch.float32)  # [25, 4h]
            for tag, dsc in (("r", dr), ("n", dn)):
                bn = dsc.bn
                scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
                shift = bn.bias.float() - bn.running_mean.float() * scale
                w2 = torch.cat([dsc.depth[2].weight.flatten(1), dsc.point[2].weight.flatten(1)], 1).float()
                w[f"w2{tag}"] = (w2 * scale[:, None]).t().contiguous().to(device, dtype)  # [2h, C]
                w[f"b{tag}"] = shift.to(device, dtype)
            wt = r.transition[0].weight.flatten(1).float()                               # [C, 2C]
            C = wt.shape[0]
            w["wt1"] = wt[:, :C].t().contiguous().to(device, dtype)
            w["wt2"] = wt[:, C:].t().contiguous().to(device, dtype)
            w["wt"] = wt.t().contiguous().to(device, dtype)                          # [2C, C]: K = [x_f*s | x_n]
            # fused bf16 GEMM operands ([N][K] = the conv weight's own [out, in] layout)
            w2nk = []
            for dsc in (dr, dn):
                bn = dsc.bn
                scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
                w2 = torch.cat([dsc.depth[2].weight.flatten(1), dsc.point[2].weight.flatten(1)], 1).float()
                w2nk.append(w2 * scale[:, None])                                     # [C, 2h]
            w["w2_nk"] = torch.stack(w2nk, 0).contiguous().to(device, torch.bfloat16)  # [2, C, 2h]
            w["w1_nk"] = w1.contiguous().to(device, torch.bfloat16)                  # [4h, C]
            if tuple(w["w1_nk"].shape) == (1024, 512) and tuple(w["w2_nk"].shape) == (2, 512, 512):
                from .ops import enc_pack_fragments                                  # rmb_front operands
                w["w1_pk"] = enc_pack_fragments(w["w1_nk"])
                w["w2_pk"] = enc_pack_fragments(w["w2_nk"])
            w["b2"] = torch.cat([w["br"].float(), w["bn"].float()]).to(device, torch.float32)
            w["wt_nk"] = wt.contiguous().to(device, torch.bfloat16)                  # [C, 2C]
            if tuple(w["wt_nk"].shape) == (512, 1024):
                from .ops import enc_pack_fragments_k                                # trans4's operand
                w["wt_pk"] = enc_pack_fragments_k(w["wt_nk"])
            w["bt_f"] = r.transition[0].bias.float().to(device)
            w["bt"] = r.transition[0].bias.to(device, dtype)
            # f32 operands of the per-ROI tail kernels (enc_se / enc_head)
            se, hd = r.se.excitation, self.head.net
            f32 = lambda t: t.detach().float().contiguous().to(device)
            w["se_w1"], w["se_b1"], w["se_w2"], w["se_b2"] = f32(se[0].weight), f32(se[0].bias), \
                f32(se[2].weight), f32(se[2].bias)
            w["h0"], w["ln_w"], w["ln_b"] = f32(hd[0].weight), f32(hd[1].weight), f32(hd[1].bias)
            w["h4"], w["h4b"] = f32(hd[4].weight), f32(hd[4].bias)
            # the tail kernels' weight operands in fragment order: only when the fused tail can
            # run (every dimension a multiple of 16); other sizes take the plain-torch SE / head
            tail = ("se_w1", "se_w2", "h0", "h4")
            if all(w[k].shape[0] % 16 == 0 and w[k].shape[1] % 16 == 0 for k in tail):
                from .ops import enc_pack_rows
                for k in tail:
                    w[k + "_pk"] = enc_pack_rows(w[k])
        self._fused, self._fused_key = w, key
        return w

    # -------------------------------------------------------------- forward --
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            raise NotImplementedError("training-mode forward is out of scope (inference hot path only)")
        if x.is_cuda:
            if x.dtype == torch.float16:
                # the reference's GPU configuration (tracking.py:177-178: model.half(), fp16
                # ROI features): computed on the fp32 path from the exact fp16 values (weights
                # and inputs widen exactly), so the result is at least as accurate as an fp16
                # forward; the throughput path is bf16 (what the bench runs)
                x = x.float()
            return self._forward_device(x)
        return self._forward_host(x)

    def _alpha(self):
        r = self.rmb
        return 0.5 if r.current_epoch < r.warmup_epochs else float(torch.rand(1))  # RMB.forward :141

    def _head(self, g):
        hd = self.head.net
        z = F.linear(g, hd[0].weight.float())
        z = F.layer_norm(z, (z.shape[1],), hd[1].weight.float(), hd[1].bias.float(), hd[1].eps)
        z = F.linear(F.silu(z), hd[4].weight.float(), hd[4].bias.float())
        return F.normalize(z, dim=1)

    def _se(self, m_r):
        se = self.rmb.se.excitation
        return F.hardsigmoid(F.linear(F.relu(F.linear(m_r, se[0].weight.float(), se[0].bias.float())),
                                      se[2].weight.float(), se[2].bias.float()))

    # bf16 inputs take the fused trk GEMMs (enc_gemm.hip) when the shapes allow;
    # fp32 (the parity path) keeps hipBLASLt GEMMs + the separate act/mean passes
    fused_gemm = True
    fused_dwconv = True  # 10x10 bf16: depthwise 5x5 fused into the first GEMM (enc_g1_dwconv)
    fused_front = True   # 10x10 bf16, C = 512: first GEMMs + depthwise + DSC GEMMs in one kernel that also
                         # writes the SE's squeeze means (enc_rmb_front_means; Y2 never reaches HBM);
                         # False: enc_g1_dwconv + enc_dsc_gemm (Y2 in HBM)
    fused_tail = True    # bf16: SE + Shake2 mix + projection head as two trk kernels (enc_se(_means) / enc_head)
    defer_head = False   # fused tail: return a DeferredHead instead of launching enc_head
    stage_hook = None    # fused bf16 path: called as stage_hook("g1" | "dsc") right after that GEMM is
                         # enqueued (a caller can record an event there to place other streams' work)
    front_progress = None  # fused front: a one-element int32 device counter the front advances by one
                           # per finished ROI (enc_rmb_front_means' `progress`; a stream_gate waits on it)

    def _forward_device(self, x: torch.Tensor) -> torch.Tensor:
        """GEMMs on hipBLASLt (torch) or the fused trk GEMMs, everything else in trk HIP kernels."""
        from .ops import (act_mean, dwconv5_nhwc, scale_rows, enc_g1_dwconv, enc_dsc_gemm, enc_rmb_front_means,
                          enc_transition_gemm, enc_se, enc_se_means, enc_head, enc_sums_reduce)
        N, C, S1, S2 = x.shape
        dt, dev = x.dtype, x.device
        W = self._fused_weights(dt, dev)
        h4 = W["w1t"].shape[1]
        h2 = h4 // 2
        ss = S1 * S2
        X = x.permute(0, 2, 3, 1).reshape(N * ss, C)                 # view when channels_last
        Co = W["w2r"].shape[1]
        # the trk GEMMs' tiles: a 128-row tile spans at most 4 ROIs (ss >= 43), N % 256 == 0
        fused = (self.fused_gemm and dt == torch.bfloat16 and ss >= 43 and C % 32 == 0 and h4 % 256 == 0 and
                 h2 % 32 == 0 and Co % 256 == 0)
        ten = fused and S1 == 10 and S2 == 10 and C == 512 and X.is_contiguous()
        front = ten and self.fused_front and "w1_pk" in W and Co == 512
        if front:
            XRN, m_r, m_n = enc_rmb_front_means(X, W["w1_pk"], W["dw_t"], W["w2_pk"], W["b2"],
                                                progress=self.front_progress)
            if self.stage_hook is not None:
                self.stage_hook("g1")
                self.stage_hook("dsc")
        elif ten and self.fused_dwconv:
            Y2 = enc_g1_dwconv(X, W["w1_nk"], W["dw_t"])               # first 1x1 convs + depthwise 5x5, one kernel
            if self.stage_hook is not None:
                self.stage_hook("g1")
        else:
            Y1 = (X @ W["w1t"]).view(N, S1, S2, h4)                    # 4 first 1x1 convs, one GEMM (hipBLASLt)
            Y2 = dwconv5_nhwc(Y1, W["dw_t"]).view(N * ss, h4)         # 4 depthwise 5x5, one kernel
        if fused:
            # DSC pair + SE squeeze + GAP(x_n) in one GEMM; SE excitation + transition
            # + SiLU + GAP in another: the [M, 512] intermediates are written once (x_r|x_n)
            if not front:
                XRN, sums = enc_dsc_gemm(Y2, ss, W["w2_nk"], W["b2"], raw=True)
                if self.stage_hook is not None:
                    self.stage_hook("dsc")
            if self.fused_tail and "se_w1_pk" in W:
                # SE MLP (+ the squeeze means unless the front wrote them), then Shake2 mix +
                # projection head: one kernel each
                if front:
                    s = enc_se_means(m_r, W["se_w1_pk"], W["se_b1"], W["se_w2_pk"], W["se_b2"])
                else:
                    m_r, m_n, s = enc_se(sums, ss, W["se_w1_pk"], W["se_b1"], W["se_w2_pk"], W["se_b2"])
                tsums = enc_transition_gemm(XRN, ss, s, W["wt_nk"], W["bt_f"], raw=True, Wtp=W.get("wt_pk"))
                head = lambda: enc_head(tsums, ss, s, m_r, m_n, self._alpha(), W["h0_pk"], W["ln_w"], W["ln_b"],
                                        self.head.net[1].eps, W["h4_pk"], W["h4b"])
                if not self.defer_head:
                    return head()
                # the head (128 latency-bound workgroups) is left to the caller, who launches
                # it on the stream that consumes the embeddings: the caller's next launches on
                # this stream (the next frame's ROI Align / first GEMM) then fill the rest of
                # the GPU beside it
                return DeferredHead(head, (tsums, s, m_r, m_n))
            if not front:  # (the front wrote m_r / m_n)
                f = enc_sums_reduce(sums, ss)
                m_r, m_n = f[:, :Co] / ss, f[:, Co:] / ss
            s = self._se(m_r)
            m_cat = enc_transition_gemm(XRN, ss, s, W["wt_nk"], W["bt_f"], Wtp=W.get("wt_pk")) / ss
            a = self._alpha()
            g = 0.5 * m_cat + 0.5 * (a * (s * m_r) + (1 - a) * m_n)
            return self._head(g)
        XRN = torch.empty((N * ss, 2 * Co), device=dev, dtype=dt)    # [x_r | x_n] rows: the transition's K
        torch.addmm(W["br"], Y2[:, :h2], W["w2r"], out=XRN[:, :Co])  # DSC reinforce (BN folded)
        torch.addmm(W["bn"], Y2[:, h2:], W["w2n"], out=XRN[:, Co:])  # DSC normal (BN folded)
        XR = XRN.view(N, ss, 2 * Co)
        xr, xn = XR[:, :, :Co], XR[:, :, Co:]
        m_r = act_mean(xr, "silu", write=False)                      # SE squeeze of SiLU(xr), no write-back
        m_n = act_mean(xn, "hardswish")                              # Hardswish + its GAP, in place
        s = self._se(m_r)
        scale_rows(xr, s, act="silu")                                # x_f * s = SiLU(xr) * s, in place
        T = torch.addmm(W["bt"], XRN, W["wt"])                       # transition over cat[x_f*s, x_n], K = 2C
        m_cat = act_mean(T.view(N, ss, Co), "silu", write=False)     # SiLU + GAP, no write-back
        a = self._alpha()
        g = 0.5 * m_cat + 0.5 * (a * (s * m_r) + (1 - a) * m_n)     # Shake2 eval :94-96 + GAP
        return self._head(g)

    def _forward_host(self, x: torch.Tensor) -> torch.Tensor:
        """The same fused graph in plain torch ops (CPU tensors)."""
        N, C, S1, S2 = x.shape
        dt, dev = x.dtype, x.device
        W = self._fused_weights(dt, dev)
        h4 = W["w1t"].shape[1]
        h2 = h4 // 2
        ss = S1 * S2
        Co = W["w2r"].shape[1]
        X = x.permute(0, 2, 3, 1).reshape(N * ss, C)
        Y1 = (X @ W["w1t"]).view(N, S1, S2, h4).permute(0, 3, 1, 2)
        Y2 = F.conv2d(Y1, W["dw"], padding=2, groups=h4).permute(0, 2, 3, 1).reshape(N * ss, h4)
        xr = F.silu(torch.addmm(W["br"], Y2[:, :h2], W["w2r"])).view(N, ss, Co)
        xn = F.hardswish(torch.addmm(W["bn"], Y2[:, h2:], W["w2n"])).view(N, ss, Co)
        m_r = xr.mean(1, dtype=torch.float32)
        s = self._se(m_r)
        xfs = (xr * s.to(dt)[:, None, :]).view(N * ss, Co)
        T = torch.addmm(W["bt"], xfs, W["wt1"])
        T.addmm_(xn.reshape(N * ss, Co), W["wt2"])
        m_cat = F.silu(T).view(N, ss, Co).mean(1, dtype=torch.float32)
        m_n = xn.mean(1, dtype=torch.float32)
        a = self._alpha()
        g = 0.5 * m_cat + 0.5 * (a * (s * m_r) + (1 - a) * m_n)
        return self._head(g)
