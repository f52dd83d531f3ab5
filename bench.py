"""Benchmark: ROIs/s for roi_align -> embed -> cost -> assign, N=256 per frame.

Workload (BASELINE.json configs[2]): each GPU runs
8 independent synthetic video streams of 256 moving objects; one step = one
frame of every stream, the full per-frame tracker hot path:
  [8,512,40,40] fp32 SPP-CSPC maps (SiLU(randn), resident) + 256 boxes/frame
  -> trk roi_align      (HIP: NCHW f32 in, NHWC bf16 out, 10x10 bins)
  -> encoder            (HIP: rmb_front = 1x1 convs + depthwise + DSC GEMM fused,
                         SE, transition GEMM, projection head; bf16 MFMA)
  -> MultiStreamTracker.step:
       KF predict + gate inputs (HIP) -> fused cost: top-5 of a 30-deep memory
       bank (f32 MFMA), bbox, conf, Mahalanobis gate (HIP) -> scipy-exact LSAP +
       cost gate (HIP) -> assignment indices to the host -> KF update / EMA /
       bank push (HIP), births, purge.
Boxes move at constant velocity (bouncing), detections arrive shuffled; a
30-frame pre-roll fills the memory banks before warm-up.  All inputs are in
HBM before timing starts.  Multi-GPU: one process per GPU, each with its own 8
streams, no data-path collective; one barrier + MAX(elapsed) all-reduce per
report ("scaling": "weak").  The ranks come from torchrun (RANK / WORLD_SIZE in
the environment, which must agree with --gpus) or, for `bench.py --gpus N`
started alone, from N child processes this script starts before anything
touches the GPU (_spawn_ranks).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import os
import sys


def _spawn_ranks():
    """`python bench.py --gpus N` with N > 1 and no WORLD_SIZE: start N rank
    processes (this script again, as children: RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set), wait for them and exit with the
    first failing child's status (the others are then stopped).  Rank 0 prints
    the JSON line on the inherited stdout.  Runs before torch or the library is
    imported, so this process never initialises the GPU (and never re-execs).
    With WORLD_SIZE already set (torchrun) it only checks that --gpus agrees."""
    import argparse
    import socket
    import subprocess
    import time as _time
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} disagrees with WORLD_SIZE={ws} "
                             f"(launch with torchrun --nproc-per-node {a.gpus}, or without torchrun)")
        return
    if a.gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {a.gpus}")
    if a.gpus == 1:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        _time.sleep(0.2)
    for p in procs:  # a failed rank leaves the others in a collective: stop them (exact PIDs)
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        if rc == 0 and p.returncode != 0:
            rc = p.returncode
    print(f"bench.py: {a.gpus} ranks finished, exit {rc}", file=sys.stderr, flush=True)
    sys.exit(rc if rc > 0 else (1 if rc else 0))


if __name__ == "__main__":
    _spawn_ranks()

import argparse
import importlib
import json
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
trk = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd")
ops = importlib.import_module("a-lightweight-unsupervised-feature-extractor-_amd.ops")

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (spec)
F32_MFMA_PEAK_TFLOPS = 157.3   # f32-input MFMA (= f32 vector peak)
ENC_FLOP_PER_ROI = {10: 320.61e6, 7: 157.57e6}   # BASELINE.md §4 (FlopCounterMode)
PREROLL = 30


# ------------------------------------------------------------ workload ----
MAP_POOL = 16  # frames' maps in the rotating pool: 16 x 26 MB > the 256 MB Infinity Cache
# map layout the detector hands over: "nchw" (the default: the reference's YOLOv7 SPPCSPC
# output, what the drop-in receives; roi_align transposes each frame's map once inside the
# timed step) or "nhwc" (channels_last, what an NHWC backbone on MI355X would emit;
# roi_align reads it directly)
MAP_LAYOUT = os.environ.get("TRK_MAP_LAYOUT", "nchw")


def make_scenes(dev, streams, N, frames, seed, C=512, H=40, pool=MAP_POOL):
    """Per stream: N objects with w, h ~ U(32, 320) px in a 1280x1280
    letterboxed frame (rows 280..1000 = a 1080p picture), velocities
    U(-2, 2) px/frame bouncing at the borders, 0.5 px detection jitter,
    conf ~ U(0.55, 0.99); detection order shuffled every frame.  Feature
    maps: a pool of `pool` frames of [streams, 512, 40, 40] f32 maps (SiLU(randn);
    channels_last unless TRK_MAP_LAYOUT=nchw), frame f reads slot f % pool, so every
    frame's map read comes from HBM, not from a cache that held it since the
    previous frame."""
    rng = np.random.default_rng(seed)
    g = torch.Generator(device=dev).manual_seed(seed)
    feat = torch.nn.functional.silu(torch.randn((pool, streams, C, H, H), generator=g, device=dev))
    if MAP_LAYOUT == "nhwc":  # per-frame [streams, C, H, W] slices with channels_last strides
        feat = feat.permute(0, 1, 3, 4, 2).contiguous().permute(0, 1, 4, 2, 3)
    elif MAP_LAYOUT != "nchw":
        raise ValueError(f"TRK_MAP_LAYOUT must be nhwc or nchw, got {MAP_LAYOUT!r}")
    w = rng.uniform(32, 320, (streams, N)); h = rng.uniform(32, 320, (streams, N))
    lo = np.stack([np.zeros_like(w), np.full_like(h, 280.0)], -1)
    hi = np.stack([1280 - w, 1000 - h], -1)
    p = lo + rng.random((streams, N, 2)) * (hi - lo)
    v = rng.uniform(-2, 2, (streams, N, 2))
    conf = rng.uniform(0.55, 0.99, (streams, N))
    rois = np.zeros((frames, streams * N, 5), np.float32)
    dbox = np.zeros((frames, streams, N, 4), np.float32)
    dconf = np.zeros((frames, streams, N), np.float32)
    obj = np.zeros((frames, streams, N), np.int64)
    for f in range(frames):
        for s in range(streams):
            perm = rng.permutation(N)
            obj[f, s] = perm
            q = p[s, perm] + rng.normal(0, 0.5, (N, 2))
            b = np.concatenate([q, q + np.stack([w[s, perm], h[s, perm]], -1)], -1)
            dbox[f, s] = b
            dconf[f, s] = np.clip(conf[s, perm] + rng.normal(0, 0.01, N), 0.5, 0.999)
            rois[f, s * N:(s + 1) * N, 0] = s
            rois[f, s * N:(s + 1) * N, 1:] = b
        p = p + v
        bounce = (p < lo) | (p > hi)
        v[bounce] *= -1
        p = np.clip(p, lo, hi)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return dict(feat=feat, rois=t(rois), dbox=t(dbox), dconf=t(dconf), confs_host=dconf,
                obj=obj, streams=streams, N=N, np=dict(rois=rois, dbox=dbox, dconf=dconf))


def frame_map(sc, f):
    """[streams, 512, 40, 40] map batch of frame f (rotating pool slot)"""
    return sc["feat"][f % sc["feat"].shape[0]]


class Pipeline:
    """The per-frame hot path over a batch of streams.

    Software-pipelined across frames: frame f+1's ROI Align + encoder (which do
    not depend on tracking state) are enqueued on a side stream at the start of
    frame f's step, so they run while frame f's cost build, solver (one
    workgroup per video stream) and host bookkeeping proceed; frame f+1's cost
    build waits for them with a stream event.  Every frame still does the full
    work once, inside the timed region."""

    def __init__(self, sc, model, S=10):
        self.sc, self.model, self.S = sc, model, S
        self.tracker = trk.MultiStreamTracker(sc["streams"], capacity=1024, device=sc["feat"].device)
        self.ids = {}
        # consecutive frames' embeddings alternate between two side streams (default 2 since
        # r05, with TRK_EMBED_OVERLAP below), so frame f's SE and transition run beside frame
        # f+1's front instead of before it
        n_side = int(os.environ.get("TRK_EMBED_STREAMS", "2"))
        self.sides = [torch.cuda.Stream(device=sc["feat"].device) for _ in range(n_side)]
        self.side = self.sides[0]
        self.pending = {}  # frame -> (embeddings, ready event)
        self.graphs = None
        # enqueue frame f+1's embedding at the start of step f (measured 1.13M vs
        # 0.94M ROIs/s against enqueueing it after step f's LSAP launch): the
        # cost build and solver of f then share the GPU with it instead of
        # serialising between consecutive encoder runs
        self.prefetch_early = os.environ.get("TRK_PREFETCH_EARLY", "1") == "1"
        self.depth = int(os.environ.get("TRK_PREFETCH_DEPTH", "1"))  # frames embedded ahead
        # the tracker's launches (mostly few-workgroup kernels) on a high-priority stream so
        # they dispatch as soon as CUs free up beside the encoder's full-GPU grids
        prio = int(os.environ.get("TRK_TRACK_PRIO", "1"))
        self.track_stream = torch.cuda.Stream(device=sc["feat"].device, priority=-1) if prio else None
        # TRK_HEAD_STREAM=1: the encoder's last kernel (projection head, 128 latency-bound
        # workgroups) launched on the tracker's stream right before the frame's tracker step (the
        # default in r02-r04, with one embedding stream).  Default 0 since r05: with the two
        # overlapping embedding streams the head stays on its frame's embedding stream behind the
        # transition, and the tracker stream carries only the tracker step (its live sum ≈ 0.63
        # vs 0.85 ms per step); pipeline 2.021-2.091 vs 2.008-2.090M ROIs/s, six of seven
        # interleaved pairs ahead (r5o, r5q)
        self.defer_head = os.environ.get("TRK_HEAD_STREAM", "0") == "1" and self.track_stream is not None
        # ROI Align of frame f+1 issued on its own stream when frame f's encoder is enqueued,
        # so the encoder stream runs GEMMs only (TRK_ROI_STREAM, default 1 since r03: with
        # NCHW maps and the 75-us sweep, 1.674-1.694 vs 1.641-1.682M ROIs/s in three
        # interleaved pairs; +0.7..2 % with r02's kernels)
        self.roi_stream = (torch.cuda.Stream(device=sc["feat"].device)
                           if os.environ.get("TRK_ROI_STREAM", "1") == "1" else None)
        self.roi_pending = {}
        # TRK_ROI_AFTER=g1|dsc: frame f+1's ROI Align waits for frame f's first GEMM / DSC GEMM
        # (an event recorded through encoder.Model.stage_hook), so it runs beside the
        # encoder's later kernels instead of as soon as it is enqueued
        # Default "dsc" since rmb_front (r03): rmb_front fills a CU's VGPRs (two 248-register
        # waves per SIMD), so a ROI Align running beside it only gets CUs between its
        # workgroups; gated behind it, it runs beside the transition GEMM instead (1.910 /
        # 1.917M vs 1.887 / 1.882M ROIs/s ungated, 1.801 / 1.807M on the embedding stream;
        # rmb_front live 657 vs 741 us)
        self.roi_after = os.environ.get("TRK_ROI_AFTER", "dsc") if self.roi_stream is not None else ""
        self.roi_gate = None
        # TRK_ROI_GATE_FRAC < 1: instead of frame f's whole front, frame f+1's ROI stage waits
        # (trk_stream_gate, bounded) until the front has finished that fraction of its ROIs, so it
        # starts on the CUs the persistent front's last, partly filled round leaves idle (the front
        # counts finished ROIs into a device counter: enc_rmb_front_means' `progress` argument)
        # Default 0.93 since r05: 2.030-2.053 vs 1.968-2.043M ROIs/s, six of seven interleaved
        # pairs ahead, +1.1 % in the means (r5l, r5l2); 0.88 / 0.91 / 0.95 / 0.97 within or below
        self.gate_frac = float(os.environ.get("TRK_ROI_GATE_FRAC", "0.93"))
        self.progress = None
        self.fronts_rois = 0       # the count the counter reaches once every enqueued front is done
        self.roi_gate_target = None
        if self.roi_after == "dsc" and self.gate_frac < 1:
            # the pipeline's own counter, passed to its fronts as their `progress` argument (the
            # library keeps no pointer); started near the u32 wrap (TRK_PROGRESS_START) to show
            # the gate's wrap-safe comparison in a run
            start = int(os.environ.get("TRK_PROGRESS_START", "0")) & 0xFFFFFFFF
            self.progress = torch.tensor([start - (1 << 32) if start >= 1 << 31 else start],
                                         dtype=torch.int32, device=sc["feat"].device)
            self.fronts_rois = start
            self.model.front_progress = self.progress
        # TRK_EMBED_OVERLAP=1 (with TRK_EMBED_STREAMS=2, both the default since r05): frame f+1's
        # encoder, on the other embedding stream, waits only for frame f's front (not its SE and
        # transition), so the next front's workgroups fill the CUs the transition's last round
        # leaves idle: 2.092-2.138 vs 2.048-2.082M ROIs/s in six interleaved pairs (r5c, r5d); the
        # front's live launch window then includes the transition it shares the GPU with
        self.overlap = os.environ.get("TRK_EMBED_OVERLAP", "1") == "1" and n_side > 1
        self.front_ev = None
        if self.roi_after or self.overlap:
            def hook(name):
                if name == "dsc" and self.progress is not None:
                    r = self.sc["streams"] * self.sc["N"]
                    self.roi_gate_target = (self.fronts_rois + int(self.gate_frac * r)) & 0xFFFFFFFF
                    self.fronts_rois = (self.fronts_rois + r) & 0xFFFFFFFF
                elif name == self.roi_after:
                    self.roi_gate = torch.cuda.Event()
                    self.roi_gate.record(torch.cuda.current_stream())
                if self.overlap and name == "dsc":
                    self.front_ev = torch.cuda.Event()
                    self.front_ev.record(torch.cuda.current_stream())
            self.model.stage_hook = hook
        # NCHW maps, TRK_MAP_AHEAD=1: frame f's NCHW -> NHWC copy (roi_align's first kernel)
        # issued on the tracker's stream two frames ahead, right after frame f-2's tracker
        # step, beside the encoder's kernels; off by default: 1.613-1.616 vs 1.622-1.625M
        # ROIs/s with the copy inside roi_align on the embedding stream (two A/B pairs)
        self.map_ahead = (MAP_LAYOUT == "nchw" and self.track_stream is not None and
                          os.environ.get("TRK_MAP_AHEAD", "0") == "1")
        self.map_pending = {}

    def close_progress(self):
        """stop the fronts' progress counting and the gates on it (graph capture, and the
        isolated kernel pass's fronts, which the pipeline's targets do not know of)"""
        if self.progress is not None:
            torch.cuda.synchronize()
            self.model.front_progress = None
            self.progress = None
            self.roi_gate_target = None

    def _map_ahead(self, f):
        if not self.map_ahead or f in self.map_pending or f >= len(self.sc["rois"]):
            return
        with torch.cuda.stream(self.track_stream):
            m = trk.nchw_to_nhwc(frame_map(self.sc, f))
            ev = torch.cuda.Event()
            ev.record(self.track_stream)
        self.map_pending[f] = (m, ev)

    def capture(self):
        """Capture roi_align + encoder as two hipGraphs (static ROI / embedding
        buffers, alternating per frame so frame f+1's replay never overwrites
        the embeddings frame f's tracker step is still reading).  Removes the
        launch gaps between the ~30 kernels of the stage."""
        sc = self.sc
        # graph replays never call the stage hook again: the events and targets it would set up
        # (the overlap's front_ev, the ROI progress gate) belong to the eager pipeline, so both
        # are switched off here, before the capture records anything
        self.close_progress()
        self.overlap = False
        self.front_ev = None
        self.roi_gate = None
        self.model.stage_hook = None
        self.graphs = []
        for _ in range(2):
            rois = sc["rois"][0].clone()
            with torch.cuda.stream(self.side):
                for _ in range(2):  # warm-up: weight caches, kernel attributes
                    self._embed_from(rois)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.side):
                emb = self._embed_from(rois)
            self.graphs.append((g, rois, emb))
        torch.cuda.synchronize()

    def _embed_from(self, rois):
        roi = trk.roi_align(frame_map(self.sc, 0), rois, (self.S, self.S), 40 / 1280.0, 2, True,
                            out_dtype=torch.bfloat16, channels_last=True)
        return self.stage_embed(roi)

    def stage_roi(self, f):
        fm = frame_map(self.sc, f)
        if self.map_ahead:
            self._map_ahead(f)  # (frames not converted ahead: now)
            fm, ev = self.map_pending.pop(f)
            st = torch.cuda.current_stream()
            st.wait_event(ev)
            fm.record_stream(st)
        return trk.roi_align(fm, self.sc["rois"][f], (self.S, self.S), 40 / 1280.0, 2, True,
                             out_dtype=torch.bfloat16, channels_last=True)

    def stage_embed(self, roi):
        with torch.no_grad():
            return self.model(roi).view(self.sc["streams"], self.sc["N"], 128)

    def embed_async(self, f):
        """enqueue frame f's roi_align + encoder on the side stream"""
        if f in self.pending or f >= len(self.sc["rois"]):
            return
        main = torch.cuda.current_stream()
        side = self.sides[f % len(self.sides)]
        if self.graphs is not None:
            side.wait_stream(main)  # graph replays reuse per-parity buffers main may still read
        # (eager: no wait on main -- an embedding reads only the frame's static map / boxes
        # and writes buffers of its own (kept alive for main by record_stream); main waits on
        # `ev`.  So the encoder runs back to back on its stream while the tracker overlaps it)
        with torch.cuda.stream(side):
            if self.overlap and self.front_ev is not None:
                side.wait_event(self.front_ev)  # the previous frame's front is done
            if self.graphs is not None:
                g, rois, emb = self.graphs[f & 1]
                rois.copy_(self.sc["rois"][f], non_blocking=True)
                g.replay()
            else:
                roi = self._roi_for(f, side)
                self.model.defer_head = self.defer_head
                try:
                    if self.defer_head:
                        with torch.no_grad():
                            emb = self.model(roi)
                    else:
                        emb = self.stage_embed(roi)
                finally:
                    self.model.defer_head = False
                self._roi_ahead(f + 1)
                if hasattr(emb, "launch"):  # deferred head: launched by _step on the tracker's stream
                    self.pending[f] = (emb, None)
                    return
                emb = emb.view(self.sc["streams"], self.sc["N"], 128)
            ev = torch.cuda.Event()
            ev.record(side)
        emb.record_stream(main)
        self.pending[f] = (emb, ev)

    def _roi_ahead(self, f):
        """ROI Align of frame f on its own stream, now: it runs beside the encoder
        launches already queued (VALU-bound next to MFMA-bound) instead of before the
        frame's first GEMM on the encoder stream"""
        if self.roi_stream is None or f in self.roi_pending or f >= len(self.sc["rois"]):
            return
        with torch.cuda.stream(self.roi_stream):
            if self.roi_gate_target is not None:
                trk.ops.stream_gate(self.progress, self.roi_gate_target, 2000)
                self.roi_gate_target = None
            if self.roi_gate is not None:
                self.roi_stream.wait_event(self.roi_gate)
                self.roi_gate = None
            roi = self.stage_roi(f)
            ev = torch.cuda.Event()
            ev.record(self.roi_stream)
        self.roi_pending[f] = (roi, ev)

    def _roi_for(self, f, side):
        if self.roi_stream is None:
            return self.stage_roi(f)
        self._roi_ahead(f)
        roi, ev = self.roi_pending.pop(f)
        side.wait_event(ev)
        roi.record_stream(side)
        return roi

    def step(self, f):
        if self.track_stream is not None:
            with torch.cuda.stream(self.track_stream):
                return self._step(f)
        return self._step(f)

    def _step(self, f):
        sc = self.sc
        self.embed_async(f)
        emb, ev = self.pending.pop(f)
        if ev is None:  # deferred head: launched here, on the tracker's stream, before the step
            with torch.no_grad():
                emb = emb.launch(torch.cuda.current_stream()).view(sc["streams"], sc["N"], 128)
        else:
            torch.cuda.current_stream().wait_event(ev)
        if self.prefetch_early:  # next frame's embedding before this frame's cost build
            for d in range(1, self.depth + 1):
                self.embed_async(f + d)
            hook = None
        else:
            hook = lambda: self.embed_async(f + 1)
        # the whole tracker step is enqueued (no host wait inside a frame); its
        # results reach pinned host memory by one copy and are read in order
        h = self.tracker.step_async(emb, sc["dbox"][f], sc["dconf"][f], [sc["N"]] * sc["streams"],
                                    [f] * sc["streams"], after_launch=hook)
        self._map_ahead(f + 2)  # on this (the tracker's) stream, behind the frame's step
        return h

    def check_identity(self, f, res):
        """fraction of detections matched to the track that has followed the
        same object since the track was created"""
        res = res.result() if hasattr(res, "result") else res
        ok = tot = 0
        for s, r in enumerate(res):
            objs = self.sc["obj"][f, s]
            for tid, j in r.matches:
                o = int(objs[j])
                k = (s, int(tid))
                if k not in self.ids:
                    self.ids[k] = o
                ok += self.ids[k] == o
            tot += self.sc["N"]
        return ok / max(tot, 1)


# ----------------------------------------------------------- measurement --
def prof_mark():
    """One marker kernel (torch.cuda._sleep -> `spin_kernel`) then a device sync: bench.py
    brackets its timed region and its isolated kernel pass with one each side, so a
    rocprofv3 trace or counter pass of the whole run splits into those two windows by
    dispatch order (tools/prof_window.py).  Outside the timed clock."""
    torch.cuda._sleep(1)
    torch.cuda.synchronize()


def _ev():
    return torch.cuda.Event(enable_timing=True)


class LiveProbe:
    """HIP-event pairs around the library calls of the hot path INSIDE the timed
    region, recorded on the stream each call launches on (the side stream for
    roi_align + encoder).  Wraps ops' handle to libtrk_amd; inactive outside
    the timed region.  Each bracketed call is one kernel launch, except
    trk_roi_align_fwd (NCHW->NHWC transpose + sweep = the roi stage) and the
    two summing GEMMs (a 4-8 MB hipMemsetAsync of the sums precedes the GEMM)."""

    NAMES = {"trk_roi_align_fwd": "roi_stage", "trk_nchw_to_nhwc": "map_nhwc", "trk_enc_g1_dwconv": "enc_g1_dwconv",
             "trk_enc_dsc_gemm": "enc_gemm_dsc", "trk_enc_transition_gemm": "enc_gemm_trans",
             "trk_enc_transition_gemm2": "enc_gemm_trans",
             "trk_enc_rmb_front_means": "enc_rmb_front", "trk_enc_se_means": "enc_se",
             "trk_enc_se": "enc_se", "trk_enc_head": "enc_head", "trk_build_cost": "cost_live",
             "trk_lsap": "lsap_live", "trk_build_cost_dev": "cost_live", "trk_lsap_dev": "lsap_live",
             "trk_step_begin": "step_begin", "trk_step_mid": "step_mid", "trk_step_end": "step_end",
             "trk_step_apply": "step_apply"}

    def __init__(self, pool=4096):
        self.on = False
        self.ev = {v: [] for v in self.NAMES.values()}
        # events made before the timed region (creating two per call inside it cost host
        # time the pipeline then waited for), handed out in order
        self.pool = [_ev() for _ in range(pool)]
        self.pi = 0
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self._orig = ops.lib
        probe = self

        class _Proxy:
            def __getattr__(self, name):  # first lookup of a name only: the result is cached
                fn = getattr(probe._orig(), name)
                key = probe.NAMES.get(name)
                if key is None:
                    setattr(self, name, fn)
                    return fn

                def call(*a):
                    if not probe.on:
                        return fn(*a)
                    st = ops.current_stream(probe.dev)  # cached Stream object (cheap lookup)
                    if probe.pi + 2 <= len(probe.pool):
                        e0, e1 = probe.pool[probe.pi], probe.pool[probe.pi + 1]
                        probe.pi += 2
                    else:
                        e0, e1 = _ev(), _ev()
                    e0.record(st)
                    rc = fn(*a)
                    e1.record(st)
                    probe.ev[key].append((e0, e1))
                    return rc
                setattr(self, name, call)
                return call

        self._proxy = _Proxy()
        ops.lib = lambda: self._proxy
        trk.tracking.lib = lambda: self._proxy  # the tracker's step launches

    def means_us(self):
        torch.cuda.synchronize()
        return {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e3 for k, v in self.ev.items() if v}

    def stage_means_us(self, key):
        """the tracker's cost / LSAP launches alternate stage 1 (main rows) and stage 2
        (ReID-only rows): mean device time of each, per launch"""
        torch.cuda.synchronize()
        v = [a.elapsed_time(b) * 1e3 for a, b in self.ev.get(key, [])]
        return {"stage1": round(float(np.mean(v[0::2])), 2) if v[0::2] else None,
                "stage2": round(float(np.mean(v[1::2])), 2) if v[1::2] else None}

    def sum_per_step_us(self, steps):
        """summed device time of every probed launch per step: compared with
        ms_per_step it shows whether streams overlapped (sum > step) or the GPU
        idled (sum < step)"""
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for v in self.ev.values() for a, b in v) * 1e3 / max(steps, 1)

    def embed_gaps_us(self, n_side=1, head_deferred=False, roi_own_stream=False):
        """mean time between one frame's last launch on the embedding stream ending
        (enc_head, or the transition GEMM when the head is deferred to the tracker's
        stream) and the next frame's first launch on it starting (the roi stage, or the
        encoder front when ROI Align has a stream of its own): the embedding stream's
        idle time per frame (None with several embedding streams: frames then overlap
        on purpose)"""
        if n_side != 1:
            return None
        ends = self.ev["enc_gemm_trans" if head_deferred else "enc_head"]
        first = "roi_stage"
        if roi_own_stream:
            first = "enc_rmb_front" if self.ev.get("enc_rmb_front") else "enc_g1_dwconv"
        starts = self.ev[first]
        gaps = [e1.elapsed_time(s0) * 1e3 for (_, e1), (s0, _) in zip(ends, starts[1:])]
        return float(np.mean(gaps)) if gaps else None


def kernel_pass(pipe, f, reps=10):
    """Average device time of each hand-written kernel on the real step inputs,
    HIP events on the stream the kernel is launched on (the current stream)."""
    sc, tr = pipe.sc, pipe.tracker
    st = torch.cuda.current_stream()
    out = {}

    def timed(name, fn):
        fn()
        e0, e1 = _ev(), _ev()
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        st.synchronize()
        out[name] = e0.elapsed_time(e1) / reps * 1e3  # us

    # roi_align kernel alone (map already NHWC) and the stage (NCHW map: + transpose)
    nhwc = frame_map(sc, f).contiguous(memory_format=torch.channels_last)
    timed("roi_align", lambda: trk.roi_align(nhwc, sc["rois"][f], (pipe.S, pipe.S), 40 / 1280.0, 2, True,
                                             out_dtype=torch.bfloat16, channels_last=True))
    timed("roi_stage", lambda: pipe.stage_roi(f))
    roi = pipe.stage_roi(f)
    m = pipe.model
    W = m._fused_weights(torch.bfloat16, roi.device)
    K = roi.shape[0]
    X = roi.permute(0, 2, 3, 1).reshape(K * 100, 512)
    if "w1_pk" in W:
        timed("enc_rmb_front", lambda: ops.enc_rmb_front_means(X, W["w1_pk"], W["dw_t"], W["w2_pk"], W["b2"]))
    timed("enc_g1_dwconv", lambda: ops.enc_g1_dwconv(X, W["w1_nk"], W["dw_t"]))
    Y2 = ops.enc_g1_dwconv(X, W["w1_nk"], W["dw_t"])
    timed("enc_gemm_dsc", lambda: ops.enc_dsc_gemm(Y2, 100, W["w2_nk"], W["b2"]))
    XRN, sum_r, _ = ops.enc_dsc_gemm(Y2, 100, W["w2_nk"], W["b2"])
    with torch.no_grad():
        s_se = m._se(sum_r / 100)
    timed("enc_gemm_trans", lambda: ops.enc_transition_gemm(XRN, 100, s_se, W["wt_nk"], W["bt_f"],
                                                            Wtp=W.get("wt_pk")))
    timed("encoder", lambda: pipe.stage_embed(roi))
    emb = pipe.stage_embed(roi)
    # tracker kernels on the current track table (rows = all live tracks)
    t = tr.table
    S_, N = sc["streams"], sc["N"]
    live = [tr.live_slots(s) for s in range(S_)]
    M = max(len(l) for l in live)
    row_slot = np.zeros((S_, M), np.int32)
    for s in range(S_):
        row_slot[s, :len(live[s])] = live[s]
    rs = torch.as_tensor(row_slot).to(emb.device)
    Ms = [len(l) for l in live]
    cost_out = {"C_total": torch.empty((S_, M, N), device=emb.device)}
    timed("cost", lambda: trk.build_cost(M=Ms, N=[N] * S_, bank=t.bank, bank_len=t.bank_len, pbox=t.pbox,
                                         conf_prev=t.last_conf, det_emb=emb, dbox=sc["dbox"][f],
                                         conf_cur=sc["dconf"][f], params=tr.params, gmean=t.gmean,
                                         gsinv=t.gsinv, gate_on=t.gate_on, row_slot=rs, out=cost_out))
    C = cost_out["C_total"]
    lo = trk.lsap_batched(C, Ms, [N] * S_, cost_max=50.0)
    timed("lsap", lambda: trk.lsap_batched(C, Ms, [N] * S_, cost_max=50.0, out=lo))
    # trk_lsap_dev (sizes in device memory, the tracker's launch) on the same matrices, its launch
    # sized by the pipeline's row bound (last_Mb: live tracks + detections in flight) and by M:
    # the kernel instantiation (column slots) is the bound's, the solve the matrix's own
    L = ops.lib()
    dnr = torch.tensor(Ms, dtype=torch.int32, device=emb.device)
    dnc = torch.full((S_,), N, dtype=torch.int32, device=emb.device)
    Mb = max(int(tr.last_Mb), M)
    Cp = torch.full((S_, Mb, N), 1e3, device=emb.device)
    Cp[:, :M] = C
    kq = min(Mb, N)
    dv = {"rows": torch.empty((S_, kq), dtype=torch.int64, device=emb.device),
          "cols": torch.empty((S_, kq), dtype=torch.int64, device=emb.device),
          "count": torch.empty((S_,), dtype=torch.int32, device=emb.device),
          "status": torch.empty((S_,), dtype=torch.int32, device=emb.device),
          "assign": torch.empty((S_, Mb), dtype=torch.int32, device=emb.device)}
    for name, bound in (("lsap_dev_bound", Mb), ("lsap_dev_m", M)):
        def run(bound=bound):
            rc = L.trk_lsap_dev(S_, ops._ptr(Cp), 0, N, Mb * N, ops._ptr(dnr), ops._ptr(dnc), bound, N, kq,
                                ops._ptr(dv["rows"]), ops._ptr(dv["cols"]), ops._ptr(dv["count"]),
                                ops._ptr(dv["status"]), ops._ptr(dv["assign"]), Mb, 50.0, ops._stream(emb.device))
            assert rc == 0, rc
        timed(name, run)
    return out, M, {"lsap_dev_bound_rows": Mb}


def _cpu_info():
    """host CPU model and physical cores (lscpu), and the threads torch uses"""
    import subprocess
    model, cores = None, None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {l.split(":", 1)[0].strip(): l.split(":", 1)[1].strip() for l in out.splitlines() if ":" in l}
        model = kv.get("Model name")
        cps, socks = kv.get("Core(s) per socket"), kv.get("Socket(s)")
        cores = int(cps) * int(socks) if cps and socks else None
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    return model, cores


def _cpu_leg(sc, sd, O, LIT, lsa, N, S, frames_vec, frames_lit, budget_s):
    """One CPU leg: the first N detections of one stream per frame (tracks = those objects,
    banks of 30), S x S ROIs; returns per-stage medians (s) and the frame counts."""
    npw = sc["np"]
    Ns = sc["N"]
    rng = np.random.default_rng(7)
    bank = rng.standard_normal((N, 30, 128)).astype(np.float32)
    bank /= np.linalg.norm(bank, axis=-1, keepdims=True)
    gm = np.zeros((N, 4)); gs = np.tile(np.eye(4).reshape(1, 16) / 11.0, (N, 1))
    kf_x = [np.zeros(8) for _ in range(N)]
    kf_P = [np.diag([10.0] * 4 + [1000.0] * 4) for _ in range(N)]
    t_roi, t_enc, t_cost, t_lsap, t_lit = [], [], [], [], []
    t_start = time.perf_counter()
    for q in range(3 + frames_vec):
        f = (PREROLL + q) % len(npw["rois"])
        st = q % sc["streams"]
        rois = npw["rois"][f, st * Ns:st * Ns + N].copy()
        rois[:, 0] = 0
        fmap = frame_map(sc, f)[st:st + 1].cpu().numpy()
        t0 = time.perf_counter()
        roi = O.roi_align(fmap, rois, (S, S), 40 / 1280.0, 2, True)
        t1 = time.perf_counter()
        with torch.no_grad():
            emb = O.encoder_forward(sd, torch.from_numpy(roi)).numpy()
        t2 = time.perf_counter()
        b, c = npw["dbox"][f, st, :N], npw["dconf"][f, st, :N]
        out = O.cost_build(bank, np.full(N, 30, np.int32), emb, b, b, c, c, gm, gs, np.ones(N, np.int32))
        t3 = time.perf_counter()
        lsa(out["C_total"])
        t4 = time.perf_counter()
        if q < frames_lit + 1:  # literal cost: 1 warm-up + frames_lit timed
            capp = LIT.build_c_app_topk_literal([list(bank[i]) for i in range(N)], list(emb))
            tot = O.cost_combine(capp, b, b, c, c)["C_total"]
            LIT.kalman_gating_literal(tot, kf_x, kf_P, b.tolist())
            if q >= 1:
                t_lit.append(time.perf_counter() - t4)
        if q >= 3:
            t_roi.append(t1 - t0); t_enc.append(t2 - t1); t_cost.append(t3 - t2); t_lsap.append(t4 - t3)
        if time.perf_counter() - t_start > 3 * budget_s:
            break
    med = lambda v: float(np.median(v))
    return dict(roi=med(t_roi), enc=med(t_enc), cost=med(t_cost), lsap=med(t_lsap), lit=med(t_lit),
                n_vec=len(t_roi), n_lit=len(t_lit))


def cpu_baseline(sc, sd, budget_s=20.0, frames_vec=20, frames_lit=6):
    """The reference's CPU path on this box's host cores, two modes (SURVEY.md
    8(d)), same inputs, 3 warm-up frames, per-frame medians:
      vectorised        oracle roi_align (C restatement of torchvision's CPU
                        kernel) + the fp32 encoder in plain torch + the oracle's
                        vectorised cost incl. gate (C) + scipy.optimize.linear_sum_assignment
      reference_literal the same roi_align / encoder / LSAP with the cost as the
                        reference's Python computes it: the per-track top-k loop
                        (mainTracking.py:173-210) and the per-pair 4x4-inverse
                        gating loop (:327-336) -- oracle/literal.py
    The headline (value) is c3's shape: one stream at N=256, 10x10 ROIs.  The literal
    mode's loops take seconds per frame, so its cost stage is sampled on frames_lit frames
    (the stages are timed separately and the medians added).  BASELINE.md §2's other CPU
    legs follow in `legs`: c1 (B=1, N=16, S=7 -- the reference tracker's own ROI size,
    tracking.py:304-309 -- and S=10) and c2 (N=64, S=10), on fewer frames.
    Threads: every physical core, capped by OMP_NUM_THREADS where the box sets it
    (16 on a one-GPU gpurun box: that GPU's CPU share); torch and the oracle's
    OpenMP loops (roi_align over ROIs, cost over track rows) use the same count."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import literal as LIT
    from scipy.optimize import linear_sum_assignment
    model, cores = _cpu_info()
    cap = os.environ.get("OMP_NUM_THREADS")
    thr = min(int(cap), cores or int(cap)) if cap else (cores or os.cpu_count() or 1)
    torch.set_num_threads(thr)
    os.environ.setdefault("OMP_NUM_THREADS", str(thr))  # the oracle's OpenMP (read at its first parallel loop)
    N = sc["N"]
    m = _cpu_leg(sc, sd, O, LIT, linear_sum_assignment, N, 10, frames_vec, frames_lit, budget_s)
    vec = m["roi"] + m["enc"] + m["cost"] + m["lsap"]
    lit = m["roi"] + m["enc"] + m["lit"] + m["lsap"]
    legs = {}
    for name, n, S in (("c1_n16_s7", 16, 7), ("c1_n16_s10", 16, 10), ("c2_n64_s10", 64, 10)):
        if n > N:
            continue
        g = _cpu_leg(sc, sd, O, LIT, linear_sum_assignment, n, S, 10, 3, budget_s / 4)
        gv = g["roi"] + g["enc"] + g["cost"] + g["lsap"]
        gl = g["roi"] + g["enc"] + g["lit"] + g["lsap"]
        legs[name] = {"N": n, "roi": S, "frames": g["n_vec"], "literal_cost_frames": g["n_lit"],
                      "vectorised": {"ms_per_frame": round(gv * 1e3, 2), "rois_per_s": round(n / gv, 2)},
                      "reference_literal": {"ms_per_frame": round(gl * 1e3, 2), "rois_per_s": round(n / gl, 2),
                                            "cost_ms": round(g["lit"] * 1e3, 2)},
                      "stages_ms": {k: round(g[k] * 1e3, 2) for k in ("roi", "enc", "cost", "lsap")}}
    return dict(value=round(N / vec, 2), unit="ROIs/s", cores=thr, kind="port",
                sample=f"one stream, N={N}, 3 warm-up frames, medians over {m['n_vec']} frames "
                       f"(literal cost stage: {m['n_lit']} frames): roi_align {m['roi'] * 1e3:.0f} ms (C, {thr} "
                       f"OpenMP threads) + fp32 encoder {m['enc'] * 1e3:.0f} ms (torch CPU, {thr} threads) + cost "
                       f"{m['cost'] * 1e3:.1f} ms (C, {thr} OpenMP threads) + scipy LSAP {m['lsap'] * 1e3:.1f} ms",
                cpu_model=model, physical_cores=cores,
                core_cap=(f"OMP_NUM_THREADS={cap} (the box's CPU share for this GPU)" if cap else None),
                modes={"vectorised": {"ms_per_frame": round(vec * 1e3, 1), "rois_per_s": round(N / vec, 2)},
                       "reference_literal": {"ms_per_frame": round(lit * 1e3, 1), "rois_per_s": round(N / lit, 2),
                                             "cost_ms": round(m["lit"] * 1e3, 1)}},
                legs=legs)


def timed_region(step, steps, dist, sync, red_dev, finish=None, own=None, mark=None):
    """Run `steps` steps between a barrier + device sync on both sides; return
    the MAX elapsed time over ranks (one all_reduce) and the step outputs
    (this rank's own elapsed time is appended to `own` if given).  mark: called
    right after the opening sync and after the closing one, outside the clock
    (prof_mark)."""
    if dist is not None:
        dist.barrier()
    sync()
    if mark is not None:
        mark()
    t0 = time.perf_counter()
    out = [step(k) for k in range(steps)]
    if finish is not None:
        finish()  # every frame's assignment indices read on the host
    sync()
    el = time.perf_counter() - t0
    if mark is not None:
        mark()
    if own is not None:
        own.append(el)
    if dist is not None:
        t = torch.tensor([el], device=red_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        dist.barrier()
    return el, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay the roi_align + encoder stage from hipGraphs (measured slower than eager "
                         "launches on the side stream, so off by default)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}")
    dist = None
    red_dev = None
    if world > 1:
        import torch.distributed as dist
        # RCCL ("nccl") over xGMI; TRK_DIST_BACKEND=gloo rehearses the multi-rank path with
        # several ranks on one device (RCCL refuses two ranks per GPU)
        backend = os.environ.get("TRK_DIST_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        if backend != "nccl":
            local %= max(1, ndev)
        elif local >= ndev:
            raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but {ndev} are visible "
                             f"(TRK_DIST_BACKEND=gloo shares devices between ranks)")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            red_dev = torch.device("cpu")  # gloo reduces host tensors
    dev = torch.device("cuda", local)
    if red_dev is None:
        red_dev = dev
    torch.cuda.set_device(dev)

    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_common as G
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    model = trk.Model(512, 512, 10, 128).eval()
    model.load_state_dict(sd, strict=True)
    model = model.to(dev)
    # TRK_FRONT=0: the two-kernel encoder front (g1dw4 -> Y2 in HBM -> gemm4<DSC>) instead of
    # rmb_front (one kernel, Y2 in LDS)
    model.fused_front = os.environ.get("TRK_FRONT", "1") == "1"

    # +depth frames: each step enqueues the embedding `depth` frames ahead (pipelining);
    # the syncs around the timed region make it do exactly `steps` embeddings (those of
    # frames first + depth .. last + depth) and `steps` assignments
    frames = PREROLL + args.warmup + args.steps + int(os.environ.get("TRK_PREFETCH_DEPTH", "1")) + 1
    sc = make_scenes(dev, args.streams, args.n, frames, seed=1000 + rank)
    pipe = Pipeline(sc, model)
    if args.graph:
        pipe.capture()
    f = 0
    for _ in range(PREROLL + args.warmup):
        pipe.step(f)
        f += 1

    probe = LiveProbe(pool=max(1024, 2 * 20 * (args.steps + 2)))
    probe.on = True
    pipe.tracker.sync_wait_s = 0.0
    own = []
    el, results = timed_region(lambda k: pipe.step(PREROLL + args.warmup + k), args.steps, dist,
                               torch.cuda.synchronize, red_dev, finish=pipe.tracker.drain, own=own, mark=prof_mark)
    el_own = own[0]
    probe.on = False
    kernel_sum = probe.sum_per_step_us(args.steps)
    live = probe.means_us()
    live = {k: v for k, v in live.items() if not k.endswith("_live")}
    tracker_live = {"lsap": probe.stage_means_us("lsap_live"), "cost": probe.stage_means_us("cost_live")}
    side_gap = probe.embed_gaps_us(len(pipe.sides), pipe.defer_head, pipe.roi_stream is not None)
    f = PREROLL + args.warmup + args.steps
    rois_total = args.steps * sc["streams"] * sc["N"] * world
    value = rois_total / el
    ident = float(np.mean([pipe.check_identity(PREROLL + args.warmup + k, r) for k, r in enumerate(results)]))

    pipe.close_progress()
    prof_mark()
    iso, M, iso_info = kernel_pass(pipe, f - 1)
    prof_mark()
    # per-launch device time: live (timed region) where probed, else isolated
    kt = dict(iso)
    kt.update(live)
    per_rank = [{"rank": rank, "device": str(dev), "elapsed_s": round(el_own, 6), "identity_rate": round(ident, 5),
                 "rois": args.steps * sc["streams"] * sc["N"]}]
    if dist is not None:  # after the timed region: which rank ran what (not a data-path collective)
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank[0])
        per_rank = gathered
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    Fs, N, S = sc["streams"], sc["N"], 10
    K = Fs * N
    # algorithmic work per launch: bytes that
    # must cross HBM and flops on the kernel's matrix core; the binding roof is
    # the larger of bytes / HBM peak and flops / MFMA peak
    R = K * S * S  # encoder rows
    algo = {  # name: (bytes, flops, mfma peak TFLOP/s)
        "roi_align": (Fs * 512 * 40 * 40 * 4 + K * 512 * S * S * 2 + K * 20, 0.0, BF16_PEAK_TFLOPS),
        "enc_g1_dwconv": (R * 512 * 2 + R * 1024 * 2 + 1024 * 512 * 2 + 25 * 1024 * 4,
                          2.0 * R * 1024 * 512 + 2.0 * R * 1024 * 25, BF16_PEAK_TFLOPS),
        "enc_gemm_dsc": (R * 1024 * 2 * 2 + 2 * 512 * 512 * 2 + K * 1024 * 8, 2.0 * R * 1024 * 512,
                         BF16_PEAK_TFLOPS),
        "enc_gemm_trans": (R * 1024 * 2 + 512 * 1024 * 2 + K * 512 * 12, 2.0 * R * 512 * 1024, BF16_PEAK_TFLOPS),
        # first 1x1 convs + depthwise + both DSC GEMMs in one kernel: X in, XRN + the squeeze
        # means out
        "enc_rmb_front": (R * 512 * 2 + R * 1024 * 2 + 2 * 1024 * 512 * 2 + 25 * 1024 * 4 + K * 1024 * 4,
                          2.0 * R * 1024 * 512 * 2 + 2.0 * R * 1024 * 25, BF16_PEAK_TFLOPS),
        "cost": (Fs * (M * 30 * 128 * 4 + N * 128 * 4 + M * N * 4), 2.0 * Fs * M * 30 * N * 128,
                 F32_MFMA_PEAK_TFLOPS),
    }
    # the encoder paths not taken in the timed region are still timed isolated (kernel_pass);
    # the dominant kernel is chosen among the ones the timed region ran (live-probed, plus the
    # ROI Align sweep and the cost build, which every step runs)
    ran = {k for k in algo if k in live} | {"roi_align", "cost"}
    per = {}
    for k, (byt, fl, mpeak) in algo.items():
        if k not in kt:
            continue
        t = kt[k] * 1e-6
        t_hbm, t_mfma = byt / (HBM_PEAK_GBS * 1e9), fl / (mpeak * 1e12)
        if t_hbm >= t_mfma:
            per[k] = dict(bound="hbm", us=round(kt[k], 2), achieved=round(byt / t / 1e9, 2), peak=HBM_PEAK_GBS,
                          unit="GB/s", frac=round(t_hbm / t, 4), work=byt)
        else:
            per[k] = dict(bound="mfma", us=round(kt[k], 2), achieved=round(fl / t / 1e12, 2), peak=mpeak,
                          unit="TFLOP/s", frac=round(t_mfma / t, 4), work=fl)
    if "cost" in per:
        per["cost"]["note"] = ("the exact f32 similarity's flops priced at the f32 MFMA peak; the kernel computes "
                               "them as three f16 MFMA products (cost_split 1, DESIGN 4.4), so this is the rate "
                               "an f32 chain would have to reach, not the f16 pipe's load")
    per["encoder_stage"] = dict(bound="mfma", us=round(kt["encoder"], 2),
                                achieved=round(K * ENC_FLOP_PER_ROI[S] / (kt["encoder"] * 1e-6) / 1e12, 2),
                                peak=BF16_PEAK_TFLOPS, unit="TFLOP/s",
                                frac=round(K * ENC_FLOP_PER_ROI[S] / (BF16_PEAK_TFLOPS * 1e12) / (kt["encoder"] * 1e-6), 4))
    # dominant hand-written kernel by measured time (LSAP is latency-bound: no roofline)
    dom = max(ran, key=lambda k: kt[k])
    # HBM traffic per launch from the committed rocprofv3 --pmc summary of this
    # bench (tools/gpu_pmc.sh -> profiles/pmc_traffic.json); null if absent
    traffic, tsrc = None, None
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as fh:
            pm = json.load(fh)
        e = pm["kernels"].get(dom)
        if e is not None:
            traffic = e["read_bytes"] + e["write_bytes"]
            tsrc = pm.get("profile", "profiles/pmc_traffic.json")
    except (OSError, KeyError, ValueError):
        pass
    t_iso = iso.get(dom)
    # the committed counter pass's timed window (profiles/pmc_clock.json, tools/pmc_clock.py): the
    # profiler runs each dispatch alone, so this is the kernel's own time at the clock it held
    ser = None
    try:
        with open(os.path.join(REPO, "profiles", "pmc_clock.json")) as fh:
            pc = json.load(fh)
        e = pc["timed"].get(dom)
        if e is not None:
            ser = {"time_us": e["avg_us"], "clock_ghz": e["clock_ghz"],
                   "frac": round(per[dom]["work"] / (e["avg_us"] * 1e-6) /
                                 (per[dom]["peak"] * (1e12 if per[dom]["unit"] == "TFLOP/s" else 1e9)), 4),
                   "source": pc.get("profile", "profiles/pmc_clock.json")}
    except (OSError, KeyError, ValueError, TypeError):
        pass
    rf = {"kernel": dom, "bound": per[dom]["bound"], "achieved": per[dom]["achieved"],
          "peak": per[dom]["peak"], "unit": per[dom]["unit"], "frac": per[dom]["frac"],
          "time_us": per[dom]["us"],
          "time_source": ("live: mean of the HIP-event pairs around this kernel's launches inside the timed "
                          "region, on the stream it is launched on (the same launches tools/kernel_stats.py "
                          "takes from a rocprofv3 trace: its timed window)" if dom in live else
                          "isolated: back-to-back launches after the timed region"),
          "time_note": ("with the two overlapping embedding streams a front's live window starts while the "
                        "previous frame's transition still holds CUs; 'serialised' is the kernel alone (a "
                        "counter pass runs each dispatch by itself), 'isolated' back to back (power-limited "
                        "clock), DESIGN.md section 6") if pipe.overlap else None,
          "isolated_time_us": None if t_iso is None else round(t_iso, 2),
          "isolated_frac": None if t_iso is None else round(per[dom]["work"] / (t_iso * 1e-6) /
                                                            (per[dom]["peak"] * (1e12 if per[dom]["unit"] == "TFLOP/s"
                                                                                 else 1e9)), 4),
          "serialised": ser,
          "traffic": traffic, "traffic_source": tsrc, "algorithmic_bytes_per_launch": algo[dom][0],
          "algorithmic_flops_per_launch": algo[dom][1], "kernel_us": {k: round(v, 2) for k, v in kt.items()},
          "kernel_us_source": {k: ("live: HIP events around each launch in the timed region (with two "
                                   "embedding streams a launch can share the GPU with the other frame's)"
                                   if k in live else "isolated: back-to-back launches after the timed region")
                               for k in kt},
          "isolated_us": {k: round(v, 2) for k, v in iso.items()},
          "isolated_note": dict(iso_info, note="lsap_dev_bound / lsap_dev_m: trk_lsap_dev on the step's stage-1 "
                                "matrices, its launch sized by the pipeline's row bound (live tracks + detections in "
                                "flight) or by the matrices' rows"),
          "per_kernel": per, "lsap_us_per_frame_batch": round(kt["lsap"], 2),
          "tracker_live_us_per_launch": dict(tracker_live, note="live HIP events in the timed region, per "
                                             "launch of all streams' frames; stage 2 = ReID-only rows (none "
                                             "matchable in this workload: the launch exits at once)"),
          "embed_stream_idle_us_per_step": None if side_gap is None else round(side_gap, 2)}
    # end-to-end ROIs/s against min(HBM / B_roi, MFMA / F_roi), with
    # B_roi = 12,800 (map share) + 2 x 102,400 (bf16 ROI tensor written + read) + 512
    # (embedding) + 16,900 (cost share) B and F_roi = the encoder's flops per ROI
    b_roi = Fs * 512 * 40 * 40 * 4 / K + 2 * 512 * S * S * 2 + 512 + 16900
    cap = min(HBM_PEAK_GBS * 1e9 / b_roi, BF16_PEAK_TFLOPS * 1e12 / ENC_FLOP_PER_ROI[S])
    rf["end_to_end"] = {"achieved": round(value / world, 1), "unit": "ROIs/s per GPU", "cap": round(cap, 1),
                        "frac": round(value / world / cap, 4), "bytes_per_roi": round(b_roi),
                        "flops_per_roi": ENC_FLOP_PER_ROI[S],
                        "cap_rule": "min(8 TB/s / bytes_per_roi, 2.5 PFLOP/s / flops_per_roi)"}
    # the encoder's flops per step over the step time: what the MFMA pipes achieve in the
    # pipeline, whatever the streams' overlap does to any one launch's event window
    enc_fl, ms = K * ENC_FLOP_PER_ROI[S], el / args.steps * 1e3
    rf["encoder_in_pipeline"] = {"achieved": round(enc_fl / (ms * 1e-3) / 1e12, 2), "unit": "TFLOP/s",
                                 "peak": BF16_PEAK_TFLOPS, "frac": round(enc_fl / (ms * 1e-3) / (BF16_PEAK_TFLOPS * 1e12), 4),
                                 "rule": "encoder flops per step (all ROIs of the step) / ms_per_step"}
    # PMC bytes over algorithmic bytes per kernel (committed profile), beside each stage's fraction
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as fh:
            pk = json.load(fh)["kernels"]
        rf["traffic_over_algorithmic"] = {k: round((pk[k]["read_bytes"] + pk[k]["write_bytes"]) / algo[k][0], 3)
                                          for k in algo if k in pk and k != "cost"}
        # the tracker's cost launches alternate stage 1 (M x N = 256 x 256 per stream) and
        # stage 2 (ReID-only rows x the detections stage 1 left: none in this workload, so
        # the launch exits at once): only stage 1 carries the algorithmic bytes
        if "cost_stage1" in pk:
            rf["traffic_over_algorithmic"]["cost_stage1"] = round(
                (pk["cost_stage1"]["read_bytes"] + pk["cost_stage1"]["write_bytes"]) / algo["cost"][0], 3)
    except (OSError, KeyError, ValueError):
        rf["traffic_over_algorithmic"] = None
    rf["env"] = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "HIP_LAUNCH_BLOCKING", "AMD_SERIALIZE_KERNEL",
                                                "AMD_SERIALIZE_COPY", "HIP_VISIBLE_DEVICES", "OMP_NUM_THREADS")
                 if os.environ.get(k) is not None}
    rf["streams"] = {"embed": len(pipe.sides), "embed_overlap": pipe.overlap, "head_on_track_stream": pipe.defer_head,
                     "roi_stream": pipe.roi_stream is not None, "roi_after": pipe.roi_after or None,
                     "roi_gate_frac": pipe.gate_frac if pipe.gate_frac < 1 else None,
                     "track_prio": pipe.track_stream is not None,
                     "prefetch_depth": pipe.depth, "graphs": pipe.graphs is not None,
                     "tuning": os.environ.get("TRK_TUNE") or None}
    step_us = el / args.steps * 1e6
    rf["step_breakdown"] = {
        "step_us": round(step_us, 1),
        "kernel_sum_us": round(kernel_sum, 1),
        "overlap": round(kernel_sum / step_us, 3),
        "host_wait_us": round(pipe.tracker.sync_wait_s / args.steps * 1e6, 1),
        "note": "kernel_sum = device time of every probed launch per step (live HIP events); overlap > 1 "
                "means streams ran concurrently; host_wait = time the host blocked reading frame results "
                "(back-pressure of the asynchronous tracker: at most 3 frames unread)"}
    line = {
        "metric": "ROIs/sec (roi_align->embed->cost->assign), N=256/frame, 1 GPU",
        "value": round(value, 1), "unit": "ROIs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16 encoder / f32 roi+cost / f64 KF+LSAP duals",
        "data": "synthetic (SiLU(randn) maps, moving boxes; seeded random encoder weights)",
        "config": {"workload": f"c3: {Fs} streams x N={N} detections/frame per GPU, [{Fs},512,40,40] "
                               f"{MAP_LAYOUT.upper()} maps, 10x10 ROIs, full tracker step (bank T=30, KF, "
                               f"2-stage assign)",
                   "streams_per_gpu": Fs, "N": N, "roi": S, "map_layout": MAP_LAYOUT,
                   "parallelism": f"replicas{world}"},
        "roofline": rf, "identity_rate": round(ident, 5),
        "ranks": {"launcher": ("torchrun" if os.environ.get("TORCHELASTIC_RUN_ID") else
                               "bench.py --gpus" if world > 1 else "single process"),
                  "backend": (os.environ.get("TRK_DIST_BACKEND", "nccl") if world > 1 else None),
                  "per_rank": per_rank},
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(sc, sd, args.cpu_budget)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
