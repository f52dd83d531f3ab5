"""Multi-rank path of bench.py on CPU (gloo, world size 2).

The path shards by video stream with no data-path collective:
each rank owns its own streams; the only communication is the barrier pair and
one MAX all_reduce of the elapsed time around the timed region.  These tests
run that exact code (`bench.timed_region`) in two gloo processes and check the
aggregate bookkeeping, plus that ranks build disjoint synthetic workloads.
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    import bench
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        calls = []

        def step(k):  # rank r's steps take (r + 1) * 20 ms
            time.sleep(0.02 * (rank + 1))
            calls.append(k)
            return rank * 100 + k

        el, out = bench.timed_region(step, 3, tdist, lambda: None, torch.device("cpu"))
        # per-rank workload: different seeds -> different boxes, same shapes
        sc = bench.make_scenes(torch.device("cpu"), 2, 8, 3, seed=1000 + rank, C=4, H=8)
        q.put((rank, el, out, calls, sc["np"]["rois"].copy()))
    finally:
        tdist.destroy_process_group()


@pytest.mark.timeout(300)
def test_timed_region_max_over_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, el, out, calls, rois = q.get(timeout=240)
        res[r] = (el, out, calls, rois)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # every rank ran exactly its own steps, in order
    for r in (0, 1):
        assert res[r][2] == [0, 1, 2]
        assert res[r][1] == [r * 100 + k for k in range(3)]
    # both ranks report the same elapsed time: the slowest rank's (3 x 40 ms)
    assert res[0][0] == res[1][0]
    assert res[0][0] >= 3 * 0.04 - 1e-3
    # replicas: the ranks' workloads are independent (different boxes)
    assert res[0][3].shape == res[1][3].shape
    assert not np.array_equal(res[0][3], res[1][3])


# --------------------------------------------- per-rank replicas, real steps ----
def _replica_steps(rank, frames=5, streams=2, N=10):
    """One rank's replica of the bench workload on the CPU: bench.make_scenes with the
    rank's seed (1000 + rank, as bench.main), then per step and stream the reference's
    CPU path restated -- oracle roi_align -> fp32 encoder -> oracle/tracker_ref
    (Tracking.update) -- returning (step fn, scene, trackers)."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import bench
    import gen_common as G
    import oracle as O
    import tracker_ref as TR
    sc = bench.make_scenes(torch.device("cpu"), streams, N, frames, seed=1000 + rank, pool=2)
    sd = {k: torch.from_numpy(v) for k, v in G.seeded_state_dict_np(0).items()}
    trackers = [TR.TrackerRef() for _ in range(streams)]

    def step(f):
        fmap = bench.frame_map(sc, f).numpy()
        out = []
        for s in range(streams):
            rois = sc["np"]["rois"][f, s * N:(s + 1) * N].copy()
            rois[:, 0] = 0
            roi = O.roi_align(fmap[s:s + 1], rois, (10, 10), 40 / 1280.0, 2, True)
            with torch.no_grad():
                emb = O.encoder_forward(sd, torch.from_numpy(roi)).numpy()
            box, conf = sc["np"]["dbox"][f, s], sc["np"]["dconf"][f, s]
            m, ut, ud = trackers[s].update(list(emb), box.tolist(), conf.tolist())
            out.append((m, ut, ud))
        return out
    return step, sc


def _identity(sc, results):
    """fraction of matches that keep the object their track first matched
    (bench.Pipeline.check_identity's rule), over frames 1.."""
    ids, ok, tot = {}, 0, 0
    for f, res in enumerate(results):
        for s, (m, _, _) in enumerate(res):
            for tid, j in m:
                o = int(sc["obj"][f, s][j])
                ids.setdefault((s, tid), o)
                ok += ids[(s, tid)] == o
                tot += 1
    return ok / max(tot, 1), tot


def _replica_worker(rank, world, port, q):
    torch.set_num_threads(2)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import bench
        step, sc = _replica_steps(rank)
        step(0)  # warm-up frame: every track is born here
        el, out = bench.timed_region(lambda k: step(k + 1), 4, tdist, lambda: None, torch.device("cpu"))
        q.put((rank, el, out, sc["np"]["rois"].copy()))
    finally:
        tdist.destroy_process_group()


@pytest.mark.timeout(300)
def test_replicas_run_real_steps_gloo():
    """Two gloo ranks each build their own bench workload (make_scenes, rank seed) and
    run real tracker steps -- ROI Align, encoder, the reference's Tracking.update, all
    restated on the CPU -- inside bench.timed_region: one barrier pair and one MAX
    all-reduce, no data-path collective.  Each rank's results equal the same replica
    run alone in this process (replicas are independent), tracks keep their objects,
    and the two ranks' workloads differ."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, el, out, rois = q.get(timeout=240)
        res[r] = (el, out, rois)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]  # MAX over ranks
    assert not np.array_equal(res[0][2], res[1][2])
    torch.set_num_threads(4)
    for r in (0, 1):
        step, sc = _replica_steps(r)
        alone = [step(f) for f in range(5)]
        assert res[r][1] == alone[1:], r
        ident, nmatch = _identity(sc, alone)
        assert nmatch >= 4 * 2 * 8 and ident == 1.0, (r, ident, nmatch)


def test_timed_region_single_process():
    sys.path.insert(0, REPO)
    import bench
    el, out = bench.timed_region(lambda k: k * k, 4, None, lambda: None, torch.device("cpu"))
    assert out == [0, 1, 4, 9] and el >= 0.0


def test_scene_shapes_and_bounds():
    sys.path.insert(0, REPO)
    import bench
    sc = bench.make_scenes(torch.device("cpu"), 3, 16, 5, seed=7, C=4, H=8)
    rois = sc["np"]["rois"]
    assert rois.shape == (5, 48, 5)
    assert set(np.unique(rois[..., 0]).astype(int)) == {0, 1, 2}
    w = rois[..., 3] - rois[..., 1]
    h = rois[..., 4] - rois[..., 2]
    assert (w > 20).all() and (w < 340).all() and (h > 20).all() and (h < 340).all()
    # every frame's detections are a permutation of the stream's objects
    for f in range(5):
        for s in range(3):
            assert sorted(sc["obj"][f, s]) == list(range(16))


# ------------------------------------------------- bench.py --gpus N launcher ----
def _bench_cmd(*extra):
    import subprocess
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *extra], capture_output=True,
                          text=True, timeout=600, cwd=REPO,
                          env=dict(os.environ, TRK_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1"))


def test_bench_gpus_disagrees_with_world_size():
    """--gpus that disagrees with a torchrun WORLD_SIZE fails loudly, before the GPU is touched"""
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, cwd=REPO,
                       env=dict(os.environ, WORLD_SIZE="3", RANK="0"))
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE=3" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus_2_spawns_ranks_running_the_pipeline():
    """`bench.py --gpus 2` with no WORLD_SIZE starts two rank processes itself (gloo on
    the one leased GPU here; RCCL, one GPU per rank, on a node), each running the real
    Pipeline on its own 8 streams; rank 0 prints one JSON line for the whole job"""
    import json
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    r = _bench_cmd("--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "replicas2"
    assert line["ranks"]["launcher"] == "bench.py --gpus" and line["ranks"]["backend"] == "gloo"
    pr = line["ranks"]["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert all(p["rois"] == 3 * 8 * 256 and p["identity_rate"] == 1.0 for p in pr), pr
    # value = all ranks' ROIs / the slowest rank's time
    assert abs(line["value"] - 2 * 3 * 8 * 256 / max(p["elapsed_s"] for p in pr)) <= 0.01 * line["value"]
