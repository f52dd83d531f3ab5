"""The profiling windows (tools/prof_window.py) and bench.timed_region's marker calls: a
rocprofv3 CSV of a whole bench run is split into the timed region's launches and the isolated
pass's by the four marker dispatches bench.py issues, whatever order the streams ran in."""
import csv
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import prof_window  # noqa: E402


def _csv(path, names):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for i, n in enumerate(names, 1):
            w.writerow([i, n, 1000 * i, 1000 * i + 10 * i])


def test_windows_split_by_markers(tmp_path):
    spin = "at::cuda::(anonymous namespace)::spin_kernel(long)"
    names = ["warm_a", "warm_b", spin, "(anonymous namespace)::rmb_front3_kernel(RfArgs)", "trans4_kernel<1, 2>",
             spin, "between", spin, "(anonymous namespace)::rmb_front3_kernel(RfArgs)", spin, "after"]
    _csv(tmp_path / "run_kernel_trace.csv", names)
    rows = prof_window.rows_of(str(tmp_path), "*kernel_trace.csv")
    assert prof_window.window_ids(rows) == {"timed": (3, 6), "isolated": (8, 10)}
    timed = [r["Kernel_Name"] for r in prof_window.select(rows, "timed")]
    assert timed == names[3:5]
    iso = [r["Kernel_Name"] for r in prof_window.select(rows, "isolated")]
    assert iso == names[8:9]
    assert prof_window.short_name(names[3]) == "enc_rmb_front"
    assert prof_window.short_name(names[4]) == "enc_gemm_trans"


def test_windows_need_four_markers(tmp_path):
    _csv(tmp_path / "run_kernel_trace.csv", ["a", "x::spin_kernel(long)", "b"])
    with pytest.raises(SystemExit):
        prof_window.window_ids(prof_window.rows_of(str(tmp_path), "*kernel_trace.csv"))


def test_kernel_stats_writes_both_windows(tmp_path):
    import kernel_stats
    spin = "spin_kernel(long)"
    _csv(tmp_path / "run_kernel_trace.csv", [spin, "k1", "k1", "k2", spin, spin, "k2", spin])
    old = sys.argv
    try:
        sys.argv = ["kernel_stats.py", str(tmp_path), str(tmp_path / "ks")]
        kernel_stats.main()
    finally:
        sys.argv = old
    rows = list(csv.DictReader(open(tmp_path / "ks_timed.csv")))
    assert {r["Name"]: int(r["Calls"]) for r in rows} == {"k1": 2, "k2": 1}
    rows = list(csv.DictReader(open(tmp_path / "ks_isolated.csv")))
    assert [(r["Name"], int(r["Calls"]), float(r["AverageNs"])) for r in rows] == [("k2", 1, 70.0)]


def test_timed_region_marks_outside_the_steps():
    import bench
    log = []
    el, out = bench.timed_region(lambda k: log.append(("step", k)) or k, 3, None, lambda: log.append("sync"),
                                 torch.device("cpu"), mark=lambda: log.append("mark"))
    assert out == [0, 1, 2]
    assert log == ["sync", "mark", ("step", 0), ("step", 1), ("step", 2), "sync", "mark"]
