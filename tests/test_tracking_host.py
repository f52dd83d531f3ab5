"""Host-side tracker logic that needs no GPU: configuration resolution."""
import os


def test_tracker_conf_defaults_are_conf_yaml_values(trk):
    c = trk.tracker_conf({})
    # conf.yaml values, not mainTracking.py's in-code defaults
    assert c["hist_max"] == 30 and c["max_age"] == 120 and c["lost_reid_after"] == 50
    assert c["cost_update_max"] == 30.0 and c["reid_only_cost_max"] == 0.4
    assert abs(trk.tracker_conf({"reid_sim_min": 0.7})["reid_only_cost_max"] - 0.3) < 1e-12


def test_tracker_conf_from_yaml(trk, tmp_path):
    p = tmp_path / "conf.yaml"
    p.write_text("tracker:\n  hist_max: 12\n  emb_top_k: 3\n")
    c = trk.tracker_conf(conf_path=str(p))
    assert c["hist_max"] == 12 and c["emb_top_k"] == 3 and c["w_bbox"] == 0.3
    bad = tmp_path / "bad.yaml"
    bad.write_text("model: {}\n")
    import pytest
    with pytest.raises(KeyError, match="tracker"):
        trk.tracker_conf(conf_path=str(bad))


def test_lsap_status_mapping():
    """LSAP statuses: -1 / -2 raise ValueError like scipy; -3 (an internal solver
    stall) and the tracker step's launch-bound / capacity statuses are library
    errors, never reported as an infeasible matrix."""
    import pytest
    from conftest import pkg
    trk = pkg()
    ops = __import__(trk.__name__ + ".ops", fromlist=["x"])
    tracking = __import__(trk.__name__ + ".tracking", fromlist=["x"])
    ops.lsap_check_status(0)
    with pytest.raises(ValueError, match="invalid numeric"):
        ops.lsap_check_status(-1)
    with pytest.raises(ValueError, match="infeasible"):
        ops.lsap_check_status(-2)
    with pytest.raises(trk.TrkError, match="stalled"):
        ops.lsap_check_status(-3)
    with pytest.raises(tracking.SolverStallError):
        tracking._raise_status(-3, 0)
    for st in (-4, -5):
        with pytest.raises(trk.TrkError) as ei:
            tracking._raise_status(st, 2)
        assert not isinstance(ei.value, ValueError)
    with pytest.raises(ValueError, match="infeasible"):
        tracking._raise_status(-2, 0)
