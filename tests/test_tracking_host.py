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
