"""bench.py host logic: a PMC pass's per-launch traffic is quoted only in a bench line whose
own run has the configuration the pass was measured on (an 8-rank line
carried Pong-N=1's conv2 bytes); otherwise the traffic fields are null with the reason."""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _cfg(**kw):
    d = dict(batch_size=512, n_actors=256, capacity=1_000_000, frame_store=True, env="synthetic",
             actor_steps_per_update=1, num_actions=6)
    d.update(kw)
    return SimpleNamespace(**d)


def test_traffic_only_for_the_measured_configuration(tmp_path, monkeypatch):
    import bench

    sig = bench.traffic_signature(1, _cfg(), True)
    prof = {"measured_on": sig, "conv2_learner_hbm_bytes_per_launch": 123,
            "hbm_bytes_per_launch": {"k_adam": 7}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "traffic_t.json").write_text(json.dumps(prof))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    p, src, why = bench.load_traffic_file("t", sig)
    assert why is None and p["hbm_bytes_per_launch"]["k_adam"] == 7
    assert bench.traffic_field(p, src, why, "conv2_learner_hbm_bytes_per_launch")[:2] == (123, src)
    v, s, r = bench.traffic_field(p, src, why, "gather_hbm_bytes_per_launch")
    assert v is None and s is None and "no gather_hbm_bytes_per_launch" in r
    # the 8-rank sharded line (32 actors, 125 k rows, B = 512, 8 actor steps per update)
    other = bench.traffic_signature(8, _cfg(n_actors=32, capacity=125_000, actor_steps_per_update=8), True)
    p, src, why = bench.load_traffic_file("t", other)
    assert p == {} and "world 1 vs 8" in why and "n_actors 256 vs 32" in why
    assert bench.traffic_field(p, src, why, "conv2_learner_hbm_bytes_per_launch") == (None, None, why)
    # Breakout, N = 1
    p, _, why = bench.load_traffic_file("t", bench.traffic_signature(1, _cfg(n_actors=2048, capacity=4_000_000,
                                                                             num_actions=4), True))
    assert p == {} and "num_actions 6 vs 4" in why
    # a pass that does not say what it measured is never quoted
    (tmp_path / "profiles" / "traffic_u.json").write_text(json.dumps({"conv2_learner_hbm_bytes_per_launch": 1}))
    p, _, why = bench.load_traffic_file("u", sig)
    assert p == {} and "does not record" in why
    p, src, why = bench.load_traffic_file("missing", sig)
    assert p == {} and src is None and "no PMC pass" in why


def test_committed_pass_records_its_configuration():
    """the default tag's committed PMC summary names the default command's configuration"""
    import bench

    with open(os.path.join(ROOT, "profiles", "traffic_r05.json")) as f:
        on = json.load(f)["measured_on"]
    assert on == bench.traffic_signature(1, _cfg(), True)
