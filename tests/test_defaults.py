"""Reference tests/test_defaults.py:4-17, against this build's utils.defaults."""

from utils.defaults import feature_count, max_dist, max_rank


def test_defaults_match_config():
    from config.base_config import HIGHWAY_CONFIG as C

    rng = C["observation"]["features_range"]
    assert max_dist() == max(abs(rng["x"][0]), abs(rng["x"][1]), abs(rng["y"][0]), abs(rng["y"][1]))
    assert max_rank() == C["observation"]["vehicles_count"]
    assert feature_count() == len(C["observation"]["features"])
