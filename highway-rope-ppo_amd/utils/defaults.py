"""
utils.defaults (reference utils/defaults.py:1-23)
Central place to pull default hyper-parameters from HIGHWAY_CONFIG so that all wrappers stay in
sync with the env definition.
"""

from config.base_config import HIGHWAY_CONFIG as _CFG


def max_dist() -> float:
    """Largest |x| or |y| the observation clip allows (metres)."""
    rng = _CFG["observation"]["features_range"]
    return max(abs(rng["x"][0]), abs(rng["x"][1]), abs(rng["y"][0]), abs(rng["y"][1]))


def max_rank() -> int:
    """Number of rows returned by the observation (ego included)."""
    return _CFG["observation"]["vehicles_count"]


def feature_count() -> int:
    """Number of scalar features per vehicle row."""
    return len(_CFG["observation"]["features"])
