"""Experiment conditions and hyper-parameter dataclasses.

API-compatible with the reference's experiments/config.py:9-70 (same enum members, field names,
defaults and cartesian sweep expansion) so sweep definitions written for the reference
(main.py:42-88) build the same Experiment list here.
"""

from __future__ import annotations

import itertools
from copy import deepcopy
from dataclasses import dataclass, field
from enum import Enum, auto
from typing import Any, Dict, List, Optional


class Condition(Enum):
    """Observation conditions swept by the study (reference experiments/config.py:9-14)."""

    SORTED = auto()
    SHUFFLED = auto()
    SHUFFLED_RANKPE = auto()
    SHUFFLED_DISTPE = auto()
    SHUFFLED_ROPE = auto()


@dataclass
class CommonHP:
    """Hyper-parameters shared by every condition (reference :17-27)."""

    gamma: float = 0.99
    lam: float = 0.95
    value_coef: float = 0.5
    entropy_coef: float = 0.005
    max_grad_norm: float = 0.5
    steps_per_update: int = 2048


@dataclass
class ConditionHP(CommonHP):
    """Per-condition hyper-parameters plus an optional sweep grid (reference :30-41)."""

    lr: float = 1e-4
    clip_eps: float = 0.2
    epochs: int = 6
    batch_size: int = 64
    hidden_dim: int = 128
    d_embed: Optional[int] = None
    sweep: Dict[str, List[Any]] = field(default_factory=dict)


@dataclass
class Experiment:
    """One training run (reference :44-55).

    ``extra`` is free-form; the vectorised runner reads ``num_envs`` (lockstep envs per GPU),
    ``rollout_len`` and ``num_minibatches`` from it, and the reference's ``log_interval`` /
    ``eval_interval``.
    """

    name: str
    condition: Condition
    hp: ConditionHP = field(default_factory=ConditionHP)
    seed: int = 42
    max_episodes: int = 1500
    target_reward: float = 130.0
    env_config_overrides: Dict[str, Any] = field(default_factory=dict)
    extra: Dict[str, Any] = field(default_factory=dict)


def expand_condition_hps(hp: ConditionHP) -> List[ConditionHP]:
    """Cartesian product over ``hp.sweep`` (keys in insertion order, reference :58-70)."""
    if not hp.sweep:
        return [hp]
    names = list(hp.sweep.keys())
    base = {k: v for k, v in deepcopy(vars(hp)).items() if k != "sweep"}
    out: List[ConditionHP] = []
    for combo in itertools.product(*(hp.sweep[n] for n in names)):
        params = dict(base)
        params.update(zip(names, combo))
        out.append(ConditionHP(**params))
    return out
