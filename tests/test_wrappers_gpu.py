"""Observation wrappers on the HIP path.

First block: the reference's own tests/test_rope_wrapper.py:34-113 (7 tests), restated against
this build's RotaryEmbedWrapper (a numpy DummyEnv, observation() / _apply_rope() run hwy_obs_pe
on the GPU).  Then golden comparisons with the reference wrappers' outputs, the fused
(in-step-kernel) path against the stand-alone kernel, and make_env's decision table."""

import os

import numpy as np
import pytest
import torch

from hwy import _abi
from hwy.gym import Env, spaces

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class DummyEnv(Env):
    def __init__(self, shape):
        super().__init__()
        self.observation_space = spaces.Box(low=-np.inf, high=np.inf, shape=shape, dtype=np.float32)
        self.action_space = spaces.Box(low=-1.0, high=1.0, shape=(1,), dtype=np.float32)

    def reset(self, *, seed=None, options=None):
        return np.zeros(self.observation_space.shape, dtype=np.float32), {}

    def step(self, action):
        return np.zeros(self.observation_space.shape, dtype=np.float32), 0.0, True, False, {}


from experiments.rope_embed import RotaryEmbedWrapper  # noqa: E402


def test_shape_preserved():
    w = RotaryEmbedWrapper(DummyEnv((5, 4)), rotate_dim=4, max_dist=10.0)
    obs = np.random.randn(5, 4).astype(np.float32)
    assert w.observation(obs).shape == obs.shape


def test_dtype_float32():
    w = RotaryEmbedWrapper(DummyEnv((3, 4)), rotate_dim=4, max_dist=10.0)
    assert w.observation(np.random.randn(3, 4).astype(np.float32)).dtype == np.float32


def test_identity_for_zero_distance():
    w = RotaryEmbedWrapper(DummyEnv((4, 4)), rotate_dim=4, max_dist=1.0)
    obs = np.zeros((4, 4), dtype=np.float32)
    obs[:, 2:] = np.random.randn(4, 2).astype(np.float32)
    assert np.allclose(w.observation(obs), obs, atol=1e-6)


def test_rotation_changes_values_for_nonzero_distance():
    w = RotaryEmbedWrapper(DummyEnv((4, 4)), rotate_dim=4, max_dist=1.0)
    obs = np.zeros((4, 4), dtype=np.float32)
    obs[:, 0] = 1.0
    out = w._apply_rope(obs.copy(), np.ones(4, dtype=np.float32))
    assert not np.allclose(out[:, :2], obs[:, :2])


def test_invertibility():
    w = RotaryEmbedWrapper(DummyEnv((6, 4)), rotate_dim=4, max_dist=1.0)
    obs = np.random.randn(6, 4).astype(np.float32)
    dn = np.random.rand(6).astype(np.float32)
    wrapped = w._apply_rope(obs.copy(), dn)
    assert np.allclose(w._apply_rope(wrapped, -dn), obs, atol=1e-6)


def test_default_rotate_dim_uses_full_features():
    assert RotaryEmbedWrapper(DummyEnv((4, 4)), max_dist=1.0).rotate_dim == 4


def test_invalid_rotate_dim_raises():
    with pytest.raises(ValueError):
        RotaryEmbedWrapper(DummyEnv((5, 4)), rotate_dim=3)
    with pytest.raises(ValueError):
        RotaryEmbedWrapper(DummyEnv((5, 4)), rotate_dim=6)


# ---------------------------------------------------------------- golden (reference outputs)
@pytest.fixture(scope="module")
def pe():
    return np.load(os.path.join(GOLD, "pe_wrappers.npz"))


def test_rope_wrapper_matches_reference(pe):
    for key in pe.files:
        p = key.split("_")
        if p[0] != "rope" or len(p) != 3:
            continue
        N, F = map(int, p[1].split("x"))
        rd = int(p[2][2:])
        w = RotaryEmbedWrapper(DummyEnv((N, F)), rotate_dim=rd)
        np.testing.assert_array_equal(w.inv_freq, pe[key + "_inv_freq"])
        got = np.stack([w.observation(o) for o in pe[f"obs_{p[1]}"]])
        np.testing.assert_allclose(got, pe[key], atol=1e-6, rtol=0, err_msg=key)
        got = np.stack([w._apply_rope(o, d) for o, d in zip(pe[f"obs_{p[1]}"], pe[key + "_dn"])])
        np.testing.assert_allclose(got, pe[key + "_applied"], atol=1e-6, rtol=0, err_msg=key)
        # batched call on a device tensor gives the same rows
        bt = w.observation(torch.as_tensor(pe[f"obs_{p[1]}"], device="cuda")).cpu().numpy()
        np.testing.assert_allclose(bt, pe[key], atol=1e-6, rtol=0)


def test_dist_wrapper_matches_reference(pe):
    from experiments.dist_embed import DistanceEmbedWrapper

    for key in pe.files:
        p = key.split("_")
        if p[0] != "dist" or len(p) != 3:
            continue
        N, F = map(int, p[1].split("x"))
        d = int(p[2][1:])
        w = DistanceEmbedWrapper(DummyEnv((N, F)), d_embed=d)
        np.testing.assert_array_equal(w._freqs_np, pe[key + "_freqs"])
        got = np.stack([w.observation(o) for o in pe[f"obs_{p[1]}"]])
        np.testing.assert_allclose(got, pe[key], atol=1e-6, rtol=0, err_msg=key)
        assert w.observation_space.shape == (N, F + d)


def test_rank_wrapper_matches_reference(pe):
    from experiments.rank_embed import RankEmbedWrapper

    for key in pe.files:
        p = key.split("_")
        if p[0] != "rank" or len(p) != 3:
            continue
        N, F = map(int, p[1].split("x"))
        d = int(p[2][1:])
        torch.manual_seed(1000 + d)  # same global-RNG draws as the reference's construction
        w = RankEmbedWrapper(DummyEnv((N, F)), d_embed=d)
        np.testing.assert_array_equal(w.table.weight.detach().numpy(), pe[key + "_weight"])
        got = np.stack([w.observation(o) for o in pe[f"obs_{p[1]}"]])
        np.testing.assert_allclose(got, pe[key], atol=1e-7, rtol=0, err_msg=key)


# ---------------------------------------------------------------- fused vs stand-alone
@pytest.mark.parametrize("cond,d", [("SHUFFLED_ROPE", 4), ("SHUFFLED_DISTPE", 4), ("SHUFFLED_RANKPE", 8)])
def test_fused_wrapper_equals_standalone_kernel(cond, d):
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env

    over = {"num_envs": 64, "observation": {"order": "shuffled"}}
    torch.manual_seed(0)
    wrapped = make_env(Condition[cond], HIGHWAY_CONFIG, d_embed=d, env_overrides=over)
    plain = make_env(Condition.SHUFFLED, HIGHWAY_CONFIG, env_overrides=over)
    assert wrapped._fused
    o1, _ = wrapped.reset(seed=5)
    o2, _ = plain.reset(seed=5)
    np.testing.assert_array_equal(o1.cpu().numpy(), wrapped.observation(o2).cpu().numpy())
    rng = np.random.default_rng(0)
    for _ in range(5):
        a = torch.as_tensor(np.tanh(rng.normal(size=(64, 2))).astype(np.float32), device="cuda")
        o1, r1, *_ = wrapped.step(a)
        o2, r2, *_ = plain.step(a)
        np.testing.assert_array_equal(o1.cpu().numpy(), wrapped.observation(o2).cpu().numpy())
        np.testing.assert_array_equal(r1.cpu().numpy(), r2.cpu().numpy())
    wrapped.close()
    plain.close()


def test_single_env_facade_runs_reference_loop_shape():
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env

    env = make_env(Condition.SHUFFLED_ROPE, HIGHWAY_CONFIG, d_embed=4)
    obs, info = env.reset(seed=43)
    assert obs.shape == (15, 4) and obs.dtype == np.float32
    total, steps, done = 0.0, 0, False
    while not done:
        obs, r, te, tr, _ = env.step(np.array([0.0, 0.0], np.float32))
        assert isinstance(r, float) and isinstance(te, bool)
        total += r
        steps += 1
        done = te or tr
    assert 1 <= steps <= env.unwrapped.max_episode_steps and 0 <= total <= steps
    # same seed -> same episode
    obs2, _ = env.reset(seed=43)
    o_again, _ = env.reset(seed=43)
    np.testing.assert_array_equal(obs2, o_again)
    env.close()
