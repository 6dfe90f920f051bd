"""Gymnasium 1.x API surface used by the reference (Env, Wrapper, ObservationWrapper, spaces.Box).

gymnasium is a dependency of the reference (uv.lock:140-151) but is not installed in this image;
when it is importable its classes are used, so wrappers built here are real gymnasium wrappers.
Otherwise this module provides the same minimal surface with gymnasium's semantics.
"""

from __future__ import annotations

from typing import Any, Optional, Tuple

import numpy as np

try:  # pragma: no cover - gymnasium absent in this image
    import gymnasium as _gym
    from gymnasium import Env, ObservationWrapper, Wrapper, spaces  # noqa: F401

    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class _Spaces:
        class Box:
            """gymnasium.spaces.Box (shape, dtype, low/high broadcasting)."""

            def __init__(self, low, high, shape=None, dtype=np.float32):
                dtype = np.dtype(dtype)
                if shape is None:
                    shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
                shape = tuple(int(s) for s in shape)
                self.shape = shape
                self.dtype = dtype
                self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
                self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()

            def sample(self, rng: Optional[np.random.Generator] = None):
                rng = rng or np.random.default_rng()
                lo = np.where(np.isfinite(self.low), self.low, -1.0)
                hi = np.where(np.isfinite(self.high), self.high, 1.0)
                return rng.uniform(lo, hi, self.shape).astype(self.dtype)

            def contains(self, x) -> bool:
                x = np.asarray(x)
                return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

            def __repr__(self) -> str:
                return f"Box({self.shape}, {self.dtype})"

    spaces = _Spaces()

    class Env:
        """gymnasium.Env: reset(*, seed, options) -> (obs, info); step(a) -> 5-tuple."""

        observation_space: Any = None
        action_space: Any = None
        metadata: dict = {"render_modes": []}
        spec = None

        def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
            return None, {}

        def step(self, action):
            raise NotImplementedError

        def close(self):
            pass

        @property
        def unwrapped(self):
            return self

    class Wrapper(Env):
        def __init__(self, env):
            self.env = env
            self.observation_space = env.observation_space
            self.action_space = env.action_space

        def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
            return self.env.reset(seed=seed, options=options)

        def step(self, action):
            return self.env.step(action)

        def close(self):
            return self.env.close()

        @property
        def unwrapped(self):
            return self.env.unwrapped

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            return getattr(self.env, name)

    class ObservationWrapper(Wrapper):
        def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None) -> Tuple:
            obs, info = self.env.reset(seed=seed, options=options)
            return self.observation(obs), info

        def step(self, action):
            obs, r, te, tr, info = self.env.step(action)
            return self.observation(obs), r, te, tr, info

        def observation(self, observation):
            raise NotImplementedError
