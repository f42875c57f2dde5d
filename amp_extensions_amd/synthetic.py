"""Synthetic humanoid3d-shaped workload (there is no network for the reference's offline /
expert datasets, README.md:26).  Distributions follow SURVEY §8d:

  offline set  s ~ 0.5 N(0,1) with s[:,0] (root y) ~ U(0.8, 0.95), a ~ N(0,1),
               s' = s + 0.01 N(0,1)                                     (normalizers, threshold)
  reset table  same distribution, then every fall body's relative y lifted to
               |y| + 0.2 so a lane starts standing (the DeepMimicCore reset poses of
               SimEnv.reset are not available; documented deviation)
  expert       [s, s'] rows of the same distribution (the 'ss' expert buffer)

Seeds: 0 normalizers/offline, 1 reset table, 3 expert buffer, 100+k ensemble members,
100 policy, 100 RFF cost (run.py --seed 100 as in the README command).
"""
from __future__ import annotations

import numpy as np

from .humanoid import FALL_BODIES


def offline(n: int, S: int, A: int, seed: int = 0):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def reset_table(n: int, S: int, seed: int = 1, pos_dim: int = 3, rot_dim: int = 6) -> np.ndarray:
    s, _, _ = offline(n, S, 1, seed)
    for b in FALL_BODIES:
        j = (pos_dim + rot_dim) * b + 2   # relative y of body b (sim_env.py:103-104, :185)
        if j < S:
            s[:, j] = np.abs(s[:, j]) + 0.2
    return s


def expert(n: int, S: int, seed: int = 3) -> np.ndarray:
    s, _, s2 = offline(n, S, 1, seed)
    return np.concatenate([s, s2], axis=1).astype(np.float32)
