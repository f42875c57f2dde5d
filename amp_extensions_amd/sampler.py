"""`sample_points` drop-in (milo/milo/sampler.py:87-130) over the GPU lane engine.

The reference forks `num_workers` processes, each stepping one SimEnv until it has
collected ceil(N / num_workers) samples in complete trajectories.  Here every lane of the
engine is a worker: lane b collects complete trajectories until its quota
ceil(N / lanes) is met, then idles (its transitions are no longer recorded).  The
return value has the reference's structure: a list of path dicts with float64
observations / next_observations / actions, rewards (0 from SimEnv), agent_infos
{mean, log_std, evaluation}, env_infos (one {} per step) and terminated = True.
Device RNG replaces the per-worker numpy seeds 12345 + base_seed * i, so actions are not
bit-identical to the reference's (parity is pinned with injected noise in the tests).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .rollout import RolloutEngine
from .sim_env import BatchedSimEnv


def _collect(eng: RolloutEngine, quota: int, mode: str, max_steps_total: int):
    """Run synchronous steps until every lane has met its quota; returns host paths."""
    B, S, A = eng.B, eng.ctx.S, eng.ctx.A
    # per-lane growing trajectory buffers on the host (the reference's python lists)
    cur = [dict(o=[], n=[], a=[], m=[]) for _ in range(B)]
    paths, samples, trajs = [], np.zeros(B, np.int64), np.zeros(B, np.int64)
    active = np.ones(B, bool)
    log_std = eng.policy.log_std_val
    eng.reset_all()
    steps = 0
    while active.any():
        if steps >= max_steps_total:
            raise RuntimeError("sample_points: step budget exhausted before every lane met its quota")
        eng.begin_rollout()
        K = eng.K
        for _ in range(K):
            eng.step()
        steps += K
        obs = eng.obs[:K].cpu().numpy()
        nxt = eng.next_obs[:K].cpu().numpy()
        act = eng.acts[:K].cpu().numpy()
        mean = eng.means[:K].cpu().numpy()
        done = eng.done[:K].cpu().numpy().astype(bool)
        for t in range(K):
            for b in np.nonzero(active)[0]:
                c = cur[b]
                c["o"].append(obs[t, b]); c["n"].append(nxt[t, b]); c["a"].append(act[t, b]); c["m"].append(mean[t, b])
                if done[t, b]:
                    T = len(c["o"])
                    m = np.array(c["m"], dtype=np.float32)
                    paths.append(dict(observations=np.array(c["o"]), next_observations=np.array(c["n"]),
                                      actions=np.array(c["a"]), rewards=np.zeros(T),
                                      agent_infos=dict(mean=m, log_std=np.tile(log_std, (T, 1)), evaluation=m),
                                      env_infos=[{} for _ in range(T)], terminated=True))
                    samples[b] += T
                    trajs[b] += 1
                    cur[b] = dict(o=[], n=[], a=[], m=[])
                    met = trajs[b] >= quota if mode == "trajectories" else samples[b] >= quota
                    if met:
                        active[b] = False
    return paths, int(samples.sum())


def sample_points(env, policy, num_to_collect: int, base_seed: int = 0, num_workers: int = 4, mode: str = "samples",
                  eval_mode: bool = False, verbose: bool = False, deepmimic: bool = False, max_steps_total=None):
    """milo.sampler.sample_points on the GPU.  `env` is a BatchedSimEnv (its lanes play the
    workers; `num_workers` is accepted for signature compatibility) and `policy` a
    DevicePolicy.  A missing info['valid'] counts as valid (SimEnv returns {}): the
    reference's deepmimic=True branch (sampler.py:61) would raise on SimEnv's info."""
    assert mode in ("samples", "trajectories")
    eng: RolloutEngine = env.engine if isinstance(env, BatchedSimEnv) else env
    if eng.means is None:
        raise ValueError("build the BatchedSimEnv with record_means=True for agent_infos")
    eng.policy = policy
    eng.eval_mode = eval_mode
    policy.seed = (12345 + int(base_seed)) & 0xFFFFFFFFFFFFFFFF
    quota = math.ceil(num_to_collect / eng.B)
    t0 = time.time()
    paths, n = _collect(eng, quota, mode, max_steps_total or 1000 * eng.term.horizon)
    if verbose:
        print(f"Collected {n} and {len(paths)} trajectories in {time.time() - t0} seconds")
    return paths
