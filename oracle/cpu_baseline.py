"""CPU baseline leg of bench.py (TEST/BENCH INFRASTRUCTURE ONLY — never the product path).

Times the repo's restatement of the reference's multiprocessing sampler
(milo/milo/sampler.py:87-130 over SimEnv.step, gym-simenv/gym_simenv/envs/sim_env.py:140-173,
with the mjrl MLP(32,32) numpy-noise policy) followed by the host relabel block
(mjrl/mjrl/algos/batch_reinforce.py:103-169: fit_cost over all samples, then per-trajectory
get_bonus_costs with the 4-model disagreement) on the host's cores.

The workers are forked with torch threads = 1 (forking after multi-threaded torch hung in
the survey probe), and inherit the model weights through module globals instead of pickling
40 MB of ensemble per task.  Must run before the process touches the GPU.
"""
from __future__ import annotations

import math
import multiprocessing as mp
import os
import time

import numpy as np
import torch

from . import milo_ref as R

_G = {}


def _work(i):
    torch.set_num_threads(1)
    g = _G
    env = R.SimEnvRef(g["ens"], g["norms"], horizon=g["horizon"])
    paths, n = R.get_samples(env, g["pw"], g["log_std"], g["quota"], 12345 + g["base_seed"] * i, g["table"])
    return paths


def run(S: int, A: int, hidden=(512, 512, 512, 512), n_models: int = 4, workers: int | None = None,
        samples: int = 20000, horizon: int = 300, expert_rows: int = 50000, feature_dim: int = 512,
        lambda_b: float = 0.0025, seed: int = 100, relabel: bool = True, relabel_threads: int | None = None,
        keep_paths: bool = False) -> dict:
    """Returns env-steps/s of the CPU sampler alone and (relabel=True) of sampler + relabel.
    The relabel runs in this process with `relabel_threads` torch threads (default: the
    worker count); the reference's relabel is one process with torch's default threading."""
    from amp_extensions_amd import synthetic as syn

    torch.set_num_threads(1)
    workers = workers or min(16, os.cpu_count() or 1)
    s, a, s2 = syn.offline(20000, S, A, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens = R.init_ensemble_weights(S, A, list(hidden), n_models, seed)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=seed, init_log_std=-0.25)
    table = syn.reset_table(4096, S, 1)
    _G.update(ens=ens, norms=norms, pw=pw, log_std=log_std, table=table, horizon=horizon,
              quota=math.ceil(samples / workers), base_seed=seed)
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        t0 = time.perf_counter()
        results = pool.map(_work, range(workers))
        t1 = time.perf_counter()
    paths = [p for r in results for p in r]
    n = sum(len(p["rewards"]) for p in paths)
    out = dict(samples=n, paths=len(paths), workers=workers, sampler_s=t1 - t0, sampler_steps_per_s=n / (t1 - t0))
    if keep_paths:
        out["_paths"] = paths
    if not relabel:
        return out
    threads = relabel_threads or workers
    rel = relabel_seconds(paths, S, A, hidden, n_models, expert_rows, feature_dim, lambda_b, seed, threads)
    out.update(relabel_threads=threads, relabel_s=rel, end_to_end_steps_per_s=n / ((t1 - t0) + rel))
    return out


def relabel_seconds(paths, S: int, A: int, hidden=(512, 512, 512, 512), n_models: int = 4, expert_rows: int = 50000,
                    feature_dim: int = 512, lambda_b: float = 0.0025, seed: int = 100, threads: int = 1) -> float:
    """Seconds of the host relabel (batch_reinforce.py:103-169: fit_cost over all samples, then
    per-path get_bonus_costs with the 4-model disagreement) over `paths`, with the reference's
    batching on `threads` torch threads.  The cost / ensemble setup is outside the timing."""
    from amp_extensions_amd import synthetic as syn
    torch.set_num_threads(threads)
    s, a, s2 = syn.offline(20000, S, A, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens = R.init_ensemble_weights(S, A, list(hidden), n_models, seed)
    expert = torch.from_numpy(syn.expert(expert_rows, S, 3))
    cost = R.RBFLinearCostRef(expert, feature_dim=feature_dim, bw_quantile=0.1, lambda_b=lambda_b, seed=seed)
    thr = R.compute_threshold(ens, norms, torch.from_numpy(s).float()[:4096], torch.from_numpy(a).float()[:4096])
    disc_fn = lambda st, ac: R.compute_discrepancy(ens, norms, st, ac)
    t2 = time.perf_counter()
    R.relabel_mmd(paths, cost, disc_fn, thr)
    t3 = time.perf_counter()
    torch.set_num_threads(1)
    return t3 - t2
