"""`sample_points` drop-in (milo/milo/sampler.py:87-130) over the GPU lane engine.

Reference contract (sampler.py:8-84, 112-130): W workers; worker i has quota q = ceil(N / W)
and collects complete trajectories one after another until it holds >= q samples (mode
'samples') or q trajectories (mode 'trajectories').  Trajectory j = 1, 2, ... of worker i is
seeded with s_ij = 12345 + base_seed * i + j: `env.seed_env(s_ij)` then `env.reset()` draws the
reset time t ~ U(0, time_max) from gym's np_random, and `np.random.seed(s_ij)` seeds the
policy's per-step draws (np.random.uniform() for the eps test, then randn(A)); the env's
reset counter makes trajectory j run on ensemble member j mod M.  The result lists worker
0's paths in order, then worker 1's, ...

Here a worker's trajectories run concurrently on GPU lanes.  Trajectory j+1 of worker i is
admitted to a free lane only while completed_i + R * in_flight_i < q (R = horizon, the longest
a trajectory can run; 'trajectories' mode: count_i + in_flight_i < q).  An admitted j
therefore has sum_{j' < j} len_j' < q, and admission continues until completed_i >= q with
nothing in flight: the admitted set is exactly trajectories 1..n_i of the sequential
reference, n_i = min{n : sum_{j <= n} len_j >= q}, whatever the lane timing.  With
rng='reference' every trajectory's reset time and noise come from the reference's own seeds
(host MT19937 / PCG64 draws, uploaded per chunk), so the output equals the reference's
paths up to the ensemble's fp32 arithmetic; rng='device' draws them from Philox on the GPU
(same structure and admission, different random streams, no host RNG work).

Lanes: W * ceil(q / R) lanes suffice for the admission rule (each in-flight trajectory
reserves R samples), capped by the env's lane count.  Steps run in chunks of K synchronous
steps between host decisions; a lane whose trajectory ends inside a chunk idles to its end.
The transitions of in-flight lanes are compacted on the device after every chunk (index
gather into a transition store) and the store is reordered into path order and copied to
the host ONCE at the end; each path's arrays are views of that copy.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .rollout import RolloutEngine
from .sim_env import BatchedSimEnv


def _gym_np_random(seed: int) -> np.random.Generator:
    """gym 0.26.1 seeding.np_random(seed) (environment.yml:123): Generator(PCG64(SeedSequence))."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


class _Traj:
    __slots__ = ("worker", "j", "seed", "rs", "lane", "length", "segs")

    def __init__(self, worker: int, j: int, seed: int):
        self.worker, self.j, self.seed = worker, j, seed
        self.rs = None
        self.lane = -1
        self.length = 0
        self.segs = []  # (store row, count) pieces in step order


def _noise_block(rs: np.random.RandomState, K: int, A: int) -> np.ndarray:
    """K steps of MLP.get_action's draws (gaussian_mlp.py:99-102): np.random.uniform() for the
    eps test, then randn(A) -- in the legacy stream order of np.random.seed(s_ij)."""
    out = np.empty((K, A))
    for k in range(K):
        rs.random_sample()
        out[k] = rs.standard_normal(A)
    return out


class _Store:
    """Device transition store (compacted lane rows), grown geometrically."""

    def __init__(self, dev, S: int, A: int, cap: int):
        self.dev, self.S, self.A, self.n = dev, S, A, 0
        self._alloc(max(cap, 1024))

    def _alloc(self, cap: int):
        old = getattr(self, "obs", None)
        z = lambda w, dt: torch.empty(cap, w, dtype=dt, device=self.dev)
        new = (z(self.S, torch.float64), z(self.S, torch.float64), z(self.A, torch.float64), z(self.A, torch.float32))
        if old is not None:
            for dst, src in zip(new, (self.obs, self.nxt, self.act, self.mean)):
                dst[:self.n].copy_(src[:self.n])
        self.obs, self.nxt, self.act, self.mean = new
        self.cap = cap

    def append(self, eng: RolloutEngine, K: int, idx: torch.Tensor) -> int:
        m = idx.numel()
        if self.n + m > self.cap:
            self._alloc(max(2 * self.cap, self.n + m))
        L = eng.B
        s = slice(self.n, self.n + m)
        torch.index_select(eng.obs[:K].reshape(K * L, self.S), 0, idx, out=self.obs[s])
        torch.index_select(eng.next_obs[:K].reshape(K * L, self.S), 0, idx, out=self.nxt[s])
        torch.index_select(eng.acts[:K].reshape(K * L, self.A), 0, idx, out=self.act[s])
        torch.index_select(eng.means[:K].reshape(K * L, self.A), 0, idx, out=self.mean[s])
        base = self.n
        self.n += m
        return base


def _sampler_engine(env, lanes: int, K: int, policy) -> RolloutEngine:
    """A lanes-sized engine on the env's ensemble, reset source and termination (cached)."""
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    cache = src.__dict__.setdefault("_sampler_engines", {})
    eng = cache.get((lanes, K))
    if eng is None:
        reset_source = src.motion if src.motion is not None else src.table
        eng = RolloutEngine(src.ens, reset_source, lanes=lanes, term=src.term, policy=policy, seed=src.seed,
                            max_steps=K, auto_reset=False, record_means=True)
        cache[(lanes, K)] = eng
    eng.policy = policy
    return eng


def _collect(eng: RolloutEngine, W: int, quota: int, mode: str, base_seed: int, rng: str, eval_mode: bool):
    c = eng.ctx
    L, S, A, K, dev = eng.B, c.S, c.A, eng.K, c.device
    R = eng.term.horizon
    reserve = R if mode == "samples" else 1
    motion = eng.motion
    time_max = motion.get_motion_length() if motion is not None else float(eng.table.shape[0])
    st = [dict(next_j=1, completed=0, ntraj=0, inflight=0, done=[]) for _ in range(W)]
    free = list(range(L - 1, -1, -1))
    active: dict[int, _Traj] = {}
    store = _Store(dev, S, A, W * (quota + R) if mode == "samples" else W * quota * 64)
    eng.eval_mode = eval_mode

    def admissible(w: int) -> bool:
        s = st[w]
        have = s["completed"] if mode == "samples" else s["ntraj"]
        return have + reserve * s["inflight"] < quota

    noise_dev = torch.zeros(K, L, A, dtype=torch.float64, device=dev) if rng == "reference" else None
    mask_dev = torch.empty(L, dtype=torch.uint8, device=dev)
    steps, budget = 0, (W * quota + W) * (R + K) + 16 * K
    while True:
        # ---- admit trajectories to free lanes (round-robin over the workers) ----
        new = []
        progress = True
        while free and progress:
            progress = False
            for w in range(W):
                if free and admissible(w):
                    s = st[w]
                    tr = _Traj(w, s["next_j"], 12345 + base_seed * w + s["next_j"])
                    s["next_j"] += 1
                    s["inflight"] += 1
                    tr.lane = free.pop()
                    active[tr.lane] = tr
                    new.append(tr)
                    progress = True
        if not active:
            break
        if steps > budget:
            raise RuntimeError("sample_points: step budget exhausted (trajectories longer than the horizon?)")
        # ---- resets: the new trajectories (reset counter j-1 -> member j mod M) and the idle lanes ----
        eng.begin_rollout()
        mask = np.zeros(L, np.uint8)
        idle = [b for b in range(L) if b not in active]
        mask[idle] = 1
        counts = np.zeros(L, np.int32)
        rows = np.zeros(L, np.float64 if motion is not None else np.int32)
        for tr in new:
            mask[tr.lane] = 1
            counts[tr.lane] = tr.j - 1
            if rng == "reference":
                t = _gym_np_random(tr.seed).uniform(low=0, high=time_max)  # seed_env + reset (sim_env.py:132,276)
                rows[tr.lane] = t if motion is not None else int(np.floor(t))
                tr.rs = np.random.RandomState(tr.seed)                   # np.random.seed (sampler.py:39)
        if mask.any():
            sel = torch.from_numpy(np.nonzero(mask)[0]).to(dev)
            eng.reset_count.index_copy_(0, sel, torch.from_numpy(counts[mask != 0]).to(dev))
            mask_dev.copy_(torch.from_numpy(mask))
            rows_dev = torch.from_numpy(rows).to(dev) if rng == "reference" else None
            eng.reset_lanes(mask_dev, rows_dev)
        # ---- K synchronous steps ----
        if noise_dev is not None and not eval_mode:
            nz = np.zeros((K, L, A))
            for lane, tr in active.items():
                nz[:, lane] = _noise_block(tr.rs, K, A)
            noise_dev.copy_(torch.from_numpy(nz))
        for k in range(K):
            eng.step(noise=None if noise_dev is None else noise_dev[k])
        steps += K
        done = eng.done[:K].cpu().numpy().astype(bool)  # [K, L]: the chunk's one host sync
        # ---- compact the in-flight lanes' transitions into the store ----
        idx, pieces = [], []
        for lane, tr in active.items():
            hit = np.nonzero(done[:, lane])[0]
            n = int(hit[0]) + 1 if hit.size else K
            idx.append(np.arange(n) * L + lane)
            pieces.append((tr, n, bool(hit.size)))
        flat = np.concatenate(idx)
        base = store.append(eng, K, torch.from_numpy(flat).to(dev))
        for tr, n, ended in pieces:
            tr.segs.append((base, n))
            base += n
            tr.length += n
            if ended:
                s = st[tr.worker]
                s["inflight"] -= 1
                s["completed"] += tr.length
                s["ntraj"] += 1
                s["done"].append(tr)
                del active[tr.lane]
                free.append(tr.lane)
    # ---- reorder into path order on the device, one copy to the host ----
    trajs = [tr for s in st for tr in sorted(s["done"], key=lambda x: x.j)]
    if not trajs:
        return [], 0
    perm = np.concatenate([np.arange(b, b + n) for tr in trajs for (b, n) in tr.segs])
    pd = torch.from_numpy(perm).to(dev)
    host = [x.index_select(0, pd).cpu().numpy() for x in (store.obs, store.nxt, store.act, store.mean)]
    log_std = np.float64(eng.policy.log_std_val)
    paths, off = [], 0
    for tr in trajs:
        T = tr.length
        sl = slice(off, off + T)
        m = host[3][sl]
        paths.append(dict(observations=host[0][sl], next_observations=host[1][sl], actions=host[2][sl],
                          rewards=np.zeros(T, dtype=np.int64),
                          agent_infos=dict(mean=m, log_std=np.tile(log_std, (T, 1)), evaluation=m),
                          env_infos=[{} for _ in range(T)], terminated=True))
        off += T
    return paths, off


def sample_points(env, policy, num_to_collect: int, base_seed: int = 0, num_workers: int = 4, mode: str = "samples",
                  eval_mode: bool = False, verbose: bool = False, deepmimic: bool = False, rng: str = "reference",
                  chunk: int = 8):
    """milo.sampler.sample_points on the GPU.  `env` is a BatchedSimEnv (or a RolloutEngine):
    its ensemble, reset source and termination are used, and its lane count caps the
    concurrency; `policy` a DevicePolicy.  Returns the reference's list of path dicts
    (observations / next_observations / actions float64, rewards 0, agent_infos {mean,
    log_std, evaluation}, env_infos, terminated).  A missing info['valid'] counts as valid
    (SimEnv returns {}; the reference's deepmimic=True branch, sampler.py:61, would raise)."""
    assert mode == "samples" or mode == "trajectories"
    if rng not in ("reference", "device"):
        raise ValueError("rng must be 'reference' or 'device'")
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    W = int(num_workers)
    quota = math.ceil(num_to_collect / W)  # sampler.py:113
    R = src.term.horizon
    need = W * (math.ceil(quota / R) if mode == "samples" else quota)
    lanes = max(1, min(need, src.B))
    K = max(1, min(int(chunk), R))
    eng = _sampler_engine(env, lanes, K, policy)
    if rng == "device":
        policy.seed = (12345 + int(base_seed)) & 0xFFFFFFFFFFFFFFFF
    t0 = time.time()
    paths, n = _collect(eng, W, quota, mode, int(base_seed), rng, eval_mode) if quota > 0 else ([], 0)
    if verbose:
        print(f"Collected {n} and {len(paths)} trajectories in {time.time() - t0} seconds")
    return paths
