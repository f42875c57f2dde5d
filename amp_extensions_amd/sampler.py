"""`sample_points` drop-in (milo/milo/sampler.py:87-130) over the GPU lane engine.

Reference contract (sampler.py:8-84, 112-130): W workers; worker i has quota q = ceil(N / W)
and collects complete trajectories one after another until it holds >= q samples (mode
'samples') or q trajectories (mode 'trajectories').  Trajectory j = 1, 2, ... of worker i is
seeded with s_ij = 12345 + base_seed * i + j: `env.seed_env(s_ij)` then `env.reset()` draws the
reset time t ~ U(0, time_max) from gym's np_random, and `np.random.seed(s_ij)` seeds the
policy's per-step draws (np.random.uniform() for the eps test, then randn(A)); the env's
reset counter makes trajectory j run on ensemble member j mod M.  The result lists worker
0's paths in order, then worker 1's, ...

Here a worker's trajectories run concurrently on GPU lanes.  Every trajectory is
exact-seeded (its reset time, noise and ensemble member depend only on (i, j)), so they can
run in any order and concurrency: trajectory j of worker i is admitted while the lengths its
predecessors have reached so far sum to less than q (a lower bound on the sum that decides
whether j is needed), dropped as soon as that bound reaches q, and the result is exactly
trajectories 1..n_i of the sequential reference, n_i = min{n : sum_{j <= n} len_j >= q}
('trajectories' mode: the first q).  How many run at once is set by an estimate of the
lengths still to come (the horizon R: the reference's worst case; or, speculatively, the
mean length of the trajectories ended so far), see _collect.  With rng='reference' every
trajectory's reset time and noise come from the reference's own seeds (the PCG64 reset draw
per trajectory; the MT19937 policy noise from per-lane generators in the HIP library's host
code, amx_mt_policy_noise, uploaded per chunk), so the output equals the reference's paths up
to the ensemble's fp32 arithmetic; rng='device' draws them from Philox on the GPU (same
structure and admission, different random streams, no host RNG work).

Lanes: W * ceil(q / R) lanes suffice for the worst-case rule (x4 with speculation), capped by
the env's lane count.  Steps run in chunks of K synchronous steps between host decisions,
replayed as one captured HIP graph per chunk; a lane whose trajectory ends inside a chunk
idles to its end.  The transitions of in-flight lanes are compacted on the device after every
chunk (one index gather into a transition store) and the store is reordered into path order
and copied to the host ONCE at the end; each path's arrays are views of that copy.
"""
from __future__ import annotations

import gc
import math
import threading
import time
import weakref

import numpy as np
import torch

from . import _native as N
from .rollout import RolloutEngine
from .sim_env import BatchedSimEnv


def _gym_np_random(seed: int) -> np.random.Generator:
    """gym 0.26.1 seeding.np_random(seed) (environment.yml:123): Generator(PCG64(SeedSequence))."""
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


class _Traj:
    __slots__ = ("worker", "j", "seed", "lane", "length", "ended", "segs")

    def __init__(self, worker: int, j: int, seed: int):
        self.worker, self.j, self.seed = worker, j, seed
        self.lane = -1
        self.length = 0       # transitions so far (the final length once ended)
        self.ended = False
        self.segs = []  # (store row, count) pieces in step order


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

    def append_from(self, src, idx: torch.Tensor) -> int:
        """Rows idx of the flat [K * L] chunk arrays src = (obs, next_obs, acts, means)."""
        m = idx.numel()
        if self.n + m > self.cap:
            self._alloc(max(2 * self.cap, self.n + m))
        s = slice(self.n, self.n + m)
        for dst, x in zip((self.obs, self.nxt, self.act, self.mean), src):
            torch.index_select(x, 0, idx, out=dst[s])
        base = self.n
        self.n += m
        return base

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


class _FreeLanes:
    """The idle lanes.  Member-blocked engines (RolloutEngine.member_blocks = Bq: lane b runs
    member b // Bq only) keep one list per member: trajectory j resets to member j mod M
    (sim_env.py:282-283 with the counter at j - 1), so it takes a lane of that block."""

    def __init__(self, L: int, M: int, Bq: int):
        self.M, self.Bq = M, Bq
        if Bq:
            self.lists = [list(range((g + 1) * Bq - 1, g * Bq - 1, -1)) for g in range(M)]
        else:
            self.lists = [list(range(L - 1, -1, -1))]

    def __bool__(self) -> bool:
        return any(self.lists)

    def take(self, j: int) -> int:
        """A lane for trajectory j (-1: none of its member's block is free)."""
        lst = self.lists[j % self.M if self.Bq else 0]
        return lst.pop() if lst else -1

    def put(self, lane: int) -> None:
        self.lists[lane // self.Bq if self.Bq else 0].append(lane)


def _reset_time_max(env) -> float:
    """The reset-time window [0, time_max) every trajectory's env.reset() draws from
    (sim_env.py:76-77, 276): reset_args['time_max'] when custom_time is on, else the clip length
    (a reset table: its length in rows).  A BatchedSimEnv keeps its reset_args; a RolloutEngine
    its reset_time_max (0: the whole source)."""
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    ra = getattr(env, "reset_args", None)
    if ra is not None and ra.get("custom_time"):
        return float(ra["time_max"])
    if float(getattr(src, "reset_time_max", 0.0) or 0.0) > 0.0:
        return float(src.reset_time_max)
    return src.motion.get_motion_length() if src.motion is not None else float(src.table.shape[0])


def _sampler_engine(env, lanes: int, K: int, policy, time_max: float, member_blocks: int = 0) -> RolloutEngine:
    """A lanes-sized engine on the env's ensemble, reset source and termination (cached per
    lane count, chunk, reset window and member blocking); its device-drawn motion resets use the
    env's window.  member_blocks = Bq > 0: lanes = M * Bq, lane b steps through member b // Bq
    only (RolloutEngine.member_blocks)."""
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    cache = src.__dict__.setdefault("_sampler_engines", {})
    key = (lanes, K, float(time_max), int(member_blocks))
    eng = cache.get(key)
    if eng is None:
        reset_source = src.motion if src.motion is not None else src.table
        eng = RolloutEngine(src.ens, reset_source, lanes=lanes, term=src.term, policy=policy, seed=src.seed,
                            max_steps=K, auto_reset=False, record_means=True)
        # (0 = the whole clip; a table source is already cut to the window's rows)
        if src.motion is not None and time_max != src.motion.get_motion_length():
            eng.reset_time_max = float(time_max)
        eng.member_blocks = int(member_blocks)
        cache[key] = eng
    # the env's reset_args noise (AddNoise) as it is NOW: a later set_reset_noise on the env
    # reaches the cached engine.  The noise draws come from Philox(engine seed; lane, reset#),
    # not from the trajectory seed, so with noise on, sample_points' paths depend on the lane
    # count and the admission order (the reference's own gRand stream is seeded from the wall
    # clock, util/Rand.cpp:8-9, so it is not reproducible either).
    eng._reset_noise = getattr(src, "_reset_noise", None)
    eng.policy = policy
    return eng


def _mjrl_fingerprint(policy) -> tuple:
    """The VALUES of every trainable tensor of an mjrl MLP (≈8.6 k floats at S = 197, a 34 KB
    copy per sample_points call).  Identities and version counters are not enough:
    set_param_values rebinds param.data (gaussian_mlp.py:67-85), but an optimizer step updates
    in place (behavior_cloning.py:125-132) and `p.data.add_()` / `p.data.copy_()` go through a
    `.data` alias whose version counter is not the parameter's, so only the values see every
    kind of update."""
    ts = [p.detach() for p in policy.model.parameters()] + [policy.log_std.detach()]
    vals = torch.cat([t.reshape(-1).to("cpu", torch.float64) for t in ts])
    return vals, np.asarray(policy.log_std_val).tobytes()


def _same_fingerprint(a: tuple, b: tuple) -> bool:
    return a[1] == b[1] and a[0].shape == b[0].shape and torch.equal(a[0], b[0])


def device_policy(env, policy):
    """`policy` as the sampler's DevicePolicy.  A DevicePolicy passes through; the reference's
    mjrl `MLP` (gaussian_mlp.py:7-104: `model.fc_layers`, `log_std`, `log_std_val`) is wrapped
    once (DevicePolicy.from_mjrl, cached on the object) and re-synced whenever its parameters
    changed since the last call, so batch_reinforce.py:88-90 passes its own policy unchanged."""
    from .policy import DevicePolicy
    if isinstance(policy, DevicePolicy):
        return policy
    model = getattr(policy, "model", None)
    if model is None or not hasattr(model, "fc_layers") or not hasattr(policy, "log_std"):
        raise TypeError(f"sample_points: policy must be a DevicePolicy or an mjrl MLP, got {type(policy).__name__}")
    if float(getattr(policy, "eps", 0.0) or 0.0) != 0.0:
        raise NotImplementedError("sample_points: mjrl MLP with eps > 0 (uniform random actions) is not supported")
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    ctx = src.ctx
    fp = _mjrl_fingerprint(policy)
    cached = policy.__dict__.get("_amx_device_policy")
    if cached is None or cached[0] is not ctx:
        dp = DevicePolicy.from_mjrl(ctx, policy)
        policy.__dict__["_amx_device_policy"] = (ctx, dp, fp)
        return dp
    _, dp, old = cached
    if not _same_fingerprint(old, fp):
        dp.sync_from([(l.weight.data, l.bias.data) for l in policy.model.fc_layers],
                     np.asarray(policy.log_std_val, np.float64))
        policy.__dict__["_amx_device_policy"] = (ctx, dp, fp)
    return dp


class _HostNoise:
    """Per-lane numpy-legacy MT19937 generators of the reference policy noise, advanced in the
    HIP library's host code (amx_mt_seed / amx_mt_policy_noise: bit-exact with
    np.random.seed(s); [np.random.uniform(); np.random.randn(A)] per step) into a pinned
    [K, L, A] buffer, one call per chunk for all lanes in flight."""

    def __init__(self, lib, L: int, K: int, A: int):
        self.lib, self.L, self.K, self.A = lib, L, K, A
        self.states = np.zeros((L, N.AMX_MT_STATE_BYTES), np.uint8)
        # pinned buffers: the next chunk's noise is drawn into one while another's upload and the
        # current chunk's steps run on the GPU (the pipelined collector rotates three: chunk
        # c + 1's draw starts before chunk c - 1 has been read back)
        pin = torch.cuda.is_available()
        self.bufs = [torch.zeros(K, L, A, dtype=torch.float64, pin_memory=pin) for _ in range(3)]
        self.cur = 0
        self.ahead = -1  # buffer already holding the continuing lanes' next draws (draw_async)
        self._thread, self._err = None, None

    def seed(self, lanes: np.ndarray, seeds: np.ndarray) -> None:
        sl = np.ascontiguousarray(lanes, np.int32)
        sd = np.asarray(seeds, np.int64)
        if sd.size and (sd.min() < 0 or sd.max() >= 2 ** 32):  # np.random.seed's own range check
            raise ValueError(f"Seed must be between 0 and 2**32 - 1 (sample_points trajectory seeds {sd.min()}..{sd.max()})")
        sd = np.ascontiguousarray(sd, np.uint32)
        N.check(self.lib.amx_mt_seed(self.states.ctypes.data, self.L, sl.ctypes.data, sd.ctypes.data, sl.size),
                "amx_mt_seed")

    def draw(self, lanes: np.ndarray, buf: torch.Tensor) -> torch.Tensor:
        """The next K steps' noise of `lanes` into their slots of `buf` (other slots untouched)."""
        sl = np.ascontiguousarray(lanes, np.int32)
        N.check(self.lib.amx_mt_policy_noise(self.states.ctypes.data, self.L, sl.ctypes.data, sl.size, self.K,
                                             self.A, buf.data_ptr(), self.L * self.A, self.A),
                "amx_mt_policy_noise")
        return buf

    # background draws (the pipelined collector): the next chunk's noise of the lanes in flight,
    # drawn on a host thread (the ctypes call releases the GIL) while the main thread reads the
    # previous chunk and admits; join() before any seed or draw touches the generator states
    def draw_async(self, lanes: np.ndarray, which: int) -> None:
        self.join()
        self._err = None

        def run():
            try:
                self.draw(lanes, self.bufs[which])
            except BaseException as e:  # re-raised by join()
                self._err = e
        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        self.ahead = which

    def join(self) -> None:
        th = getattr(self, "_thread", None)
        if th is not None:
            th.join()
            self._thread = None
            if self._err is not None:
                raise self._err


class _ChunkGraph:
    """The K synchronous steps of a chunk captured once as a HIP graph (the lanes' resets and
    the noise upload stay outside, on the same stream), so a chunk costs one replay instead of
    ~8 launches per step from Python."""

    def __init__(self, eng: RolloutEngine, K: int, noise_dev):
        c = eng.ctx
        # (a weak reference: the graph is cached on the engine, engine -> graph -> engine would be
        # a reference cycle that only the garbage collector frees)
        self.eng, self.K = weakref.proxy(eng), K
        self.g = torch.cuda.CUDAGraph()
        if eng._graph_ahead:
            eng.step_counter = int(eng.dev_step.item())
        eng.dev_step.fill_(eng.step_counter)
        side = torch.cuda.Stream(c.device)
        side.wait_stream(torch.cuda.current_stream(c.device))
        t0 = eng.t
        # no garbage collection during the capture: a collected cycle holding another graph or
        # device memory would be torn down in the middle of it (a HIP error / abort).  One
        # collection up front (torch.cuda.graph does the same), then the collector is off until
        # capture_end.  (capture_begin/end directly: torch.cuda.graph's context manager also
        # synchronises and empties the allocator cache, 13 ms per capture)
        gc.collect()
        gc_was_on = gc.isenabled()
        gc.disable()
        with torch.cuda.stream(side):
            eng._capturing = True
            self.g.capture_begin(capture_error_mode="thread_local")
            try:
                for k in range(K):
                    eng.step(noise=None if noise_dev is None else noise_dev[k])
                N.check(c.lib.amx_counter_add(c.h, eng.dev_step.data_ptr(), K, c.stream), "amx_counter_add")
            finally:
                self.g.capture_end()
                eng._capturing = False
                if gc_was_on:
                    gc.enable()
        torch.cuda.current_stream(c.device).wait_stream(side)
        eng.t, eng.step_counter = t0, eng.step_counter - K  # the captured steps did not run
        eng._graph_ahead = True

    def replay(self) -> None:
        self.g.replay()
        self.eng.t = self.K
        self.eng.step_counter += self.K
        self.eng._graph_ahead = True


# The device rows of the last sample_points call, in path order, beside the read-only host
# arrays they were copied to: relabel_paths (relabel.py:_device_rows) reads them instead of
# uploading the same bytes back when its paths are views of those host arrays.  One entry (the
# newest call); the host arrays are read-only, so the two copies cannot diverge.
_last_rows: dict = {}


def _to_host_path_order(perm: torch.Tensor, arrays, wait: bool = True):
    """The store's rows gathered into path order on the device, then ONE copy each into pinned
    host memory (2-4x the pageable .cpu() rate; torch's pinned-block cache reuses the blocks of
    paths the caller has dropped).  The returned numpy arrays keep their pinned tensors alive and
    are read-only (the reference's own code only reads the paths' arrays); the device rows of
    (observations, next observations, actions) stay registered in _last_rows.  wait=False:
    returns (arrays, event) with the copies still in flight (the event completes them)."""
    sel = [x.index_select(0, perm) for x in arrays]
    pin = torch.cuda.is_available()
    host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=pin) for t in sel]
    for h, t in zip(host, sel):
        h.copy_(t, non_blocking=pin)
    ev = None
    if pin:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(sel[0].device))
        if wait:
            ev.synchronize()
    out = [h.numpy() for h in host]
    for a in out:
        a.flags.writeable = False
    _last_rows.clear()
    _last_rows.update(observations=(out[0], sel[0]), next_observations=(out[1], sel[1]), actions=(out[2], sel[2]))
    return out if wait else (out, ev)


def _build_paths(trajs, store, eng: RolloutEngine, dev):
    """The trajectories' transitions in path order: one device gather, one asynchronous copy
    into pinned host memory, the path dicts built as views while it runs."""
    segs = [seg for tr in trajs for seg in tr.segs]
    starts = np.fromiter((b for b, _ in segs), np.int64, len(segs))
    lens = np.fromiter((n for _, n in segs), np.int64, len(segs))
    total = int(lens.sum())
    perm = np.repeat(starts - (np.cumsum(lens) - lens), lens) + np.arange(total, dtype=np.int64)
    pd = torch.from_numpy(perm).to(dev)
    host, copied = _to_host_path_order(pd, (store.obs, store.nxt, store.act, store.mean), wait=False)
    log_std = np.asarray(eng.policy.log_std_val, dtype=np.float64)
    # every step's log_std row (gaussian_mlp.py:102) as read-only broadcast views of one row
    ls_rows = np.broadcast_to(log_std, (total, log_std.shape[-1]))
    paths, off = [], 0
    for tr in trajs:
        T = tr.length
        sl = slice(off, off + T)
        m = host[3][sl]
        paths.append(dict(observations=host[0][sl], next_observations=host[1][sl], actions=host[2][sl],
                          rewards=np.zeros(T, dtype=np.int64),
                          agent_infos=dict(mean=m, log_std=ls_rows[sl], evaluation=m),
                          env_infos=[{} for _ in range(T)], terminated=True))
        off += T
    if copied is not None:
        copied.synchronize()
    return paths, off


def _chunk_graph(eng: RolloutEngine, K: int, noise_dev, eval_mode: bool) -> _ChunkGraph:
    """The chunk's captured graph, cached on the engine across sample_points calls: it bakes in
    the engine's and the policy's device buffers (persistent; DevicePolicy.sync_from rewrites
    them in place), the noise buffer, eval_mode and, for device-drawn noise, the policy seed."""
    pol = eng.policy
    key = (K, 0 if noise_dev is None else noise_dev.data_ptr(), bool(eval_mode), id(pol), pol.blob.data_ptr(),
           pol.noise_scale.data_ptr(), pol.H1, pol.H2, pol.seed if noise_dev is None else 0, bool(eng.fuse_assembly))
    cache = eng.__dict__.setdefault("_chunk_graphs", {})
    g = cache.get(key)
    if g is None:
        if len(cache) >= 4:  # (re-created policies: keep the newest few)
            cache.pop(next(iter(cache)))
        eng.begin_rollout()
        g = cache[key] = _ChunkGraph(eng, K, noise_dev)
    else:
        eng.begin_rollout()
        if eng._graph_ahead:
            eng.step_counter = int(eng.dev_step.item())
    return g


def _noise_buffer(eng: RolloutEngine, K: int, L: int, A: int) -> torch.Tensor:
    """The [K, L, A] device buffer of the uploaded reference noise (persistent per engine: the
    cached chunk graphs read it)."""
    buf = eng.__dict__.get("_noise_dev")
    if buf is None or tuple(buf.shape) != (K, L, A):
        buf = eng.__dict__["_noise_dev"] = torch.zeros(K, L, A, dtype=torch.float64, device=eng.ctx.device)
    return buf


def _collect(eng: RolloutEngine, W: int, quota: int, mode: str, base_seed: int, rng: str, eval_mode: bool,
             time_max: float, speculate: bool = True, graph: bool = True):
    """Run the W workers' trajectory sequences on the engine's lanes (see the module notes).

    Admission: a worker's trajectories are admitted in seed order j.  Trajectory j is needed iff
    the exact lengths of 1..j-1 sum to less than the quota q; the lengths reached so far give a
    lower bound LB_j of that sum, so j is admitted only while LB_j < q and an in-flight
    trajectory whose LB_j >= q is provably not needed and is dropped (its lane freed).  Among
    admissible trajectories the concurrency is capped by an estimate: sum over the admitted of
    (final length, or max(length so far, L^)) < q, with L^ = the horizon R (speculate=False: the
    reference's worst case, never wasted work) or the mean length of the trajectories ended so far
    (speculate=True: short trajectories admit more at once; any surplus trajectory completes or is
    dropped and never enters the result).  Each trajectory is exact-seeded, so its transitions do
    not depend on when or on which lane it ran: the result is trajectories 1..n_i of every worker,
    n_i = min{n : sum_{j <= n} len_j >= q}, for any admission order."""
    c = eng.ctx
    L, S, A, K, dev = eng.B, c.S, c.A, eng.K, c.device
    R = eng.term.horizon
    motion = eng.motion
    adm: list[list[_Traj]] = [[] for _ in range(W)]   # admitted trajectories, in j order
    next_j = [1] * W
    done_w = [False] * W
    lane_tr: list[_Traj | None] = [None] * L
    free = _FreeLanes(L, c.M, eng.member_blocks)
    store = _Store(dev, S, A, W * (quota + R) if mode == "samples" else W * quota * 64)
    eng.eval_mode = eval_mode
    ref_noise = rng == "reference" and not eval_mode
    hn = _HostNoise(c.lib, L, K, A) if ref_noise else None
    noise_dev = _noise_buffer(eng, K, L, A) if ref_noise else None
    pin = torch.cuda.is_available()
    # per-chunk reset inputs: staged in pinned memory, uploaded without a host wait
    mask_h = torch.zeros(L, dtype=torch.uint8, pin_memory=pin)
    counts_h = torch.zeros(L, dtype=torch.int32, pin_memory=pin)
    rows_h = torch.zeros(L, dtype=torch.float64 if motion is not None else torch.int32, pin_memory=pin)
    mask_dev = torch.empty(L, dtype=torch.uint8, device=dev)
    counts_dev = torch.empty(L, dtype=torch.int32, device=dev)
    rows_dev = torch.empty(L, dtype=rows_h.dtype, device=dev)
    mask_np, counts_np, rows_np = mask_h.numpy(), counts_h.numpy(), rows_h.numpy()
    pre_drawn = False
    ended_sum, ended_n = 0, 0
    chunk_graph = None
    chunks, budget = 0, 4 * (W * quota + W) * (R + K) // K + 64

    def drop(tr: _Traj) -> None:
        if tr.lane >= 0:
            lane_tr[tr.lane] = None
            free.put(tr.lane)
            tr.lane = -1

    while True:
        # ---- per worker: drop the unneeded, detect completion, admit (round-robin) ----
        # speculation: 2x the worst-case concurrency until lengths are known (lanes are nearly free
        # at these counts: the step time is latency-bound), then the mean ended length
        lhat = float(R) if not speculate else (ended_sum / ended_n if ended_n >= 4 else 0.5 * R)
        for w in range(W):
            if done_w[w]:
                continue
            trs = adm[w]
            if mode == "samples":
                lb, cut = 0, len(trs)
                for i, tr in enumerate(trs):
                    if lb >= quota:
                        cut = i
                        break
                    lb += tr.length
                for tr in trs[cut:]:
                    drop(tr)
                del trs[cut:]
                if trs and all(tr.ended for tr in trs) and sum(tr.length for tr in trs) >= quota:
                    done_w[w] = True
            elif len(trs) == quota and all(tr.ended for tr in trs):
                done_w[w] = True
        new = []
        # per worker: the lower bound (lengths so far) and the estimate, summed once per chunk
        # and extended as trajectories are admitted (a new one adds 0 and lhat)
        lbs, ests = [0] * W, [0.0] * W
        if mode == "samples":
            for w in range(W):
                if not done_w[w]:
                    lbs[w] = sum(tr.length for tr in adm[w])
                    ests[w] = sum(tr.length if tr.ended else max(tr.length, lhat) for tr in adm[w])
        progress = True
        while free and progress:
            progress = False
            for w in range(W):
                if not free or done_w[w]:
                    continue
                trs = adm[w]
                ok = (lbs[w] < quota and ests[w] < quota) if mode == "samples" else len(trs) < quota
                if ok:
                    j = next_j[w]
                    lane = free.take(j)
                    if lane < 0:  # (member-blocked: j waits for a lane of its member's block)
                        continue
                    next_j[w] += 1
                    tr = _Traj(w, j, 12345 + base_seed * w + j)
                    tr.lane = lane
                    lane_tr[tr.lane] = tr
                    trs.append(tr)
                    new.append(tr)
                    ests[w] += max(0, lhat)
                    progress = True
        active = np.array([b for b in range(L) if lane_tr[b] is not None], np.int64)
        if active.size == 0:
            break
        chunks += 1
        if chunks > budget:
            raise RuntimeError("sample_points: step budget exhausted (trajectories longer than the horizon?)")
        # ---- resets: the new trajectories (reset counter j-1 -> member j mod M) and the idle lanes ----
        eng.begin_rollout()
        mask_np.fill(1)
        mask_np[active] = 0
        counts_np.fill(0)
        new_lanes = np.array([tr.lane for tr in new], np.int64)
        for tr in new:
            mask_np[tr.lane] = 1
            counts_np[tr.lane] = tr.j - 1
            if rng == "reference":
                t = _gym_np_random(tr.seed).uniform(low=0, high=time_max)  # seed_env + reset (sim_env.py:132,276)
                rows_np[tr.lane] = t if motion is not None else int(np.floor(t))
        mask_dev.copy_(mask_h, non_blocking=True)
        counts_dev.copy_(counts_h, non_blocking=True)
        # reset lanes restart their counter at j - 1 (idle lanes at 0); the reset kernel adds one
        torch.where(mask_dev.bool(), counts_dev, eng.reset_count, out=eng.reset_count)
        if rng == "reference":
            rows_dev.copy_(rows_h, non_blocking=True)
        eng.reset_lanes(mask_dev, rows_dev if rng == "reference" else None)
        # ---- K synchronous steps ----
        if hn is not None:
            if new:
                hn.seed(new_lanes, np.array([tr.seed for tr in new]))  # np.random.seed (sampler.py:39)
            buf = hn.bufs[hn.cur]
            hn.draw(new_lanes if pre_drawn else active, buf)  # (the continuing lanes' noise is drawn)
            noise_dev.copy_(buf, non_blocking=True)
        # (the first chunk of a new shape allocates the workspaces: captured from the second on)
        if graph and chunk_graph is None and (chunks >= 2 or "_chunk_graphs" in eng.__dict__):
            chunk_graph = _chunk_graph(eng, K, noise_dev, eval_mode)
        if chunk_graph is not None:
            chunk_graph.replay()
        else:
            for k in range(K):
                eng.step(noise=None if noise_dev is None else noise_dev[k])
        if hn is not None:  # the next chunk's noise of the lanes in flight, while the GPU steps
            hn.cur ^= 1
            hn.draw(active, hn.bufs[hn.cur])
            pre_drawn = True
        done = eng.done[:K].cpu().numpy().astype(bool)  # [K, L]: the chunk's one host sync
        # ---- compact the in-flight lanes' transitions into the store (vectorised) ----
        d = done[:, active]
        hit = d.any(axis=0)
        n = np.where(hit, d.argmax(axis=0) + 1, K)
        tot = int(n.sum())
        starts = np.cumsum(n) - n
        step_of = np.arange(tot) - np.repeat(starts, n)
        flat = step_of * L + np.repeat(active, n)
        base = store.append(eng, K, torch.from_numpy(flat).to(dev))
        for i, b in enumerate(active.tolist()):
            tr = lane_tr[b]
            tr.segs.append((base + int(starts[i]), int(n[i])))
            tr.length += int(n[i])
            if hit[i]:
                tr.ended = True
                ended_sum += tr.length
                ended_n += 1
                drop(tr)
    # ---- reorder into path order on the device, one copy to the host ----
    trajs = [tr for w in range(W) for tr in adm[w]]
    if not trajs:
        return [], 0
    return _build_paths(trajs, store, eng, dev)



class _ChunkRing:
    """Two device copies of a chunk's K x L transitions: chunk i is copied into slot i % 2 right
    after its steps (no host information needed), so chunk i + 1 can be queued before chunk i's
    done flags are read; chunk i's rows are compacted from its slot one iteration later."""

    def __init__(self, eng: RolloutEngine, K: int):
        c = eng.ctx
        m = K * eng.B
        z = lambda w, dt: torch.empty(m, w, dtype=dt, device=c.device)
        self.slots = [(z(c.S, torch.float64), z(c.S, torch.float64), z(c.A, torch.float64), z(c.A, torch.float32))
                      for _ in range(2)]
        self.K, self.m = K, m

    def snapshot(self, eng: RolloutEngine, si: int) -> None:
        K, m = self.K, self.m
        for dst, src in zip(self.slots[si], (eng.obs, eng.next_obs, eng.acts, eng.means)):
            dst.copy_(src[:K].reshape(m, dst.shape[1]))


def _collect_pipelined(eng: RolloutEngine, W: int, quota: int, mode: str, base_seed: int, rng: str,
                       eval_mode: bool, time_max: float, speculate: bool = True, graph: bool = True):
    """_collect with the host one chunk behind the GPU: chunk i is queued (resets, noise, the
    captured steps, a raw copy of its transitions and an async copy of its done flags) before
    chunk i-1's done flags are read and its trajectories advanced.  Admission therefore sees
    the results through chunk i-2: a lane whose trajectory ended in chunk i-1 runs chunk i
    idle (its steps are never attributed: each chunk keeps the lane -> trajectory map it was
    launched with) and is re-admitted one chunk later.  Trajectories are exact-seeded, so the
    result is _collect's (the same trajectories 1..n_i per worker, the same transitions)."""
    c = eng.ctx
    L, S, A, K, dev = eng.B, c.S, c.A, eng.K, c.device
    R = eng.term.horizon
    motion = eng.motion
    adm: list[list[_Traj]] = [[] for _ in range(W)]
    next_j = [1] * W
    done_w = [False] * W
    lane_tr: list[_Traj | None] = [None] * L
    free = _FreeLanes(L, c.M, eng.member_blocks)
    store = _Store(dev, S, A, W * (quota + R) if mode == "samples" else W * quota * 64)
    ring = _ChunkRing(eng, K)
    eng.eval_mode = eval_mode
    ref_noise = rng == "reference" and not eval_mode
    hn = _HostNoise(c.lib, L, K, A) if ref_noise else None
    noise_dev = _noise_buffer(eng, K, L, A) if ref_noise else None
    pin = torch.cuda.is_available()
    # two sets of pinned staging: set i % 2 is rewritten only after chunk i - 2 has completed
    stage = []
    for _ in range(2):
        mh = torch.zeros(L, dtype=torch.uint8, pin_memory=pin)
        ch = torch.zeros(L, dtype=torch.int32, pin_memory=pin)
        rh = torch.zeros(L, dtype=torch.float64 if motion is not None else torch.int32, pin_memory=pin)
        dh = torch.zeros(K, L, dtype=torch.uint8, pin_memory=pin)
        fh = torch.zeros(K * L, dtype=torch.int64, pin_memory=pin)  # compaction indices (async upload)
        stage.append((mh, ch, rh, dh, torch.cuda.Event() if pin else None, fh,
                      torch.empty(K * L, dtype=torch.int64, device=dev)))
    mask_dev = torch.empty(L, dtype=torch.uint8, device=dev)
    counts_dev = torch.empty(L, dtype=torch.int32, device=dev)
    rows_dev = torch.empty(L, dtype=stage[0][2].dtype, device=dev)
    ended_sum, ended_n = 0, 0
    chunk_graph = None
    chunks, budget = 0, 4 * (W * quota + W) * (R + K) // K + 64
    pending = None  # (set index, [(lane, trajectory)]) of the queued, unread chunk

    def drop(tr: _Traj) -> None:
        if tr.lane >= 0:
            lane_tr[tr.lane] = None
            free.put(tr.lane)
            tr.lane = -1

    def process(p) -> None:
        nonlocal ended_sum, ended_n
        si, launched = p
        ev = stage[si][4]
        if ev is not None:
            ev.synchronize()
        # lanes whose trajectory is still running on them (not ended earlier, not dropped)
        live = [(b, tr) for b, tr in launched if not tr.ended and tr.lane == b]
        if not live:
            return
        lanes = np.array([b for b, _ in live], np.int64)
        d = stage[si][3].numpy().astype(bool)[:, lanes]  # [K, n live]
        hit = d.any(axis=0)
        n = np.where(hit, d.argmax(axis=0) + 1, K)
        starts = np.cumsum(n) - n
        step_of = np.arange(int(n.sum())) - np.repeat(starts, n)
        flat = step_of * L + np.repeat(lanes, n)
        # pinned + non_blocking: a pageable upload would wait for the chunk queued behind this one
        fh, fd = stage[si][5], stage[si][6]
        fh.numpy()[:flat.size] = flat
        fd[:flat.size].copy_(fh[:flat.size], non_blocking=True)
        base = store.append_from(ring.slots[si], fd[:flat.size])
        for i, (b, tr) in enumerate(live):
            tr.segs.append((base + int(starts[i]), int(n[i])))
            tr.length += int(n[i])
            if hit[i]:
                tr.ended = True
                ended_sum += tr.length
                ended_n += 1
                drop(tr)

    while True:
        lhat = float(R) if not speculate else (ended_sum / ended_n if ended_n >= 4 else 0.5 * R)
        for w in range(W):
            if done_w[w]:
                continue
            trs = adm[w]
            if mode == "samples":
                lb, cut = 0, len(trs)
                for i, tr in enumerate(trs):
                    if lb >= quota:
                        cut = i
                        break
                    lb += tr.length
                for tr in trs[cut:]:
                    drop(tr)
                del trs[cut:]
                if trs and all(tr.ended for tr in trs) and sum(tr.length for tr in trs) >= quota:
                    done_w[w] = True
            elif len(trs) == quota and all(tr.ended for tr in trs):
                done_w[w] = True
        new = []
        # per worker: the lower bound (lengths so far) and the estimate, summed once per chunk
        # and extended as trajectories are admitted (a new one adds 0 and lhat)
        lbs, ests = [0] * W, [0.0] * W
        if mode == "samples":
            for w in range(W):
                if not done_w[w]:
                    lbs[w] = sum(tr.length for tr in adm[w])
                    ests[w] = sum(tr.length if tr.ended else max(tr.length, lhat) for tr in adm[w])
        progress = True
        while free and progress:
            progress = False
            for w in range(W):
                if not free or done_w[w]:
                    continue
                trs = adm[w]
                ok = (lbs[w] < quota and ests[w] < quota) if mode == "samples" else len(trs) < quota
                if ok:
                    j = next_j[w]
                    lane = free.take(j)
                    if lane < 0:  # (member-blocked: j waits for a lane of its member's block)
                        continue
                    next_j[w] += 1
                    tr = _Traj(w, j, 12345 + base_seed * w + j)
                    tr.lane = lane
                    lane_tr[tr.lane] = tr
                    trs.append(tr)
                    new.append(tr)
                    ests[w] += max(0, lhat)
                    progress = True
        active = np.array([b for b in range(L) if lane_tr[b] is not None], np.int64)
        # nothing to admit and every trajectory in flight reaches the horizon inside the queued
        # chunk (its length through the chunks read back + K >= R): another chunk would only step
        # idle lanes -- read the queued one back first
        tail = (pending is not None and not new
                and all(lane_tr[b].length + K >= R for b in active.tolist()))
        if active.size == 0 or tail:
            if pending is None:
                break
            process(pending)  # the last queued chunk may end trajectories or free admissions
            pending = None
            continue
        chunks += 1
        if chunks > budget:
            raise RuntimeError("sample_points: step budget exhausted (trajectories longer than the horizon?)")
        si = chunks & 1
        mask_h, counts_h, rows_h, done_h, ev = stage[si][:5]
        mask_np, counts_np, rows_np = mask_h.numpy(), counts_h.numpy(), rows_h.numpy()
        eng.begin_rollout()
        mask_np.fill(1)
        mask_np[active] = 0
        counts_np.fill(0)
        new_lanes = np.array([tr.lane for tr in new], np.int64)
        for tr in new:
            mask_np[tr.lane] = 1
            counts_np[tr.lane] = tr.j - 1
            if rng == "reference":
                t = _gym_np_random(tr.seed).uniform(low=0, high=time_max)  # seed_env + reset (sim_env.py:132,276)
                rows_np[tr.lane] = t if motion is not None else int(np.floor(t))
        mask_dev.copy_(mask_h, non_blocking=True)
        counts_dev.copy_(counts_h, non_blocking=True)
        torch.where(mask_dev.bool(), counts_dev, eng.reset_count, out=eng.reset_count)
        if rng == "reference":
            rows_dev.copy_(rows_h, non_blocking=True)
        eng.reset_lanes(mask_dev, rows_dev if rng == "reference" else None)
        if hn is not None:
            nb = chunks % 3
            buf = hn.bufs[nb]
            if hn.ahead == nb:  # the lanes of the previous chunk were drawn in the background
                hn.join()
                hn.ahead = -1
                if new:
                    hn.seed(new_lanes, np.array([tr.seed for tr in new]))  # np.random.seed (sampler.py:39)
                    hn.draw(new_lanes, buf)
            else:
                hn.join()
                if new:
                    hn.seed(new_lanes, np.array([tr.seed for tr in new]))
                hn.draw(active, buf)  # the next K draws of every lane in flight (finished ones idle)
            noise_dev.copy_(buf, non_blocking=True)
        # (the first chunk of a new shape allocates the workspaces: captured from the second on)
        if graph and chunk_graph is None and (chunks >= 2 or "_chunk_graphs" in eng.__dict__):
            chunk_graph = _chunk_graph(eng, K, noise_dev, eval_mode)
        if chunk_graph is not None:
            chunk_graph.replay()
        else:
            for k in range(K):
                eng.step(noise=None if noise_dev is None else noise_dev[k])
        ring.snapshot(eng, si)
        done_h.copy_(eng.done[:K], non_blocking=True)
        if ev is not None:
            ev.record()
        if hn is not None:
            # the next chunk's draws of this chunk's lanes, on a host thread while chunk c - 1 is
            # read back (buffer (c + 1) % 3 last served chunk c - 2, whose upload completed before
            # process() returned for it); a lane that ends or is dropped is re-seeded and re-drawn
            # if admitted again, so its surplus draws are never used
            hn.draw_async(active, (chunks + 1) % 3)
        launched = [(int(b), lane_tr[b]) for b in active.tolist()]
        if pending is not None:
            process(pending)
        pending = (si, launched)
    if hn is not None:
        hn.join()
    trajs = [tr for w in range(W) for tr in adm[w]]
    if not trajs:
        return [], 0
    return _build_paths(trajs, store, eng, dev)

def sample_points(env, policy, num_to_collect: int, base_seed: int = 0, num_workers: int = 4, mode: str = "samples",
                  eval_mode: bool = False, verbose: bool = False, deepmimic: bool = False, rng: str = "reference",
                  chunk: int = 16, speculate: bool = True, graph: bool = True, pipeline: bool = True,
                  member_blocked: bool = True):
    """milo.sampler.sample_points on the GPU.  `env` is a BatchedSimEnv (or a RolloutEngine):
    its ensemble, reset source, reset-time window (reset_args custom_time / time_max) and
    termination are used, and its lane count caps the concurrency; `policy` a DevicePolicy or
    the reference's mjrl MLP (wrapped and kept in sync by device_policy).  Returns the reference's list of path dicts
    (observations / next_observations / actions float64, rewards 0, agent_infos {mean,
    log_std, evaluation}, env_infos, terminated).  A missing info['valid'] counts as valid
    (SimEnv returns {}; the reference's deepmimic=True branch, sampler.py:61, would raise).
    `speculate`: admit beyond the worst-case reservation from the observed trajectory lengths
    (same result, see _collect); `graph`: replay each chunk's steps as a captured HIP graph;
    `pipeline`: queue chunk i before reading chunk i-1's done flags (same result,
    _collect_pipelined); `member_blocked` (f16x3 ensembles with M >= 2): every lane steps through
    its trajectory's member only, as SimEnv.step does (the engine's lanes in M blocks of a
    multiple of 128; a quarter of the ensemble rows per step at M = 4), instead of all M members
    on every lane (same paths up to the GEMM's fp32 rounding)."""
    assert mode == "samples" or mode == "trajectories"
    if rng not in ("reference", "device"):
        raise ValueError("rng must be 'reference' or 'device'")
    src = env.engine if isinstance(env, BatchedSimEnv) else env
    W = int(num_workers)
    quota = math.ceil(num_to_collect / W)  # sampler.py:113
    R = src.term.horizon
    need = W * (math.ceil(quota / R) if mode == "samples" else quota)
    if speculate and mode == "samples":
        need *= 4  # room for trajectories shorter than the horizon (lengths ~R/4) to run at once
    lanes = max(1, min(need, src.B))
    M = src.ctx.M
    Bq = 0
    if member_blocked and M >= 2 and src.ens.W2 is not None:
        # member blocks of a multiple of 128 lanes, rounded down: the lanes in flight at once stay
        # well below the speculative estimate (~125 of 544 at 40 000 samples), and a member's
        # single 128-row tile runs the 8-wave small-row GEMM (68 vs 85 us per forward at 256)
        Bq = max(128, math.ceil(need / M) // 128 * 128)
        while Bq > 128 and M * Bq > max(src.B, M * 128):
            Bq -= 128
        lanes = M * Bq
    K = max(1, min(int(chunk), R))
    time_max = _reset_time_max(env)
    policy = device_policy(env, policy)
    eng = _sampler_engine(env, lanes, K, policy, time_max, Bq)
    if rng == "device":
        policy.seed = (12345 + int(base_seed)) & 0xFFFFFFFFFFFFFFFF
    t0 = time.time()
    collect = _collect_pipelined if pipeline else _collect
    paths, n = (collect(eng, W, quota, mode, int(base_seed), rng, eval_mode, time_max, speculate=speculate,
                        graph=graph)
                if quota > 0 else ([], 0))
    if verbose:
        print(f"Collected {n} and {len(paths)} trajectories in {time.time() - t0} seconds")
    return paths
