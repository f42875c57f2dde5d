"""Drop-in env surfaces over the rollout engine.

* `SimEnv`        — gym_simenv's single learned-dynamics env (gym-simenv/gym_simenv/envs/
                    sim_env.py:13-288): same constructor arguments, step/reset/seed_env/
                    get_observation/set_observation/is_done, reward 0 and info {}.
* `BatchedSimEnv` — B of them in lock-step on the GPU (vectorised-env semantics:
                    done lanes auto-reset; the returned observation is the pre-reset s').

Reset source: SimEnv.reset asks DeepMimicCore for the state at a random motion time
t ~ U(0, motion_length) (sim_env.py:276-280).  With a `ReferenceMotion` the facade draws t
exactly as the reference does (np_random.uniform(0, time_max), time_max = the clip length)
and the state is computed on the device from the clip (csrc/amx_motion.hip); with a
reset-state table (the synthetic benchmark) it uses row floor(t) of the table.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from .engine import AmxContext
from .humanoid import BODY_DEFS, FALL_BODIES, HORIZON, TerminationConfig
from .rollout import RolloutEngine


class Box:
    """Minimal stand-in for gym.spaces.Box (gym is not a dependency of the engine)."""

    def __init__(self, low, high, dtype=np.float64):
        self.low, self.high = np.asarray(low, dtype), np.asarray(high, dtype)
        self.shape, self.dtype = self.low.shape, np.dtype(dtype)


def termination_from_args(deepmimic_args: str | None, horizon: int, enable_velocity_check: bool) -> TerminationConfig:
    """Read the ctrl flags and BodyDefs the reference reads (sim_env.py:84-115) when the
    DeepMimic arg file is available; otherwise the humanoid3d spinkick defaults."""
    cfg = TerminationConfig(horizon=horizon, enable_velocity_check=enable_velocity_check)
    if not deepmimic_args or not os.path.exists(deepmimic_args):
        return cfg
    args = {}
    key = None
    for tok in open(deepmimic_args).read().split():
        if tok.startswith("--"):
            key = tok[2:]
            args[key] = []
        elif key is not None:
            args[key].append(tok)
    base = os.path.dirname(os.path.abspath(deepmimic_args))

    def _resolve(p):
        for cand in (p, os.path.join(base, p), os.path.join(os.getcwd(), p)):
            if os.path.exists(cand):
                return cand
        return None

    ctrl = _resolve(args.get("char_ctrl_files", [""])[0]) if args.get("char_ctrl_files") else None
    if ctrl:
        cj = json.load(open(ctrl))
        cfg.record_vel_as_pos = bool(cj.get("RecordVelAsPos", False))
        cfg.record_all_world = bool(cj.get("RecordAllWorld", False))
        cfg.record_world_root_pos = bool(cj.get("RecordWorldRootPos", False))
        if "UpdateRate" in cj:
            cfg.sampling_rate = 1.0 / float(cj["UpdateRate"])
    char = _resolve(args.get("character_files", [""])[0]) if args.get("character_files") else None
    if char:
        hj = json.load(open(char))
        defs = hj["BodyDefs"]
        cfg.body_defs = {i: (d["Shape"], float(d["Param0"]), float(d["Param1"])) for i, d in enumerate(defs)}
    return cfg


class SimEnv:
    """gym_simenv SimEnv (sim_env.py:13-288) on the HIP engine, one lane."""

    def __init__(self, dynamic_ensemble, deepmimic_args=None, enable_velocity_check=False, horizon=HORIZON,
                 device=None, seed=None, reset_args=None, reset_table=None):
        """`reset_table`: a [R, S] reset-state table (row floor(t)), or a `ReferenceMotion`
        (amp_extensions_amd.motion): the state at motion time t computed on the device as
        DeepMimicCore's reset_time(t) builds it."""
        if reset_table is None:
            raise ValueError("SimEnv needs a reset source: a ReferenceMotion or a reset_table")
        self.dynamic_ensemble = dynamic_ensemble
        dev_ens = getattr(dynamic_ensemble, "device", dynamic_ensemble)
        self.enable_velocity_check = enable_velocity_check
        self.horizon = horizon
        self.term = termination_from_args(deepmimic_args, horizon, enable_velocity_check)
        self._eng = RolloutEngine(dev_ens, reset_table, lanes=1, term=self.term, seed=0, max_steps=1,
                                  auto_reset=False)
        c = self._eng.ctx
        self.state_size, self.action_size = c.S, c.A
        self.observation_space = Box([-np.inf] * c.S, [np.inf] * c.S)
        self.action_space = Box([-np.inf] * c.A, [np.inf] * c.A)
        self.motion = self._eng.motion
        # sim_env.py:77: time_max = the motion length (a table's length in rows otherwise)
        self.time_max = self.motion.get_motion_length() if self.motion is not None else \
            float(np.asarray(reset_table).shape[0])
        self.ob = None
        self.num_steps = 0
        self.reset_counter = 0
        self.seed_env(seed)

    def seed_env(self, seed=None):
        """sim_env.py:122-132 (gym 0.26 seeding: Generator(PCG64(SeedSequence(seed))))."""
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))

    def get_observation(self):
        return self.ob

    def set_observation(self, value):
        self.ob = value
        self._eng.obs[0, 0].copy_(torch.as_tensor(np.asarray(value, np.float64)))

    def step(self, action):
        """sim_env.py:140-162: one learned-dynamics step; returns (ob, 0, done, {})."""
        assert self.ob is not None
        e = self._eng
        e.begin_rollout()
        e.obs[0, 0].copy_(torch.as_tensor(np.asarray(self.ob, np.float64)))
        act = torch.as_tensor(np.asarray(action, np.float64).reshape(1, -1)).to(e.ctx.device)
        e.step(actions=act)
        ob = e.next_obs[0, 0].cpu().numpy()
        done = bool(e.done[0, 0].item())
        self.num_steps = int(e.num_steps[0].item())
        self.ob = ob.copy()
        self._last_done = done
        return ob.copy(), 0, done, {}

    def is_done(self):
        """sim_env.py:164-173 evaluated on the current observation (re-runs the check with a
        zero delta through the same kernel, so the answer is bit-identical to step's)."""
        e = self._eng
        ens = e.ens
        ws = ens.workspace(1)
        ws["preds"].zero_()
        from . import _native as N
        c = e.ctx
        ob = torch.as_tensor(np.asarray(self.ob, np.float64).reshape(1, -1)).to(c.device)
        nxt = torch.empty_like(ob)
        ns = torch.tensor([self.num_steps - 1], dtype=torch.int32, device=c.device)
        done = torch.empty(1, dtype=torch.uint8, device=c.device)
        zero = torch.zeros(1, dtype=torch.int32, device=c.device)
        N.check(c.lib.amx_step(c.h, ws["preds"].data_ptr(), c.S, ws["preds"].shape[1] * c.S, zero.data_ptr(),
                               ob.data_ptr(), nxt.data_ptr(), ns.data_ptr(), done.data_ptr(), None, None, 0, None, 1,
                               c.stream), "amx_step")
        return bool(done.item())

    def reset(self):
        """sim_env.py:270-285: t ~ U(0, time_max) -> reset pose; next ensemble member."""
        t = self.np_random.uniform(low=0, high=self.time_max)
        if self.motion is not None:
            self._eng.reset_all(rows=torch.tensor([t], dtype=torch.float64, device=self._eng.ctx.device))
        else:
            row = torch.tensor([int(np.floor(t))], dtype=torch.int32, device=self._eng.ctx.device)
            self._eng.reset_all(rows=row)
        self.last_reset_time = t
        self.num_steps = 0
        self.reset_counter = (self.reset_counter + 1) % self._eng.ctx.M
        self.ob = self._eng.obs[0, 0].cpu().numpy().copy()
        return self.ob.copy()

    def render(self, mode="human", close=False):
        pass


class BatchedSimEnv:
    """B SimEnv lanes in lock-step (vectorised semantics, auto-reset)."""

    def __init__(self, dynamic_ensemble, reset_table, lanes: int, deepmimic_args=None, enable_velocity_check=False,
                 horizon=HORIZON, seed: int = 0, policy=None, cost=None, max_steps: int = 32, record_means=False):
        dev_ens = getattr(dynamic_ensemble, "device", dynamic_ensemble)
        self.term = termination_from_args(deepmimic_args, horizon, enable_velocity_check)
        self.engine = RolloutEngine(dev_ens, reset_table, lanes=lanes, term=self.term, policy=policy, cost=cost,
                                    seed=seed, max_steps=max_steps, record_means=record_means)
        self.num_envs = lanes

    def reset(self):
        self.engine.reset_all()
        return self.engine.obs[0]

    def step(self, actions=None):
        """Returns (next_obs [B,S] f64 device, reward zeros [B], done [B] bool, infos)."""
        e = self.engine
        if e.t >= e.K:
            e.begin_rollout()
        t = e.step(actions=None if actions is None else torch.as_tensor(actions, dtype=torch.float64,
                                                                         device=e.ctx.device))
        return e.next_obs[t], torch.zeros(e.B, device=e.ctx.device), e.done[t].bool(), {}

    @property
    def observations(self):
        return self.engine.obs[self.engine.t]
