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
from .ensemble import as_device_ensemble
from .humanoid import BODY_DEFS, FALL_BODIES, HORIZON, TerminationConfig
from .rollout import RolloutEngine


class Box:
    """Minimal stand-in for gym.spaces.Box (gym is not a dependency of the engine)."""

    def __init__(self, low, high, dtype=np.float64):
        self.low, self.high = np.asarray(low, dtype), np.asarray(high, dtype)
        self.shape, self.dtype = self.low.shape, np.dtype(dtype)


# SimEnv's reset_args default (gym-simenv/gym_simenv/envs/sim_env.py:29-32; run.py:113-117 builds
# the same keys from milo/milo/arguments.py:26-43)
DEFAULT_RESET_ARGS = {'custom_time': False, 'time_min': 0, 'time_max': 0, 'resolve': True, 'noise_bef_rot': False,
                      'noise_min': 0, 'noise_max': 0, 'radian': 0, 'rot_vel_w_pose': False, 'vel_noise': False,
                      'interp': False, 'knee_rot': False}


def parse_deepmimic_args(path: str) -> dict:
    """DeepMimic's ArgParser.load_file (deepmimic/deepmimic/util/arg_parser.py:40-54, 14-38):
    lines starting with '#' and '#' tokens are comments, '--key' opens a key, the first
    occurrence of a key wins."""
    table: dict = {}
    key, vals = "", []
    toks = []
    with open(path) as f:
        for line in f.read().splitlines():
            if line and not line.startswith("#"):
                toks += line.split()
    for tok in toks:
        if tok.startswith("#"):
            continue
        if tok.startswith("--"):
            if key and key not in table:
                table[key] = vals
            key, vals = tok[2:], []
        else:
            vals.append(tok)
    if key and key not in table:
        table[key] = vals
    return table


def _resolve_data_path(p: str, args_path: str) -> str | None:
    """DeepMimic opens the arg file's data paths relative to its working directory (the
    deepmimic package root, the arg file's parent's parent): try the path as given, relative to
    the arg file's directory and its parent, then relative to the current directory."""
    base = os.path.dirname(os.path.abspath(args_path))
    for cand in (p, os.path.join(base, p), os.path.join(os.path.dirname(base), p), os.path.join(os.getcwd(), p)):
        if os.path.exists(cand):
            return cand
    return None


def _arg_file(table: dict, key: str, args_path: str, required: bool = False) -> str | None:
    val = table.get(key)
    path = _resolve_data_path(val[0], args_path) if val else None
    if required and path is None:
        raise FileNotFoundError(f"{args_path}: --{key} {val[0] if val else '(missing)'} not found")
    return path


def termination_from_args(deepmimic_args: str | None, horizon: int, enable_velocity_check: bool) -> TerminationConfig:
    """Read the ctrl flags and BodyDefs the reference reads (sim_env.py:84-115) when the
    DeepMimic arg file is available; otherwise the humanoid3d spinkick defaults."""
    cfg = TerminationConfig(horizon=horizon, enable_velocity_check=enable_velocity_check)
    if not deepmimic_args or not os.path.exists(deepmimic_args):
        return cfg
    args = parse_deepmimic_args(deepmimic_args)
    ctrl = _arg_file(args, "char_ctrl_files", deepmimic_args)
    if ctrl:
        cj = json.load(open(ctrl))
        cfg.record_vel_as_pos = bool(cj.get("RecordVelAsPos", False))
        cfg.record_all_world = bool(cj.get("RecordAllWorld", False))
        cfg.record_world_root_pos = bool(cj.get("RecordWorldRootPos", False))
        if "UpdateRate" in cj:
            cfg.sampling_rate = 1.0 / float(cj["UpdateRate"])
    char = _arg_file(args, "character_files", deepmimic_args)
    if char:
        hj = json.load(open(char))
        defs = hj["BodyDefs"]
        cfg.body_defs = {i: (d["Shape"], float(d["Param0"]), float(d["Param1"])) for i, d in enumerate(defs)}
    return cfg


def motion_from_args(ctx: AmxContext, deepmimic_args: str, resolve: bool = True):
    """The reset source DeepMimicCore builds from the arg file (`--character_files`,
    `--motion_file`, `--char_ctrl_files`; run_amp_humanoid3d_spinkick_args.txt:17,24,23): a
    `ReferenceMotion` with the controller's record flags (sim_env.py:86-91)."""
    from .motion import ReferenceMotion
    if not deepmimic_args or not os.path.exists(deepmimic_args):
        raise FileNotFoundError(f"DeepMimic arg file {deepmimic_args!r} not found")
    args = parse_deepmimic_args(deepmimic_args)
    char = _arg_file(args, "character_files", deepmimic_args, required=True)
    motion = _arg_file(args, "motion_file", deepmimic_args, required=True)
    ctrl = _arg_file(args, "char_ctrl_files", deepmimic_args)
    cj = json.load(open(ctrl)) if ctrl else {}
    return ReferenceMotion(ctx, char, motion, record_world_root_pos=bool(cj.get("RecordWorldRootPos", False)),
                           record_world_root_rot=bool(cj.get("RecordWorldRootRot", False)),
                           record_all_world=bool(cj.get("RecordAllWorld", False)), resolve=resolve)


def check_reset_args(reset_args: dict | None) -> dict:
    """reset_args with the reference's defaults filled in.  The noise options (noise_min /
    noise_max, radian, rot_vel_w_pose, vel_noise, interp, knee_rot, noise_bef_rot) are
    cKinCharacter::AddNoise (anim/KinCharacter.cpp:340-470), applied on the device to the
    kinematic pose / velocity of every motion reset (csrc/amx_motion.hip add_noise).  The
    reference draws them from DeepMimicCore's process-global std::default_random_engine, which
    cannot be reproduced: the device draws come from Philox(seed; lane, reset #) -- same
    distribution and transform, another stream.  `interp` and the rotation-noise
    flags act only inside RandomRotatePoseVel, which returns before touching the state when
    radian == 0 (KinCharacter.cpp:367-371)."""
    ra = dict(DEFAULT_RESET_ARGS)
    ra.update(reset_args or {})
    for k in ("noise_min", "noise_max", "radian", "interp"):
        v = float(ra[k])
        if v != v:
            raise ValueError(f"reset_args[{k!r}] is NaN")
    return ra


try:  # gym is optional: register the drop-in under the reference's id when it is importable
    import gym as _gym
    _EnvBase = _gym.Env
except Exception:  # pragma: no cover - gym is not installed in this image
    _gym = None
    _EnvBase = object


class SimEnv(_EnvBase):
    """gym_simenv SimEnv (sim_env.py:13-288) on the HIP engine, one lane."""

    def __init__(self, dynamic_ensemble, deepmimic_args=None, enable_velocity_check=False, horizon=HORIZON,
                 device=None, seed=None, reset_args=None, reset_table=None):
        """Constructed as run.py:120 does (`gym.make('simenv-v0', deepmimic_args=...,
        dynamic_ensemble=..., reset_args=...)`): the reset source is the arg file's character
        and motion (DeepMimicCore's reset_time path restated on the device, motion.py).
        `reset_table` (extension): a ReferenceMotion or a [R, S] reset-state table (row
        floor(t); the synthetic benchmark layout) in place of the arg file's motion.
        reset_args: custom_time / time_max set the reset-time window (sim_env.py:76-77),
        resolve the ground lift; the noise options perturb every motion reset (AddNoise on the
        device, check_reset_args; a reset-state table with noise raises NotImplementedError)."""
        self.reset_args = check_reset_args(reset_args)
        self.dynamic_ensemble = dynamic_ensemble
        dev_ens = as_device_ensemble(dynamic_ensemble)
        self.device = device
        self.enable_velocity_check = enable_velocity_check
        self.horizon = horizon
        self.term = termination_from_args(deepmimic_args, horizon, enable_velocity_check)
        if reset_table is None:
            if not deepmimic_args:
                raise ValueError("SimEnv needs a reset source: deepmimic_args (character + motion files), "
                                 "a ReferenceMotion or a reset_table")
            reset_table = motion_from_args(dev_ens.ctx, deepmimic_args, resolve=bool(self.reset_args["resolve"]))
        self._eng = RolloutEngine(dev_ens, reset_table, lanes=1, term=self.term, seed=0, max_steps=1,
                                  auto_reset=False)
        self._eng.set_reset_noise(self.reset_args)  # AddNoise (raises for a table source with noise)
        c = self._eng.ctx
        self.state_size, self.action_size = c.S, c.A
        self.observation_space = Box([-np.inf] * c.S, [np.inf] * c.S)
        self.action_space = Box([-np.inf] * c.A, [np.inf] * c.A)
        self.motion = self._eng.motion
        if self.motion is not None and not self.reset_args["resolve"] and self.motion.resolve:
            raise ValueError("reset_args['resolve'] is False but the ReferenceMotion resolves ground intersections")
        # sim_env.py:76-77: the window is [0, time_max) (time_min is stored but reset ignores it,
        # :276); time_max = the motion length (a table's length in rows) unless custom_time
        n_src = self.motion.get_motion_length() if self.motion is not None else float(np.asarray(reset_table).shape[0])
        self.time_min = self.reset_args["time_min"] if self.reset_args["custom_time"] else 0
        self.time_max = float(self.reset_args["time_max"]) if self.reset_args["custom_time"] else n_src
        if self.motion is None and self.time_max > n_src:
            raise ValueError(f"reset_args time_max {self.time_max} exceeds the reset table's {int(n_src)} rows")
        self.ob = None
        self.num_steps = 0
        self.reset_counter = 0
        self.seed_env(seed)

    def seed_env(self, seed=None):
        """sim_env.py:122-132 (gym 0.26 seeding: Generator(PCG64(SeedSequence(seed)))); the seed
        also keys the device reset noise's Philox stream (AddNoise, check_reset_args)."""
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        if hasattr(self, "_eng"):
            self._eng.seed = int(seed or 0) & 0xFFFFFFFFFFFFFFFF

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
                 horizon=HORIZON, seed: int = 0, policy=None, cost=None, max_steps: int = 32, record_means=False,
                 reset_args=None):
        """`reset_table` None: the arg file's character + motion (as SimEnv); reset_args as
        SimEnv's (custom_time / time_max bound the lanes' Philox reset times, or the table rows
        drawn; the noise options perturb every motion reset, check_reset_args)."""
        self.reset_args = check_reset_args(reset_args)
        dev_ens = as_device_ensemble(dynamic_ensemble)
        self.term = termination_from_args(deepmimic_args, horizon, enable_velocity_check)
        if reset_table is None:
            if not deepmimic_args:
                raise ValueError("BatchedSimEnv needs a reset source: deepmimic_args, a ReferenceMotion or a table")
            reset_table = motion_from_args(dev_ens.ctx, deepmimic_args, resolve=bool(self.reset_args["resolve"]))
        custom = self.reset_args["custom_time"]
        from .motion import ReferenceMotion
        if isinstance(reset_table, ReferenceMotion) and not self.reset_args["resolve"] and reset_table.resolve:
            raise ValueError("reset_args['resolve'] is False but the ReferenceMotion resolves ground intersections")
        if custom and not isinstance(reset_table, ReferenceMotion):
            rows = int(np.ceil(float(self.reset_args["time_max"])))
            n = int(torch.as_tensor(reset_table).shape[0])
            if not 0 < rows <= n:
                raise ValueError(f"reset_args time_max {self.reset_args['time_max']} outside the table's {n} rows")
            reset_table = torch.as_tensor(reset_table)[:rows]
        self.engine = RolloutEngine(dev_ens, reset_table, lanes=lanes, term=self.term, policy=policy, cost=cost,
                                    seed=seed, max_steps=max_steps, record_means=record_means)
        self.engine.set_reset_noise(self.reset_args)
        if custom and self.engine.motion is not None:
            self.engine.reset_time_max = float(self.reset_args["time_max"])
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


if _gym is not None:  # gym-simenv/gym_simenv/__init__.py:3-6 (milo/milo/__init__.py:3-6)
    try:
        _gym.envs.registration.register(id="simenv-v0", entry_point="amp_extensions_amd.sim_env:SimEnv")
    except Exception:  # already registered (e.g. by the reference's own gym_simenv package)
        pass
