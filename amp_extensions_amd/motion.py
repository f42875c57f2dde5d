"""Reference-motion reset states (SimEnv.reset's DeepMimicCore path).

`ReferenceMotion` loads a DeepMimic character file (Skeleton.Joints + BodyDefs, e.g.
deepmimic/deepmimic/data/characters/humanoid3d.txt) and a motion clip ({"Loop", "Frames":
[[duration, root pos, root quat (w,x,y,z), joint params...]]}, e.g.
data/motions/humanoid3d_spinkick.txt), preprocesses the clip exactly as cMotion::Load does
(PostProcessFrames: frame times, root x/z recentred on frame 0, quaternions normalized;
BuildFrameVel with KinTree::CalcVel — anim/Motion.cpp:104-188, 415-442,
anim/KinTree.cpp:1518-1575) and uploads it (amx_set_motion).  The per-lane state at a reset
time is then computed on the device (csrc/amx_motion.hip): the state the simulated
character records after reset_time(t) with SimEnv's default reset_args.

Only the state layout the reference scene builds is supported: S = 1 + 15 J (CtController
positions + tangent-normal rotations + linear/angular velocities, humanoid3d: 226).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os

import numpy as np
import torch

from . import _native as N
from .engine import AmxContext

_JOINT_TYPES = {"revolute": 0, "planar": 1, "prismatic": 2, "fixed": 3, "spherical": 4, "none": 5}
_PARAM_SIZE = {0: 1, 1: 3, 2: 1, 3: 0, 4: 4, 5: 7}
_SHAPES = {"box": 0, "capsule": 1, "sphere": 2}
HDR = 16


def _qmul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz, aw * bz + az * bw + ax * by - ay * bx])


def _axis_angle(q):
    """cMathUtil::QuaternionToAxisAngle (util/MathUtil.cpp:468-486) with NormalizeAngle."""
    if q[0] > 1:
        q = q / np.linalg.norm(q)
    s = math.sqrt(1 - q[0] * q[0])
    if s > 0.000001:
        th = math.fmod(2 * math.acos(q[0]), 2 * math.pi)
        if th > math.pi:
            th = -2 * math.pi + th
        elif th < -math.pi:
            th = 2 * math.pi + th
        return q[1:] / s, th
    return np.array([0.0, 0.0, 1.0]), 0.0


def _conj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def skeleton_tables(character: dict):
    """Joint table [J][8] (type, parent, offset, size, attach xyz, is-end-effector) and body table [J][8]
    (shape, attach xyz, Param0-2, valid) of a parsed character file."""
    joints = character["Skeleton"]["Joints"]
    bodies = {b["ID"]: b for b in character["BodyDefs"]}
    J = len(joints)
    jt = np.zeros((J, 8))
    bt = np.zeros((J, 8))
    off = 0
    for j, d in enumerate(joints):
        if d["ID"] != j:
            raise ValueError("joints must be listed in ID order")
        t = _JOINT_TYPES["none"] if d["Parent"] == -1 else _JOINT_TYPES[d["Type"]]
        if t in (1, 2):
            raise NotImplementedError("planar / prismatic joints are not used by the humanoid")
        if any(d.get(k, 0.0) != 0.0 for k in ("AttachThetaX", "AttachThetaY", "AttachThetaZ")):
            raise NotImplementedError("non-zero joint AttachTheta")
        attach = [0.0, 0.0, 0.0] if d["Parent"] == -1 else [d["AttachX"], d["AttachY"], d["AttachZ"]]
        jt[j] = [t, d["Parent"], off, _PARAM_SIZE[t], *attach, float(d.get("IsEndEffector", 0))]
        off += _PARAM_SIZE[t]
        b = bodies.get(j)
        if b is not None:
            if any(b.get(k, 0.0) != 0.0 for k in ("AttachThetaX", "AttachThetaY", "AttachThetaZ")):
                raise NotImplementedError("non-zero body AttachTheta")
            bt[j] = [_SHAPES[b["Shape"]], b["AttachX"], b["AttachY"], b["AttachZ"], b["Param0"], b["Param1"],
                     b["Param2"], 1.0]
    return jt, bt, off


def preprocess_frames(raw: np.ndarray, jt: np.ndarray):
    """cMotion::Load's PostProcessFrames + BuildFrameVel: (times [F], frames [F][D], vels [F][D])."""
    raw = np.asarray(raw, dtype=np.float64)
    durs, frames = raw[:, 0].copy(), raw[:, 1:].copy()
    F, D = frames.shape
    times = np.zeros(F)
    t = 0.0
    off = frames[0, 0:3].copy()
    off[1] = 0.0
    sph = [int(r[2]) for r in jt[1:] if int(r[0]) == 4]
    for f in range(F):
        times[f] = t
        t += durs[f]
        frames[f, 0:3] -= off
        frames[f, 3:7] /= np.linalg.norm(frames[f, 3:7])
        for o in sph:
            frames[f, o:o + 4] /= np.linalg.norm(frames[f, o:o + 4])
    vels = np.zeros_like(frames)
    for f in range(F - 1):
        dt = times[f + 1] - times[f]
        p0, p1 = frames[f], frames[f + 1]
        v = vels[f]
        v[0:3] = (p1[0:3] - p0[0:3]) / dt
        axis, th = _axis_angle(_qmul(p1[3:7], _conj(p0[3:7])))     # CalcQuaternionVel
        v[3:6] = (th / dt) * axis
        for r in jt[1:]:
            typ, o, s = int(r[0]), int(r[2]), int(r[3])
            if typ == 4:
                axis, th = _axis_angle(_qmul(_conj(p0[o:o + 4]), p1[o:o + 4]))   # CalcQuaternionVelRel
                v[o:o + 3] = (th / dt) * axis
                v[o + 3] = 0.0
            elif s > 0:
                v[o:o + s] = (p1[o:o + s] - p0[o:o + s]) / dt
    if F > 1:
        vels[F - 1] = vels[F - 2]
    return times, frames, vels


def build_blob(jt, bt, times, frames, vels, loop: bool, ground_pad: float = 0.001) -> np.ndarray:
    F, D = frames.shape
    J = jt.shape[0]
    hdr = np.zeros(HDR)
    cycle = frames[-1, 0:3] - frames[0, 0:3]
    cycle[1] = 0.0                      # CalcCycleDeltaRootPos without root-height sync
    hdr[:12] = [J, D, F, float(loop), times[-1], 0, 0, 0, *cycle, ground_pad]
    return np.concatenate([hdr, jt.ravel(), bt.ravel(), times, frames.ravel(), vels.ravel()]).astype(np.float64)


class ReferenceMotion:
    """A reference clip on the device; `states(t)` = SimEnv.reset's recorded state at t."""

    def __init__(self, ctx: AmxContext, character, motion, record_world_root_pos: bool = False,
                 record_world_root_rot: bool = True, record_all_world: bool = False, resolve: bool = True):
        """`character`/`motion`: file paths (DeepMimic JSON) or already-parsed dicts
        ({"Skeleton", "BodyDefs"} / {"Loop", "Frames"}).  The record flags come from the
        controller file (humanoid3d_rot_ctrl.txt: RecordWorldRootPos false,
        RecordWorldRootRot true); `resolve` is reset_args['resolve'] (False: no ground lift,
        SceneSimChar.cpp:714-716)."""
        if isinstance(character, str):
            character = json.load(open(character))
        if isinstance(motion, str):
            motion = json.load(open(motion))
        self.ctx = ctx
        jt, bt, D = skeleton_tables(character)
        raw = np.asarray(motion["Frames"], dtype=np.float64)
        if raw.shape[1] != D + 1:
            raise ValueError(f"motion frames have {raw.shape[1] - 1} values, the character {D}")
        self.loop = motion.get("Loop", "none") != "none"
        times, frames, vels = preprocess_frames(raw, jt)
        self.blob = build_blob(jt, bt, times, frames, vels, self.loop)
        self.flags = int(record_world_root_pos) | (int(record_world_root_rot) << 1) | (int(record_all_world) << 2)
        self.resolve = bool(resolve)
        N.check(ctx.lib.amx_set_motion(ctx.h, self.blob.ctypes.data, self.blob.size), "amx_set_motion")
        self.duration = float(times[-1])
        self.S = ctx.S

    DEFAULT_BUNDLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "humanoid3d_spinkick.npz")

    @classmethod
    def from_bundle(cls, ctx: AmxContext, path: str | None = None, **flags) -> "ReferenceMotion":
        """Load a character + clip bundle written by tools/pack_motion.py (default: humanoid3d
        with the spinkick clip, the reference's run_amp_humanoid3d_spinkick_args.txt data)."""
        with np.load(path or cls.DEFAULT_BUNDLE, allow_pickle=False) as z:
            character = json.loads(str(z["character_json"]))
            motion = {"Loop": str(z["loop"]), "Frames": z["frames"].tolist()}
        return cls(ctx, character, motion, **flags)

    @property
    def kernel_flags(self) -> int:
        """The record flags + bit 3 (no ground resolve) as amx_motion_states takes them."""
        return self.flags | (0 if self.resolve else 8)

    @property
    def amp_obs_size(self) -> int:
        """SceneImitateAMP::GetAMPObsSize (2 x (pose part + vel part); humanoid3d: 226)."""
        return int(self.ctx.lib.amx_amp_obs_size(self.ctx.h))

    def expert_amp_obs(self, times, dt: float = 1.0 / 30, local_root: bool = False) -> torch.Tensor:
        """RecordAMPObsExpert (scenes/SceneImitateAMP.cpp:167-193) at the given clip times:
        BuildAMPObs of the clip frame at t - dt (prev) and t, dt = 1 / UpdateRate."""
        c = self.ctx
        t = torch.as_tensor(times, dtype=torch.float64).reshape(-1).to(c.device).contiguous()
        D = self.amp_obs_size
        out = torch.empty(t.numel(), D, dtype=torch.float64, device=c.device)
        N.check(c.lib.amx_motion_amp_obs(c.h, t.data_ptr(), float(dt), t.numel(), int(local_root), out.data_ptr(), D,
                                         c.stream), "amx_motion_amp_obs")
        return out

    def amp_obs_from_states(self, s_prev: torch.Tensor, s_cur: torch.Tensor, local_root: bool = False,
                            out: torch.Tensor | None = None) -> torch.Tensor:
        """RecordAMPObsAgent (BuildAMPObs of the previous and the current simulated pose) from
        two recorded SimEnv states per row ([B, S] float64, CtController layout with
        RecordWorldRootRot): the joint rotations, joint velocities and root velocity are
        recovered from the tangent-normal rotations and body velocities of the states."""
        if self.flags != 2:
            raise NotImplementedError("AMP features from states need RecordWorldRootRot only (humanoid3d_rot_ctrl)")
        c = self.ctx
        B = s_cur.shape[0]
        D = self.amp_obs_size
        if out is None:
            out = torch.empty(B, D, dtype=torch.float64, device=c.device)
        N.check(c.lib.amx_state_amp_obs(c.h, s_prev.data_ptr(), s_cur.data_ptr(), s_cur.stride(0), B, int(local_root),
                                        out.data_ptr(), out.stride(0), c.stream), "amx_state_amp_obs")
        return out

    def get_motion_length(self) -> float:
        """DeepMimicEnv.get_motion_length (SimEnv's time_max, sim_env.py:77)."""
        return self.duration

    def states(self, times, reset_args: dict | None = None, draws: torch.Tensor | None = None,
               seed: int = 0) -> torch.Tensor:
        """[B, S] float64 device states at the given motion times.  `reset_args` with noise
        (noise_min / noise_max / radian, ...): cKinCharacter::AddNoise applied before the
        placement and the ground resolve, its uniforms from Philox(seed; lane) or `draws`
        ([B, >= 48 + 2 D] float64 in [0, 1): RandomRotatePoseVel's draws first, AddNoisePoseVel's
        from column 48)."""
        c = self.ctx
        t = torch.as_tensor(times, dtype=torch.float64).reshape(-1).to(c.device).contiguous()
        out = torch.empty(t.numel(), self.S, dtype=torch.float64, device=c.device)
        noise = N.ResetNoise.from_reset_args(reset_args) if reset_args is not None else None
        if draws is not None:
            draws = torch.as_tensor(draws, dtype=torch.float64).to(c.device).contiguous()
        N.check(c.lib.amx_motion_states_noise(c.h, t.data_ptr(), t.numel(), self.kernel_flags,
                                              None if noise is None else C.byref(noise),
                                              None if draws is None else draws.data_ptr(),
                                              0 if draws is None else draws.stride(0), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                              out.data_ptr(), self.S, c.stream),
                "amx_motion_states_noise")
        return out
