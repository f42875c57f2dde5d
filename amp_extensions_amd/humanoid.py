"""humanoid3d scene constants for the fall-termination check and the state layout.

Data (not code) taken from the reference scene the MILO path runs
(run_amp_humanoid3d_spinkick_args.txt + humanoid3d_rot_ctrl.txt):
  * fall bodies: run_amp_humanoid3d_spinkick_args.txt:19, hard-coded in
    gym-simenv/gym_simenv/envs/sim_env.py:102;
  * BodyDefs Shape/Param0/Param1: deepmimic/deepmimic/data/characters/humanoid3d.txt;
  * ctrl flags: deepmimic/deepmimic/data/controllers/humanoid3d_rot_ctrl.txt:2-5
    (RecordWorldRootPos false, no RecordAllWorld / RecordVelAsPos -> false);
  * state layout S = 1 + 15*(3+6) + 15*(3+3) = 226, action A = 8*3 + 4*1 = 28
    (DeepMimicCore sim/CtController.cpp:305-319, sim/CtCtrlUtil.cpp:10-22);
    velocity block starts after the pose block at 1 + 15*9 = 136.
BASELINE.json quotes the upstream DeepMimic sizes obs~197 / act~36; both are supported
(the engine is dimension-parametric; the fall bodies index < 132 in either layout).
"""
from __future__ import annotations

from dataclasses import dataclass, field

FALL_BODIES = (0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 12, 13, 14)

# body id -> (shape, Param0, Param1)
BODY_DEFS = {
    0: ("sphere", 0.18, 0.18), 1: ("sphere", 0.22, 0.22), 2: ("sphere", 0.205, 0.205),
    3: ("capsule", 0.11, 0.3), 4: ("capsule", 0.1, 0.31), 5: ("box", 0.177, 0.055),
    6: ("capsule", 0.09, 0.18), 7: ("capsule", 0.08, 0.135), 8: ("sphere", 0.08, 0.08),
    9: ("capsule", 0.11, 0.3), 10: ("capsule", 0.1, 0.31), 11: ("box", 0.177, 0.055),
    12: ("capsule", 0.09, 0.18), 13: ("capsule", 0.08, 0.135), 14: ("sphere", 0.08, 0.08),
}

SHAPE_CODE = {"sphere": 0, "capsule": 1, "box": 2}

STATE_DIM = 226        # faithful layout (rotation as tan-norm 6D, no phase)
ACTION_DIM = 28
BASELINE_STATE_DIM = 197   # BASELINE.json shape (quaternion + phase upstream layout)
BASELINE_ACTION_DIM = 36
VEL_OFFSET = 136
UPDATE_RATE = 30           # humanoid3d_rot_ctrl.txt:2 -> sampling_rate = 1/30 (sim_env.py:92)
HORIZON = 300              # sim_env.py:28


@dataclass
class TerminationConfig:
    """Everything SimEnv.is_done reads (sim_env.py:83-115, 164-268)."""
    fall_bodies: tuple = FALL_BODIES
    body_defs: dict = field(default_factory=lambda: dict(BODY_DEFS))
    record_all_world: bool = False
    record_world_root_pos: bool = False
    record_vel_as_pos: bool = False
    pos_dim: int = 3
    rot_dim: int = 6
    horizon: int = HORIZON
    enable_velocity_check: bool = False
    vel_offset: int = VEL_OFFSET
    vel_threshold: float = 100.0   # check_velocity default (sim_env.py:259)
    sampling_rate: float = 1.0 / UPDATE_RATE

    def tables(self):
        ids = list(self.fall_bodies)
        shapes = [SHAPE_CODE[self.body_defs[i][0]] for i in ids]
        p0 = [float(self.body_defs[i][1]) for i in ids]
        p1 = [float(self.body_defs[i][2]) for i in ids]
        return ids, shapes, p0, p1
