"""Reset-from-motion: host preprocessing of the product against the oracle's
restatement of cMotion::Load, and properties of the oracle's reset states.  Parity against
the reference itself is unpinned (DeepMimicCore is not buildable here); see DESIGN.md."""
import json

import numpy as np
import pytest

from oracle import deepmimic_ref as D


@pytest.fixture(scope="module")
def g12(golden):
    g = golden("g12_motion.npz")
    char = json.loads(str(g["character_json"]))
    motion = {"Loop": str(g["loop"]), "Frames": g["frames"].tolist()}
    J, B, dof = D.load_character(char)
    return g, char, motion, J, B, D.Motion(motion, J)


def test_preprocessing_matches_oracle(g12):
    from amp_extensions_amd.motion import preprocess_frames, skeleton_tables
    g, char, motion, J, B, M = g12
    jt, bt, dof = skeleton_tables(char)
    assert dof == M.frames.shape[1] == 43 and jt.shape == (15, 8)
    times, frames, vels = preprocess_frames(g["frames"], jt)
    np.testing.assert_array_equal(times, M.times)
    np.testing.assert_array_equal(frames, M.frames)
    np.testing.assert_allclose(vels, M.vels, rtol=0, atol=1e-12)
    assert M.loop and abs(M.duration - 77 * 0.016666) < 1e-9


def test_reset_state_properties(g12):
    g, char, motion, J, B, M = g12
    rs = np.random.RandomState(0)
    for t in np.concatenate([M.times[:-1], rs.uniform(0, M.duration, 40)]):
        s = D.reset_state(J, B, M, t)
        assert s.shape == (226,) and np.isfinite(s).all()
        for i in range(15):
            nrm, tan = s[9 * i + 4:9 * i + 7], s[9 * i + 7:9 * i + 10]
            assert abs(np.linalg.norm(nrm) - 1) < 1e-12 and abs(np.linalg.norm(tan) - 1) < 1e-12
            assert abs(nrm @ tan) < 1e-12
        # non-root body positions are heading-frame offsets from the root: root body offset is the
        # rotated attach point (0, 0.07, 0) of the pelvis sphere
        assert abs(np.linalg.norm(s[1:4]) - 0.07) < 1e-12
        # after the ground resolve every body clears the ground by >= the 0.001 pad
        pose = M.pose(t)
        pose[0] = pose[2] = 0.0
        R, o, w, v = D.forward_kinematics(J, pose, M.vel(t))
        lift = s[0] - pose[1]
        assert lift >= -1e-12
        lows = [D.body_aabb_min_y(B[j], R[j], o[j] + R[j] @ B[j]["attach"]) + lift for j in range(15)]
        assert min(lows) >= 0.001 - 1e-12
        if lift > 1e-12:
            assert abs(min(lows) - 0.001) < 1e-12


def test_reset_state_at_frame_time_uses_the_frame(g12):
    """At a frame time the pose is that frame (blend 0) and the root height is the frame's
    (plus any ground lift); StandardizeQuat keeps w >= 0."""
    g, char, motion, J, B, M = g12
    for f in (0, 10, 40):
        p = M.pose(M.times[f])
        np.testing.assert_allclose(p[7:], M.frames[f, 7:], atol=1e-15)
        assert p[3] >= 0


def test_state_amp_obs_oracle_equals_pose_amp_obs(g12):
    """The oracle's AMP features of two recorded states equal BuildAMPObs of the (pose, vel)
    pairs those states were recorded from (the state -> pose recovery is consistent)."""
    g, char, motion, J, B, M = g12
    ee, dt = [5, 8, 11, 14], 1.0 / 30
    for t in np.random.RandomState(2).uniform(dt, M.duration, 6):
        sp, sc = D.reset_state(J, B, M, t - dt), D.reset_state(J, B, M, t)
        pp, vp = D.reset_pose_vel(J, B, M, t - dt)
        pc, vc = D.reset_pose_vel(J, B, M, t)
        for local in (False, True):
            a = D.state_amp_obs(J, ee, sp, sc, local)
            b = D.amp_obs(J, B, ee, pp, vp, pc, vc, local_root=local)
            assert a.shape == (226,) and np.abs(a - b).max() <= 1e-12


@pytest.mark.parametrize("interp", [1.0, 0.4])
def test_pure_root_yaw_noise_keeps_heading_frame_velocities(g12, interp):
    """RandomRotatePoseVel's root yaw goes through cKinCharacter::SetRootRotation ->
    RotateOrigin (anim/KinCharacter.cpp:259-264, 300-337), which rotates the root's linear and
    angular velocity with the pose: with only the yaw draw non-zero (every other rotation draw
    u = 0.5, i.e. RandDouble(-r, r) = 0) the heading-frame part of the state equals the plain
    reset state scaled by interp (velocities), and the world-frame root entries are the plain
    ones rotated about y."""
    g, char, motion, J, B, M = g12
    world_root = bool(g["record_world_root_rot"])
    ra = dict(noise_bef_rot=False, noise_min=0, noise_max=0, radian=0.3, rot_vel_w_pose=False,
              vel_noise=False, interp=interp, knee_rot=False)
    nr, npv = D.noise_draws(J, ra)
    n = len(J)
    base = 1 + 9 * n
    for k, t in enumerate(np.random.RandomState(5).uniform(0, M.duration, 8)):
        u = np.full(nr, 0.5)
        u[0] = 0.1 + 0.1 * k
        a = -0.3 + u[0] * 0.6
        Ry = D.rotmat(np.array([np.cos(a / 2), 0.0, np.sin(a / 2), 0.0]))
        s = D.reset_state(J, B, M, float(t), noise=ra, u_rot=u)
        p = D.reset_state(J, B, M, float(t))
        exp = p.copy()
        exp[base:] *= interp
        if world_root:
            exp[4:7], exp[7:10] = Ry @ p[4:7], Ry @ p[7:10]
            exp[base:base + 3] = Ry @ exp[base:base + 3]
            exp[base + 3:base + 6] = Ry @ exp[base + 3:base + 6]
        assert np.abs(s - exp).max() <= 1e-10, (t, np.abs(s - exp).max(), np.abs(s - exp).argmax())
