"""Reset-from-motion on the device (csrc/amx_motion.hip) vs the oracle's restatement of
DeepMimicCore's reset_time path (oracle/deepmimic_ref.py).  Parity against the reference
itself is unpinned (its C++ core is not buildable); tolerance here covers device vs host libm
(sin/cos/acos/atan2/sqrt last bits): |dev - oracle| <= 1e-10 * max(1, |oracle|)."""
import json

import numpy as np
import pytest
import torch

from oracle import deepmimic_ref as D

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def setup(golden):
    import amp_extensions_amd as amx
    from amp_extensions_amd.motion import ReferenceMotion
    g = golden("g12_motion.npz")
    char = json.loads(str(g["character_json"]))
    motion = {"Loop": str(g["loop"]), "Frames": g["frames"].tolist()}
    ctx = amx.AmxContext(226, 28, n_models=4, hidden=128, n_hidden=2, device=DEV)
    rm = ReferenceMotion(ctx, char, motion, record_world_root_pos=bool(g["record_world_root_pos"]),
                         record_world_root_rot=bool(g["record_world_root_rot"]),
                         record_all_world=bool(g["record_all_world"]))
    J, B, _ = D.load_character(char)
    M = D.Motion(motion, J)
    return amx, ctx, rm, J, B, M


def oracle_states(J, B, M, times):
    return np.stack([D.reset_state(J, B, M, float(t)) for t in times])


def test_motion_states_match_oracle(setup):
    amx, ctx, rm, J, B, M = setup
    assert abs(rm.get_motion_length() - M.duration) < 1e-15
    rs = np.random.RandomState(1)
    times = np.concatenate([[0.0, M.duration * (1 - 1e-12)], M.times[:-1], M.times[1:-1] - 1e-9,
                            rs.uniform(0, M.duration, 300), rs.uniform(M.duration, 3 * M.duration, 20)])
    got = rm.states(times).cpu().numpy()
    ref = oracle_states(J, B, M, times)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-10, (err.max(), np.unravel_index(err.argmax(), err.shape))


def test_reset_lanes_motion_draws_and_records(setup):
    """Philox t ~ U(0, duration) per lane; t_out records it; the state is the motion state at
    t; counters advance like SimEnv.reset (sim_env.py:277, 282-283)."""
    amx, ctx, rm, J, B, M = setup
    from amp_extensions_amd import _native as N
    L = 500
    ob = torch.zeros(L, 226, dtype=torch.float64, device=DEV)
    ns = torch.full((L,), 7, dtype=torch.int32, device=DEV)
    mi = torch.zeros(L, dtype=torch.int32, device=DEV)
    rc = torch.zeros(L, dtype=torch.int32, device=DEV)
    tout = torch.zeros(L, dtype=torch.float64, device=DEV)
    N.check(ctx.lib.amx_reset_lanes_motion(ctx.h, None, None, 1234, 0.0, rm.flags, ob.data_ptr(), ob.data_ptr(),
                                           ns.data_ptr(), mi.data_ptr(), rc.data_ptr(), tout.data_ptr(), L,
                                           ctx.stream))
    t = tout.cpu().numpy()
    assert (t >= 0).all() and (t < M.duration).all() and len(np.unique(t)) == L
    np.testing.assert_array_equal(ob.cpu().numpy(), rm.states(t).cpu().numpy())
    assert (ns.cpu().numpy() == 0).all() and (rc.cpu().numpy() == 1).all() and (mi.cpu().numpy() == 1).all()


def test_rollout_engine_with_motion_resets(setup):
    """RolloutEngine with a ReferenceMotion reset source: initial and auto resets produce motion
    states at the recorded times; carried lanes keep their state."""
    amx, ctx, rm, J, B, M = setup
    from amp_extensions_amd.ensemble import init_ensemble_weights
    from amp_extensions_amd.policy import init_mlp_policy_params
    s, a = np.random.RandomState(0).randn(512, 226) * 0.5, np.random.RandomState(1).randn(512, 28)
    norms = [torch.from_numpy(x) for x in (s.mean(0), np.abs(s).mean(0) + 1e-8, a.mean(0), np.abs(a).mean(0) + 1e-8,
                                           np.zeros(226), np.full(226, 0.01))]
    norms = [x.float() for x in norms]
    ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(226, 28, [128] * 2, 4, 100), norms)
    pw, ls = init_mlp_policy_params(226, 28)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=4)
    eng = amx.RolloutEngine(ens, rm, lanes=256, policy=pol, seed=9, max_steps=6)
    eng.reset_all()
    assert np.isfinite(eng.obs[0].cpu().numpy()).all()
    eng.rollout()
    torch.cuda.synchronize()
    done = eng.done.cpu().numpy()
    rt = eng.reset_times.cpu().numpy()
    obs = eng.obs.cpu().numpy()
    nxt = eng.next_obs.cpu().numpy()
    for t in range(6):
        d = np.nonzero(done[t])[0]
        nd = np.nonzero(done[t] == 0)[0]
        assert (rt[t, nd] == -1).all()
        if len(d):
            np.testing.assert_array_equal(obs[t + 1, d], rm.states(rt[t, d]).cpu().numpy())
        np.testing.assert_array_equal(obs[t + 1, nd], nxt[t, nd])


def test_simenv_facade_motion_reset(setup):
    """SimEnv(reset_table=ReferenceMotion): t drawn exactly as the reference
    (np_random.uniform(0, motion length), sim_env.py:276) -> the oracle's state at t."""
    amx, ctx, rm, J, B, M = setup
    from amp_extensions_amd.ensemble import init_ensemble_weights
    norms = [torch.zeros(226), torch.ones(226), torch.zeros(28), torch.ones(28), torch.zeros(226), torch.ones(226)]
    ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(226, 28, [128] * 2, 4, 100), norms)
    env = amx.SimEnv(ens, reset_table=rm, seed=5)
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(5)))
    for _ in range(3):
        ob = env.reset()
        t = rng.uniform(low=0, high=M.duration)
        assert env.last_reset_time == t
        ref = D.reset_state(J, B, M, t)
        assert np.abs(ob - ref).max() <= 1e-10 * max(1.0, np.abs(ref).max())


def test_expert_amp_obs_match_oracle(setup):
    """RecordAMPObsExpert features from the clip (prev frame at t - 1/30) vs the oracle's
    BuildAMPObs restatement; both local_root settings."""
    amx, ctx, rm, J, B, M = setup
    import json
    ee = [5, 8, 11, 14]
    assert rm.amp_obs_size == 226
    rs = np.random.RandomState(3)
    times = np.concatenate([[0.0, 0.01, M.duration * 0.999], rs.uniform(0, M.duration, 200)])
    for local in (False, True):
        got = rm.expert_amp_obs(times, local_root=local).cpu().numpy()
        ref = np.stack([D.expert_amp_obs(J, B, ee, M, t, local_root=local) for t in times])
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 1e-10, (local, err.max(), np.unravel_index(err.argmax(), err.shape))


def test_state_amp_obs_recovers_the_pose_features(setup):
    """AMP features of a SimEnv transition computed from the two recorded states equal
    BuildAMPObs of the simulated character's (pose, vel) pair the states were recorded from
    (joint rotations / velocities recovered from the tangent-normal rotations and body
    velocities of the states)."""
    amx, ctx, rm, J, B, M = setup
    ee = [5, 8, 11, 14]
    dt = 1.0 / 30
    rs = np.random.RandomState(4)
    times = rs.uniform(dt, M.duration, 100)
    sp = rm.states(times - dt)
    sc = rm.states(times)
    for local in (False, True):
        got = rm.amp_obs_from_states(sp, sc, local_root=local).cpu().numpy()
        ref = []
        for t in times:
            pp, vp = D.reset_pose_vel(J, B, M, t - dt)
            pc, vc = D.reset_pose_vel(J, B, M, t)
            ref.append(D.amp_obs(J, B, ee, pp, vp, pc, vc, local_root=local))
        ref = np.stack(ref)
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 1e-9, (local, err.max(), np.unravel_index(err.argmax(), err.shape))


NOISE_BASE = dict(custom_time=False, time_min=0, time_max=0, resolve=True, noise_bef_rot=False, noise_min=0,
                  noise_max=0, radian=0, rot_vel_w_pose=False, vel_noise=False, interp=1.0, knee_rot=False)


@pytest.mark.parametrize("opts", [dict(radian=0.2), dict(noise_min=-0.05, noise_max=0.08),
                                  dict(radian=0.25, noise_min=-0.03, noise_max=0.03, rot_vel_w_pose=True,
                                       vel_noise=True, interp=0.3),
                                  dict(radian=0.15, noise_min=-0.02, noise_max=0.04, noise_bef_rot=True,
                                       knee_rot=True, vel_noise=True, interp=0.0),
                                  dict(radian=3.0, vel_noise=True, rot_vel_w_pose=True, knee_rot=True)])
def test_reset_noise_with_injected_draws_matches_oracle(setup, opts):
    """SimEnv reset_args noise = cKinCharacter::AddNoise (anim/KinCharacter.cpp:340-470) before the
    placement and the ground resolve: with the same uniforms injected on both sides
    (RandomRotatePoseVel's draws at [0, 48), AddNoisePoseVel's after them) the device states equal
    the oracle's add_noise + reset_state at 1e-10 for every option combination."""
    amx, ctx, rm, J, B, M = setup
    ra = dict(NOISE_BASE, **opts)
    nr, npv = D.noise_draws(J, ra)
    assert nr <= 48
    Dof = sum(j["size"] for j in J)
    rs = np.random.RandomState(7)
    L = 64
    times = rs.uniform(0, M.duration, L)
    draws = rs.rand(L, 48 + 2 * Dof)
    got = rm.states(times, reset_args=ra, draws=torch.from_numpy(draws)).cpu().numpy()
    ref = np.stack([D.reset_state(J, B, M, float(times[i]), noise=ra, u_rot=draws[i, :nr], u_pv=draws[i, 48:48 + npv])
                    for i in range(L)])
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-10, (err.max(), np.unravel_index(err.argmax(), err.shape))
    plain = np.stack([D.reset_state(J, B, M, float(t)) for t in times])
    assert np.abs(ref - plain).max() > 1e-3  # the noise does move the state


def test_reset_noise_root_yaw_rotates_root_velocity(setup):
    """Only the root-yaw draw non-zero (every other RandomRotatePoseVel draw u = 0.5 gives
    RandDouble(-r, r) = 0), interp = 1: RotateRoot -> SetRootRotation -> RotateOrigin
    (anim/KinCharacter.cpp:259-264, 300-337) turns the root velocities with the pose, so the
    heading-frame entries of the device state equal the plain reset state and the world-frame
    root entries are the plain ones rotated about y."""
    amx, ctx, rm, J, B, M = setup
    ra = dict(NOISE_BASE, radian=0.3, interp=1.0)
    n = len(J)
    base = 1 + 9 * n
    L = 16
    times = np.random.RandomState(8).uniform(0, M.duration, L)
    draws = np.full((L, 48 + 2 * sum(j["size"] for j in J)), 0.5)
    draws[:, 0] = np.linspace(0.05, 0.95, L)
    got = rm.states(times, reset_args=ra, draws=torch.from_numpy(draws)).cpu().numpy()
    plain = oracle_states(J, B, M, times)
    assert rm.flags == 2   # world-frame root rotation only (the reference scene's flags)
    for i in range(L):
        a = -0.3 + draws[i, 0] * 0.6
        Ry = D.rotmat(np.array([np.cos(a / 2), 0.0, np.sin(a / 2), 0.0]))
        exp = plain[i].copy()
        exp[4:7], exp[7:10] = Ry @ plain[i, 4:7], Ry @ plain[i, 7:10]
        exp[base:base + 3] = Ry @ plain[i, base:base + 3]
        exp[base + 3:base + 6] = Ry @ plain[i, base + 3:base + 6]
        assert np.abs(got[i] - exp).max() <= 1e-10, (i, np.abs(got[i] - exp).max())


def test_reset_noise_philox_stream(setup):
    """Without injected draws the uniforms come from Philox(seed; lane, reset#): repeatable,
    seed-dependent, finite, and zero amounts give the plain states bit for bit."""
    amx, ctx, rm, J, B, M = setup
    ra = dict(NOISE_BASE, radian=0.2, noise_min=-0.05, noise_max=0.05, vel_noise=True)
    times = np.linspace(0.05, M.duration - 0.05, 40)
    a = rm.states(times, reset_args=ra, seed=11)
    b = rm.states(times, reset_args=ra, seed=11)
    c = rm.states(times, reset_args=ra, seed=12)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and not torch.equal(a, c) and torch.isfinite(a).all()
    assert torch.equal(rm.states(times, reset_args=NOISE_BASE), rm.states(times))


def test_simenv_with_reset_noise_runs(setup):
    """SimEnv(..., reset_args={'noise_max': 0.1, 'radian': 0.2, ...}) constructs and runs: its
    resets carry the noise (states differ from the noise-free reset at the same drawn time),
    BatchedSimEnv and sample_points too; a reset-state table with noise is refused (AddNoise
    perturbs a pose / velocity the table does not hold)."""
    amx, ctx, rm, J, B, M = setup
    from oracle import milo_ref as R
    S, A = 226, 28
    rs = np.random.RandomState(3)
    s = 0.5 * rs.randn(2048, S)
    s[:, 0] = rs.uniform(0.8, 0.95, 2048)
    a = rs.randn(2048, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s + 0.01 * rs.randn(2048, S))])
    ens = amx.DeviceEnsemble(ctx, R.init_ensemble_weights(S, A, [128] * 2, 4, 100), norms)
    ra = dict(NOISE_BASE, noise_min=-0.1, noise_max=0.1, radian=0.2, vel_noise=True, interp=1.0)
    env = amx.SimEnv(ens, reset_table=rm, reset_args=ra, seed=5)
    env0 = amx.SimEnv(ens, reset_table=rm, reset_args=NOISE_BASE, seed=5)
    for _ in range(5):
        o, o0 = env.reset(), env0.reset()
        assert env.last_reset_time == env0.last_reset_time and np.abs(o - o0).max() > 1e-3
        for _ in range(10):
            o, r, d, info = env.step(np.zeros(A))
            assert np.isfinite(o).all()
            if d:
                break
    benv = amx.BatchedSimEnv(ens, rm, lanes=64, reset_args=ra, seed=2, max_steps=4)
    benv.reset()
    for _ in range(4):
        benv.step(torch.zeros(64, A, dtype=torch.float64, device=DEV))
    assert torch.isfinite(benv.engine.obs[:4]).all()
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std)
    paths = amx.sample_points(benv, pol, num_to_collect=60, base_seed=1, num_workers=2)
    assert sum(len(p["rewards"]) for p in paths) >= 60
    with pytest.raises(NotImplementedError):
        amx.BatchedSimEnv(ens, s[:64], lanes=8, reset_args=ra)
