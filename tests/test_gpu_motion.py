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
