"""Pin the CPU oracle (oracle/milo_ref.py) to the reference's own outputs.

The fixtures were produced by running the reference Python (tests/golden/make_golden.py).
Termination/indexing/integer results must match exactly; floating-point results are
checked bit-for-bit too (same torch-CPU kernels, same op order) with a 1e-6 relative
escape hatch for a CPU whose BLAS blocks differently.
"""
import math

import numpy as np
import pytest
import torch

from oracle import milo_ref as R

S, A = 226, 28

# the fixtures were generated single-threaded; torch-CPU reductions are bit-stable per
# thread count, so pin it for the bit-exact comparisons
torch.set_num_threads(1)


def synthetic_offline(n, seed):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def close(x, y, rtol=1e-6, atol=1e-7):
    x, y = np.asarray(x), np.asarray(y)
    if np.array_equal(x, y):
        return
    np.testing.assert_allclose(x, y, rtol=rtol, atol=atol)


@pytest.fixture(scope="module")
def norms():
    s, a, s2 = synthetic_offline(2048, 0)
    return R.get_transformations(torch.from_numpy(s).float(), torch.from_numpy(a).float(),
                                 torch.from_numpy(s2).float())


def test_transformations(golden, norms):
    g = golden("g7_transformations.npz")
    for k, v in zip(["mu_s", "sd_s", "mu_a", "sd_a", "mu_d", "sd_d"], norms):
        np.testing.assert_array_equal(v.numpy(), g[k])


@pytest.mark.parametrize("tag", ["h64", "h512"])
def test_ensemble_forward_disc_threshold(golden, norms, tag):
    g = golden(f"g1_ensemble_{tag}.npz")
    hidden = [int(x) for x in g["hidden"]]
    ens = R.init_ensemble_weights(S, A, hidden, 4, int(g["base_seed"]))
    np.testing.assert_array_equal(ens[0][0][0].numpy()[:4, :8], g["first_w0"])
    rs = np.random.RandomState(int(g["query_seed"]))
    B = int(g["B"])
    qs = torch.from_numpy(rs.randn(B, S) * 0.5).float()
    qa = torch.from_numpy(rs.randn(B, A)).float()
    close(R.ensemble_preds(ens, norms, qs, qa).numpy(), g["preds"])
    close(R.compute_discrepancy(ens, norms, qs, qa).numpy(), g["disc"])
    s, a, _ = synthetic_offline(2048, 0)
    thr = R.compute_threshold(ens, norms, torch.from_numpy(s).float(), torch.from_numpy(a).float())
    close(thr, float(g["threshold"]))


def test_ensemble_checkpoint(golden, golden_path, norms):
    """G13: the reference's save_ensemble file (run.py's ensemble.pt) read back by the oracle's
    load_ensemble_weights reproduces the reference's run.py:72-78 + 108 outputs."""
    g = golden("g13_ensemble_ckpt.npz")
    ens = R.load_ensemble_weights(golden_path("g13_ensemble.pt"))
    hidden = [int(x) for x in g["hidden"]]
    assert len(ens) == 4 and [W.shape[0] for W, _ in ens[0][:-1]] == hidden
    # one Adam step moved every member off its seeded init
    init = R.init_ensemble_weights(S, A, hidden, 4, int(g["base_seed"]))
    assert all(not torch.equal(w[0][0], i[0][0]) for w, i in zip(ens, init))
    qs, qa = torch.from_numpy(g["query_s"]), torch.from_numpy(g["query_a"])
    close(R.ensemble_preds(ens, norms, qs, qa).numpy(), g["preds"])
    with torch.no_grad():
        pn = torch.stack([R.dynamics_forward(w, norms, qs, qa, unnormalize_out=False) for w in ens])
    close(pn.numpy(), g["preds_norm"])
    close(R.compute_discrepancy(ens, norms, qs, qa).numpy(), g["disc"])
    s, a, _ = synthetic_offline(2048, 0)
    close(R.compute_threshold(ens, norms, torch.from_numpy(s).float(), torch.from_numpy(a).float()),
          float(g["threshold"]))


def test_simenv_trace(golden, norms):
    g = golden("g2_simenv_trace.npz")
    ens = R.init_ensemble_weights(S, A, [64] * 4, 4, 100)
    table, _, _ = synthetic_offline(int(g["table_rows"]), int(g["table_seed"]))
    env = R.SimEnvRef(ens, norms, horizon=int(g["horizon"]))
    rows = list(g["reset_rows"])
    o = env.reset(table[rows.pop(0)])
    for t in range(g["actions"].shape[0]):
        assert env.model_index == g["model_idx"][t]
        no, r, d, info = env.step(g["actions"][t].copy())
        np.testing.assert_array_equal(o, g["obs"][t])
        close(no, g["next_obs"][t], rtol=1e-12, atol=0)
        assert d == bool(g["done"][t])
        assert env.num_steps == g["num_steps"][t]
        o = env.reset(table[rows.pop(0)]) if d else no
    assert not rows


def test_fall_boundary(golden):
    g = golden("g3_fall_boundary.npz")
    env = R.SimEnvRef([None], None)
    for ob, hit in zip(g["obs"], g["collided"]):
        env.ob = ob.copy()
        assert env.check_collision() == bool(hit)
    # the fixture really straddles thresholds
    assert 0 < g["collided"].sum() < len(g["collided"])


def test_rff_mmd(golden):
    g = golden("g5_rff_mmd.npz")
    es, _, es2 = synthetic_offline(int(g["n_expert"]), int(g["expert_seed"]))
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    c = R.RBFLinearCostRef(expert, feature_dim=int(g["feature_dim"]), bw_quantile=float(g["bw_quantile"]),
                           lambda_b=float(g["lambda_b"]), seed=int(g["seed"]))
    assert c.bw == float(g["bw"])
    np.testing.assert_array_equal(c.W.numpy()[:4, :8], g["W_head"])
    np.testing.assert_array_equal(c.b.numpy()[:8], g["b_head"])
    close(c.phi_e.numpy(), g["phi_e"])
    ps, pa, ps2 = synthetic_offline(int(g["n_pi"]), int(g["pi_seed"]))
    mmd = c.fit_cost(torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float())
    close(mmd, float(g["mb_mmd"]))
    close(c.w.numpy(), g["w"])
    ens = R.init_ensemble_weights(S, A, [64] * 4, 4, 100)
    s, a, _ = synthetic_offline(2048, 0)
    _, _, _ = s, a, None
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in synthetic_offline(2048, 0)])
    thr = R.compute_threshold(ens, norms, torch.from_numpy(s).float(), torch.from_numpy(a).float())
    close(thr, float(g["threshold"]))
    disc_fn = lambda st, ac: R.compute_discrepancy(ens, norms, st, ac)
    cost, info = c.get_bonus_costs(torch.from_numpy(ps).float(), torch.from_numpy(pa).float(), disc_fn, thr,
                                   next_states=torch.from_numpy(ps2).float())
    close(cost.numpy(), g["cost"])
    close(info["ipm"].numpy(), g["ipm"])
    close(info["bonus"].numpy(), g["bonus"])
    close(info["v_targ"].numpy(), g["v_targ"])
    close(c.get_expert_cost().item(), float(g["expert_cost"]))


@pytest.mark.parametrize("tag", ["h64", "h1024"])
def test_gail(golden, tag):
    g = golden(f"g6_gail_{tag}.npz")
    hid = [int(x) for x in g["hidden"]]
    wts = R.init_disc_weights(2 * S, hid, 1, int(g["seed"]))
    ps, pa, ps2 = synthetic_offline(96, 4)
    ss = torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float()
    close(R.disc_forward(wts, ss).numpy(), g["logits"])
    close(R.gail_ls_costs(wts, ss).numpy(), g["cost_plain"])
    ens = R.init_ensemble_weights(S, A, [64] * 4, 4, 100)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in synthetic_offline(2048, 0)])
    disc_fn = lambda st, ac: R.compute_discrepancy(ens, norms, st, ac)
    cost, info = R.gail_bonus_costs(wts, torch.from_numpy(ps).float(), torch.from_numpy(pa).float(),
                                    torch.from_numpy(ps2).float(), disc_fn, float(g["lambda_b"]))
    close(cost.numpy(), g["cost"])
    close(info["ipm"].numpy(), g["ipm"])
    close(info["bonus"].numpy(), g["bonus"])


def test_sample_points(golden, norms):
    g = golden("g8_sample_points.npz")
    ens = R.init_ensemble_weights(S, A, [64] * 4, 4, 100)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    np.testing.assert_array_equal(pw[0][0].numpy()[:4, :8], g["pol_w0"])
    table, _, _ = synthetic_offline(64, 1)
    paths = R.sample_points(ens, norms, pw, log_std, int(g["num_to_collect"]), int(g["base_seed"]), table,
                            num_workers=int(g["num_workers"]), env_kw=dict(horizon=int(g["horizon"])))
    np.testing.assert_array_equal([len(p["rewards"]) for p in paths], g["lengths"])
    np.testing.assert_array_equal([p["terminated"] for p in paths], g["terminated"])
    close(np.concatenate([p["agent_infos"]["mean"] for p in paths]), g["means"])
    close(np.concatenate([p["actions"] for p in paths]), g["actions"], rtol=1e-12, atol=1e-12)
    close(np.concatenate([p["observations"] for p in paths]), g["observations"], rtol=1e-12, atol=1e-12)
    close(np.concatenate([p["next_observations"] for p in paths]), g["next_observations"], rtol=1e-12,
          atol=1e-12)


def test_philox_known_answers():
    """Random123 known-answer vectors for Philox4x32-10 (kat_vectors)."""
    z = R.philox4x32_10(np.zeros((1, 4), np.uint32), (0, 0))[0]
    assert [int(x) for x in z] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = R.philox4x32_10(np.full((1, 4), 0xFFFFFFFF, np.uint32), (0xFFFFFFFF, 0xFFFFFFFF))[0]
    assert [int(x) for x in f] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    p = R.philox4x32_10(np.array([[0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344]], np.uint32),
                        (0xA4093822, 0x299F31D0))[0]
    assert [int(x) for x in p] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_policy_noise_is_standard_normal():
    z = R.policy_noise(seed=1234, counter=7, B=4096, A=28)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01


# ---- G9: returns / MLP baseline / GAE / whitening (mjrl process_samples, mlp_baseline) ----
def g9_paths(g):
    lens, term = g["lengths"], g["terminated"]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    return [dict(observations=g["observations"][o:o + l], rewards=g["rewards"][o:o + l], terminated=bool(t),
                 actions=np.zeros((l, A))) for o, l, t in zip(offs, lens, term)]


def test_g9_baseline_features_and_predict(golden):
    g = golden("g9_gae.npz")
    layers = R.init_mlp_baseline(S, (128, 128), seed=int(g["baseline_seed"]))
    np.testing.assert_array_equal(layers[0][0].numpy()[:4, :8], g["w0_head"])
    np.testing.assert_array_equal(layers[2][0].numpy(), g["w2"])
    paths = g9_paths(g)
    feat = R.mlp_baseline_features(paths)
    np.testing.assert_array_equal(feat[:, :8], g["features_head"])
    np.testing.assert_array_equal(feat[:, -4:], g["features_time"])
    assert feat[:, 3].max() == 1.0 and feat[:, 3].min() == -1.0  # the clip is exercised
    v = R.mlp_baseline_predict(layers, feat)
    close(v, g["baseline_gae"])


@pytest.mark.parametrize("mode,lam", [("gae", 0.97), ("std", None)])
def test_g9_returns_advantages(golden, mode, lam):
    g = golden("g9_gae.npz")
    paths = g9_paths(g)
    base = g[f"baseline_{mode}"]
    offs = np.concatenate([[0], np.cumsum(g["lengths"])])
    by_id = {id(p): base[offs[i]:offs[i + 1]] for i, p in enumerate(paths)}
    R.compute_returns(paths, float(g["gamma"]))
    R.compute_advantages(paths, lambda p: by_id[id(p)], float(g["gamma"]), lam)
    # fp64 algebra in the reference's order: bit-exact given the same baseline values
    np.testing.assert_array_equal(np.concatenate([p["returns"] for p in paths]), g[f"returns_{mode}"])
    np.testing.assert_array_equal(np.concatenate([p["advantages"] for p in paths]), g[f"adv_{mode}"])
    if mode == "gae":
        adv_w, stats = R.whiten_advantages(paths)
        np.testing.assert_array_equal(adv_w, g["adv_whitened"])
        np.testing.assert_array_equal(np.array(stats), g["base_stats"])


def test_g11_npg_update(golden):
    """Oracle NPG update (VPG, HVP, CG, step, clamp, surr_after) vs the reference's NPG."""
    g = golden("g11_npg.npz")
    shapes = R.policy_param_shapes(226, 28, (32, 32))
    obs, act = g["observations"].astype(np.float64), g["actions"]
    hv = R.npg_hvp(g["params0"], shapes, obs, act, g["hvp_v"], float(g["damping"]))
    np.testing.assert_array_equal(hv, g["hvp"])
    out = R.npg_update(g["params0"], shapes, obs, act, g["advantages"], step=float(g["step"]),
                       damping=float(g["damping"]), cg_iters=int(g["cg_iters"]), min_log_std=float(g["min_log_std"]))
    np.testing.assert_array_equal(out["adv_whitened"], g["adv_whitened"])
    np.testing.assert_array_equal(out["vpg"], g["vpg"])
    np.testing.assert_array_equal(out["npg"], g["npg"])
    np.testing.assert_array_equal(out["params1"], g["params1"])
    assert out["surr_after"] == float(g["surr_after"])


def test_oracle_reset_noise_structure():
    """oracle.deepmimic_ref.add_noise (cKinCharacter::AddNoise, KinCharacter.cpp:340-470) on the
    humanoid3d character: the draw counts per option, the no-noise identity, noise_bef_rot's
    order, the hip / ankle / knee exclusions (their pose parameters untouched by the rotation
    noise), interp scaling of every velocity, normalised quaternions, and EulerToQuaternion's
    known values (zero angles -> identity; a pure x rotation -> its axis-angle quaternion).
    Parity with the C++ core itself is unpinned (no Bullet/Eigen/GL here)."""
    import json
    import math
    from oracle import deepmimic_ref as DR
    from amp_extensions_amd.motion import ReferenceMotion
    z = np.load(ReferenceMotion.DEFAULT_BUNDLE, allow_pickle=False)
    J, bodies, D = DR.load_character(json.loads(str(z["character_json"])))
    M = DR.Motion({"Loop": str(z["loop"]), "Frames": z["frames"].tolist()}, J)
    base = dict(noise_bef_rot=False, noise_min=0, noise_max=0, radian=0, rot_vel_w_pose=False, vel_noise=False,
                interp=1.0, knee_rot=False)
    pose, vel = M.pose(0.41), M.vel(0.41)
    assert DR.noise_draws(J, base) == (0, 0)
    p0, v0 = DR.add_noise(J, pose, vel, base, [], [])
    np.testing.assert_array_equal(p0, pose)
    np.testing.assert_array_equal(v0, vel)
    ra = dict(base, radian=0.3)
    nr, npv = DR.noise_draws(J, ra)
    # root yaw + revolute elbows (7, 13) + spherical chest, neck, shoulders (1, 2, 6, 12) x 3
    assert (nr, npv) == (1 + 2 + 4 * 3, 0)
    assert DR.noise_draws(J, dict(ra, knee_rot=True))[0] == nr + 2
    assert DR.noise_draws(J, dict(ra, vel_noise=True))[0] == nr + 3 + 1 + 4 * 3  # only joint 10's vel
    assert DR.noise_draws(J, dict(base, noise_min=-0.1, noise_max=0.1)) == (0, 2 * D)
    rs = np.random.RandomState(1)
    u = rs.rand(nr)
    p1, v1 = DR.add_noise(J, pose, vel, dict(ra, interp=0.5), u, [])
    for j in (3, 4, 5, 9, 10, 11):   # hips, knees, ankles untouched by the pose rotation noise
        o, s = J[j]["offset"], J[j]["size"]
        np.testing.assert_allclose(p1[o:o + s], pose[o:o + s] / (np.linalg.norm(pose[o:o + s]) if s == 4 else 1.0),
                                   rtol=0, atol=1e-15)
    # the joints' velocities are only interp-scaled; the root's linear and angular velocity are
    # also turned by the root yaw (RotateRoot -> SetRootRotation -> RotateOrigin,
    # KinCharacter.cpp:259-264, 300-337): y components and xz norms kept, the pad slot zeroed
    np.testing.assert_allclose(v1[7:], 0.5 * vel[7:], rtol=0, atol=0)
    for a in (0, 3):
        assert abs(v1[a + 1] - 0.5 * vel[a + 1]) <= 1e-15
        assert abs(math.hypot(v1[a], v1[a + 2]) - 0.5 * math.hypot(vel[a], vel[a + 2])) <= 1e-14
    assert v1[6] == 0.0 and np.abs(v1[[0, 2, 3, 5]] - 0.5 * vel[[0, 2, 3, 5]]).max() > 1e-3
    for j in range(len(J)):
        if J[j]["type"] == 4:
            o = J[j]["offset"]
            assert abs(np.linalg.norm(p1[o:o + 4]) - 1.0) < 1e-14
    assert abs(np.linalg.norm(p1[3:7]) - 1.0) < 1e-14
    np.testing.assert_allclose(DR.euler_to_quat(0.0, 0.0, 0.0), [1, 0, 0, 0], atol=0)
    np.testing.assert_allclose(DR.euler_to_quat(0.4, 0.0, 0.0), [math.cos(0.2), math.sin(0.2), 0, 0], atol=1e-15)
    # noise_bef_rot changes the order of the two perturbations (different results, same draws)
    ra2 = dict(base, radian=0.3, noise_min=-0.05, noise_max=0.05)
    nr2, npv2 = DR.noise_draws(J, ra2)
    ur, up = rs.rand(nr2), rs.rand(npv2)
    a, _ = DR.add_noise(J, pose, vel, ra2, ur, up)
    b, _ = DR.add_noise(J, pose, vel, dict(ra2, noise_bef_rot=True), ur, up)
    assert np.abs(a - b).max() > 1e-6
