"""GPU tests of the drop-in surfaces: SimEnv facade against the REFERENCE SimEnv trace and relabel_paths against the oracle's
restatement of the relabel block (mjrl/mjrl/algos/batch_reinforce.py:103-169)."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu

S, A = 226, 28
DEV = "cuda"


def synthetic_offline(n, seed):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


@pytest.fixture(scope="module")
def setup():
    import amp_extensions_amd as amx
    from amp_extensions_amd.ensemble import DynamicsEnsemble
    s, a, s2 = synthetic_offline(2048, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens = DynamicsEnsemble.random_init(S, A, norms, hidden_sizes=(64, 64, 64, 64), num_models=4, base_seed=100)
    ens_w = R.init_ensemble_weights(S, A, [64] * 4, 4, 100)
    return amx, ens, ens_w, norms


def test_simenv_facade_matches_reference_trace(setup, golden):
    """Same seed, same injected actions: the facade reproduces the reference SimEnv's reset
    rows and model rotation exactly, done flags exactly, next states to fp32 tolerance."""
    amx, ens, ens_w, norms = setup
    g = golden("g2_simenv_trace.npz")
    table, _, _ = synthetic_offline(int(g["table_rows"]), int(g["table_seed"]))
    env = amx.SimEnv(ens, horizon=int(g["horizon"]), seed=int(g["env_seed"]), reset_table=table)
    rows = []
    o = env.reset()
    rows.append(int(np.where((table == o).all(1))[0][0]))
    for t in range(g["actions"].shape[0]):
        assert env.reset_counter == g["model_idx"][t]
        ref_ob = g["obs"][t]
        np.testing.assert_allclose(o, ref_ob, rtol=0, atol=1e-4)
        env.set_observation(ref_ob.copy())  # per-step parity (re-anchor on the reference state)
        no, r, d, info = env.step(g["actions"][t].copy())
        assert r == 0 and info == {}
        np.testing.assert_allclose(no, g["next_obs"][t], rtol=0, atol=2e-5 * max(1, np.abs(no).max()))
        assert d == bool(g["done"][t]), t
        assert env.num_steps == g["num_steps"][t]
        if d:
            o = env.reset()
            rows.append(int(np.where((table == o).all(1))[0][0]))
        else:
            o = no
    np.testing.assert_array_equal(rows, g["reset_rows"])


def test_relabel_paths_matches_oracle(setup):
    amx, ens, ens_w, norms = setup
    from amp_extensions_amd.relabel import relabel_paths
    from amp_extensions_amd.synthetic import reset_table
    s, a, _ = synthetic_offline(2048, 0)
    thr = ens.compute_threshold(torch.from_numpy(s).float(), torch.from_numpy(a).float())
    es, _, es2 = synthetic_offline(800, 3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    cost = amx.RBFLinearCost(expert, feature_dim=512, lambda_b=0.0025, seed=100, ctx=ens.ctx)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ens.ctx, pw, log_std)
    env = amx.BatchedSimEnv(ens, reset_table(256, S, 1), lanes=12, horizon=15, max_steps=8, record_means=True)
    paths = amx.sample_points(env, pol, num_to_collect=120, base_seed=1)
    ref_paths = [{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()} for p in paths]
    infos = relabel_paths(paths, cost, ens)
    ref = R.RBFLinearCostRef(expert, feature_dim=512, lambda_b=0.0025, seed=100)
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    ref_infos = R.relabel_mmd(ref_paths, ref, disc_fn, thr)
    np.testing.assert_allclose(infos["mb_mmd"], ref_infos["mb_mmd"], rtol=1e-4)
    got = np.concatenate([p["rewards"] for p in paths])
    want = np.concatenate([p["rewards"] for p in ref_paths])
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
    np.testing.assert_allclose(infos["int"], ref_infos["int"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(infos["ext"], ref_infos["ext"], rtol=1e-4, atol=1e-4 * np.abs(ref_infos["ext"]).max())
    assert infos["ep_len"] == ref_infos["ep_len"]
    np.testing.assert_allclose(infos["bonus_mmd"], ref_infos["bonus_mmd"], rtol=1e-4, atol=1e-7)


def test_relabel_paths_device_rows_match_uploaded_copies(setup, monkeypatch):
    """relabel_paths on sample_points' own paths reads the sampler's device rows (the paths'
    arrays are read-only views of its host copy: no upload); on writable copies of the same
    paths it uploads them.  Same bits either way; a subset of the paths (a contiguous range of
    the views) also takes the device rows."""
    amx, ens, ens_w, norms = setup
    from amp_extensions_amd import relabel as RL
    from amp_extensions_amd.synthetic import reset_table
    s, a, _ = synthetic_offline(2048, 0)
    ens.compute_threshold(torch.from_numpy(s).float(), torch.from_numpy(a).float())
    es, _, es2 = synthetic_offline(800, 3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    cost = amx.RBFLinearCost(expert, feature_dim=512, lambda_b=0.0025, seed=100, ctx=ens.ctx)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ens.ctx, pw, log_std)
    env = amx.BatchedSimEnv(ens, reset_table(256, S, 1), lanes=64, horizon=15, record_means=True)
    paths = amx.sample_points(env, pol, num_to_collect=300, base_seed=2)
    assert not paths[0]["observations"].flags.writeable and not paths[0]["agent_infos"]["log_std"].flags.writeable
    with pytest.raises(ValueError):
        paths[0]["observations"][0, 0] = 1.0
    copies = [{k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()} for p in paths]
    used = []
    real = RL._device_rows

    def spy(ps, key, dev):
        r = real(ps, key, dev)
        used.append(r is not None)
        return r
    monkeypatch.setattr(RL, "_device_rows", spy)
    RL.relabel_paths(paths, cost, ens)
    assert used and all(used)
    used.clear()
    RL.relabel_paths(copies, cost, ens)
    assert used and not any(used)
    np.testing.assert_array_equal(np.concatenate([p["rewards"] for p in paths]),
                                  np.concatenate([p["rewards"] for p in copies]))
    used.clear()
    sub, sub_copies = paths[2:5], copies[2:5]
    RL.relabel_paths(sub, cost, ens)
    assert used and all(used)
    RL.relabel_paths(sub_copies, cost, ens)
    np.testing.assert_array_equal(np.concatenate([p["rewards"] for p in sub]),
                                  np.concatenate([p["rewards"] for p in sub_copies]))
