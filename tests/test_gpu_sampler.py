"""GPU tests of the drop-in `sample_points` (milo/milo/sampler.py:8-130) against the
REFERENCE's recorded 2-worker run (G8) and the oracle's restatement of get_samples /
sample_points: same seeds -> same trajectories (lengths, terminations, reset poses, member
rotation exact; states, actions and policy means to the ensemble's fp32 tolerance), the
reference's per-worker quota ceil(N/W) with complete trajectories, at 8192 lanes too."""
import math

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
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ens.device.ctx, pw, log_std)
    return amx, ens, ens_w, norms, pw, log_std, pol


def _state_close(got, want, what):
    got, want = np.asarray(got), np.asarray(want)
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-4 * max(1.0, np.abs(want).max()), err_msg=what)


def _compare_paths(paths, ref):
    assert [len(p["rewards"]) for p in paths] == [len(p["rewards"]) for p in ref]
    for i, (p, q) in enumerate(zip(paths, ref)):
        assert p["terminated"] is True and bool(q["terminated"]) is True
        # the reset pose (env.seed_env(12345 + base_seed * i + j) -> np_random.uniform -> row) is exact
        np.testing.assert_array_equal(p["observations"][0], q["observations"][0])
        _state_close(p["observations"], q["observations"], f"path {i} observations")
        _state_close(p["next_observations"], q["next_observations"], f"path {i} next_observations")
        np.testing.assert_allclose(p["agent_infos"]["mean"], q["agent_infos"]["mean"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(p["actions"], q["actions"], rtol=0, atol=2e-4)
        assert p["observations"].dtype == np.float64 and p["actions"].dtype == np.float64
        assert p["agent_infos"]["mean"].dtype == np.float32
        np.testing.assert_array_equal(p["agent_infos"]["log_std"], q["agent_infos"]["log_std"])
        assert len(p["env_infos"]) == len(q["env_infos"]) and all(x == {} for x in p["env_infos"])


def test_sample_points_reproduces_reference_g8(setup, golden):
    """The reference's own 2-worker sample_points run (G8: h64 ensemble, horizon 8, N=24,
    base_seed 100, stub reset core = table row floor(t)) through the GPU drop-in."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    g = golden("g8_sample_points.npz")
    np.testing.assert_array_equal(pw[0][0].numpy()[:4, :8], g["pol_w0"])
    table, _, _ = synthetic_offline(64, 1)
    env = amx.BatchedSimEnv(ens, table, lanes=64, horizon=int(g["horizon"]), record_means=True)
    paths = amx.sample_points(env, pol, num_to_collect=int(g["num_to_collect"]), base_seed=int(g["base_seed"]),
                              num_workers=int(g["num_workers"]))
    np.testing.assert_array_equal([len(p["rewards"]) for p in paths], g["lengths"])
    np.testing.assert_array_equal([p["terminated"] for p in paths], g["terminated"])
    cat = lambda k: np.concatenate([p[k] for p in paths])
    _state_close(cat("observations"), g["observations"], "observations")
    _state_close(cat("next_observations"), g["next_observations"], "next_observations")
    np.testing.assert_allclose(cat("actions"), g["actions"], rtol=0, atol=2e-4)
    np.testing.assert_allclose(np.concatenate([p["agent_infos"]["mean"] for p in paths]), g["means"], rtol=1e-4,
                               atol=1e-5)


@pytest.mark.parametrize("mode,N,horizon,chunk", [("samples", 400, 40, 8), ("samples", 257, 25, 5),
                                                  ("trajectories", 9, 30, 8), ("samples", 900, 30, 4)])
@pytest.mark.parametrize("speculate,graph,pipeline", [(True, True, True), (False, False, True), (True, False, True),
                                                       (True, True, False), (False, False, False)])
def test_sample_points_matches_oracle(setup, mode, N, horizon, chunk, speculate, graph, pipeline):
    """W=2 and W=3 workers vs the oracle's sequential get_samples with the same seeds, on a
    standing reset table (long trajectories: several chunks, mid-chunk ends, refills), with the
    speculative admission (surplus trajectories run and are dropped), the chunk HIP graph and the
    pipelined chunk loop (the host one chunk behind the GPU) on and off: the same paths."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(256, S, 1)
    table[::7, 2] = -2.0  # root below the ground: these reset poses fall at once (length-1 trajectories)
    table[1::3, 2] = -0.3  # these fall after a few steps: short trajectories drive the speculation
    for W in (2, 3):
        env = amx.BatchedSimEnv(ens, table, lanes=512, horizon=horizon, record_means=True)
        paths = amx.sample_points(env, pol, num_to_collect=N, base_seed=7, num_workers=W, mode=mode, chunk=chunk,
                                  speculate=speculate, graph=graph, pipeline=pipeline)
        per = math.ceil(N / W)
        ref = []
        for i in range(W):
            envr = R.SimEnvRef(ens_w, norms, horizon=horizon)
            p, _ = R.get_samples(envr, pw, log_std, per, 12345 + 7 * i, table, mode=mode)
            ref.extend(p)
        _compare_paths(paths, ref)


def test_sample_points_quota_at_8192_lanes(setup):
    """num_to_collect=10000 from an 8192-lane env returns the reference's sample count (>= N,
    each worker stops at its first trajectory that reaches ceil(N/W)), not one trajectory per
    lane; 'trajectories' mode returns exactly W * ceil(N/W) trajectories."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    env = amx.BatchedSimEnv(ens, reset_table(4096, S, 1), lanes=8192, horizon=300, record_means=True)
    for rng in ("reference", "device"):
        paths = amx.sample_points(env, pol, num_to_collect=10000, base_seed=3, num_workers=4, rng=rng)
        n = sum(len(p["rewards"]) for p in paths)
        assert 10000 <= n < 10000 + 4 * 300, n
        # per worker (paths come worker by worker): the quota is met by the last trajectory only
        lens = [len(p["rewards"]) for p in paths]
        q, i, w = 2500, 0, 0
        while i < len(lens):
            tot = 0
            while tot < q:
                tot += lens[i]
                i += 1
            w += 1
        assert w == 4
        assert all(p["terminated"] is True and 1 <= len(p["rewards"]) <= 300 for p in paths)
    paths = amx.sample_points(env, pol, num_to_collect=10, num_workers=4, mode="trajectories")
    assert len(paths) == 4 * 3


def test_sample_points_eval_mode_and_member_rotation(setup):
    """eval_mode: actions are the policy means (gaussian_mlp.py 'evaluation'); trajectory j of
    a worker runs on ensemble member j mod M (sim_env.py:282-283): its first transition equals
    that member's prediction."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    env = amx.BatchedSimEnv(ens, reset_table(256, S, 1), lanes=64, horizon=6, record_means=True)
    paths = amx.sample_points(env, pol, num_to_collect=30, base_seed=2, num_workers=1, eval_mode=True)
    assert len(paths) == 5
    for j, p in enumerate(paths, start=1):
        np.testing.assert_array_equal(p["actions"], p["agent_infos"]["mean"].astype(np.float64))
        o, a = p["observations"][:1], p["actions"][:1]
        pred = R.ensemble_preds(ens_w, norms, torch.from_numpy(o).float(), torch.from_numpy(a).float()).numpy()
        want = o[0] + pred[j % 4, 0].astype(np.float64)
        _state_close(p["next_observations"][0], want, f"trajectory {j}")


def test_sample_points_pipelined_bit_identical(setup):
    """The pipelined chunk loop (chunk i queued before chunk i-1's done flags are read; lanes
    re-admitted one chunk later) returns the serial loop's paths bit for bit: the same
    trajectories in the same order, every array equal."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(256, S, 2)
    table[::5, 2] = -2.0
    table[1::4, 2] = -0.3
    env = amx.BatchedSimEnv(ens, table, lanes=512, horizon=60, record_means=True)
    for W, N, chunk in ((2, 1500, 16), (4, 999, 7)):
        a = amx.sample_points(env, pol, num_to_collect=N, base_seed=11, num_workers=W, chunk=chunk, pipeline=False)
        b = amx.sample_points(env, pol, num_to_collect=N, base_seed=11, num_workers=W, chunk=chunk, pipeline=True)
        assert len(a) == len(b)
        for pa, pb in zip(a, b):
            for k in ("observations", "next_observations", "actions"):
                np.testing.assert_array_equal(pa[k], pb[k])
            np.testing.assert_array_equal(pa["agent_infos"]["mean"], pb["agent_infos"]["mean"])
