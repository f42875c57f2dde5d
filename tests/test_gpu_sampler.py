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
    pol = amx.DevicePolicy(ens.ctx, pw, log_std)
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


def test_forward_blocked_matches_member_rows(setup):
    """DeviceEnsemble.forward_blocked (lanes [g*Bq, (g+1)*Bq) through member g alone) equals
    member g's rows of the all-member forward."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    dev = ens.engine
    rs = np.random.RandomState(5)
    for Bq in (128, 256):
        B = 4 * Bq
        ob = torch.from_numpy(0.5 * rs.randn(B, S)).to(DEV)
        ac = torch.from_numpy(rs.randn(B, A)).to(DEV)
        full = dev.forward_preds(ob, ac, B).clone()
        blk = dev.forward_blocked(ob, ac, Bq).clone()
        assert tuple(blk.shape) == (B, S)
        for g in range(4):
            np.testing.assert_allclose(blk[g * Bq:(g + 1) * Bq].cpu().numpy(),
                                       full[g, g * Bq:(g + 1) * Bq].cpu().numpy(), rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        dev.forward_blocked(ob, ac, 100)


def test_sample_points_member_blocked_matches_all_member_lanes(setup):
    """member_blocked=True (the default: each lane steps through its trajectory's member only,
    the lanes in M blocks of a multiple of 128) against every member on every lane: the same
    trajectories (lengths, terminations, reset poses exact), states / actions / means within the
    ensemble's fp32 tolerance; both against the oracle."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(256, S, 3)
    table[::6, 2] = -2.0
    table[1::4, 2] = -0.3
    env = amx.BatchedSimEnv(ens, table, lanes=512, horizon=40, record_means=True)
    W, N = 3, 700
    a = amx.sample_points(env, pol, num_to_collect=N, base_seed=5, num_workers=W, member_blocked=False)
    b = amx.sample_points(env, pol, num_to_collect=N, base_seed=5, num_workers=W, member_blocked=True)
    _compare_paths(b, a)
    ref = []
    for i in range(W):
        envr = R.SimEnvRef(ens_w, norms, horizon=40)
        p, _ = R.get_samples(envr, pw, log_std, math.ceil(N / W), 12345 + 5 * i, table)
        ref.extend(p)
    _compare_paths(b, ref)


def test_sample_points_member_blocked_fused_assembly_bit_identical(setup):
    """Member-blocked lanes with the policy launch writing x0 and its exponents in the blocked
    layout (amx_policy_act's fused assembly, slot stride Bq) against the separate assembly
    launch: the same paths bit for bit."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(256, S, 4)
    table[::5, 2] = -2.0
    table[1::4, 2] = -0.3
    env = amx.BatchedSimEnv(ens, table, lanes=512, horizon=30, record_means=True)
    kw = dict(num_to_collect=600, base_seed=4, num_workers=3)
    a = amx.sample_points(env, pol, **kw)
    engines = list(env.engine.__dict__["_sampler_engines"].values())
    assert any(e.member_blocks for e in engines)
    before = {id(e): e.fuse_assembly for e in engines}
    for e in engines:
        e.fuse_assembly = not e.fuse_assembly
    try:
        b = amx.sample_points(env, pol, **kw)
    finally:
        for e in engines:
            e.fuse_assembly = before[id(e)]
    assert len(a) == len(b)
    for pa, pb in zip(a, b):
        for k in ("observations", "next_observations", "actions"):
            np.testing.assert_array_equal(pa[k], pb[k])
        np.testing.assert_array_equal(pa["agent_infos"]["mean"], pb["agent_infos"]["mean"])


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


def test_sample_points_custom_time_window_table(setup):
    """reset_args custom_time / time_max (sim_env.py:76-77, 276): every trajectory's reset draws
    t ~ U(0, time_max), not U(0, table rows) -- with time_max 2.5 the rows are floor(t) in
    {0, 1, 2}, row 2 half as likely.  The paths equal the oracle's get_samples over the same
    window (the window was ignored)."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(64, S, 4)
    ra = dict(custom_time=True, time_min=0, time_max=2.5)
    env = amx.BatchedSimEnv(ens, table, lanes=128, horizon=12, record_means=True, reset_args=ra)
    W, N = 2, 150
    paths = amx.sample_points(env, pol, num_to_collect=N, base_seed=5, num_workers=W)
    ref = []
    for i in range(W):
        envr = R.SimEnvRef(ens_w, norms, horizon=12)
        p, _ = R.get_samples(envr, pw, log_std, math.ceil(N / W), 12345 + 5 * i, table, time_max=2.5)
        ref.extend(p)
    _compare_paths(paths, ref)
    firsts = np.stack([p["observations"][0] for p in paths])
    rows = [int(np.flatnonzero((table == f).all(1))[0]) for f in firsts]
    assert set(rows) <= {0, 1, 2} and 2 in rows


class _MjrlFC(torch.nn.Module):
    """mjrl FCNetwork's attribute layout (mjrl/utils/fc_network.py: fc_layers)."""

    def __init__(self, layers):
        super().__init__()
        self.fc_layers = torch.nn.ModuleList(layers)


class _MjrlMLP:
    """The attribute layout of mjrl's MLP policy (gaussian_mlp.py:7-85): model.fc_layers,
    log_std, log_std_val, eps, trainable_params, set_param_values rebinding param.data."""

    def __init__(self, pw, log_std):
        layers = []
        for W, b in pw:
            lin = torch.nn.Linear(W.shape[1], W.shape[0])
            lin.weight.data = W.clone().float()
            lin.bias.data = b.clone().float()
            layers.append(lin)
        self.model = _MjrlFC(layers)
        self.log_std = torch.autograd.Variable(log_std.clone().float(), requires_grad=True)
        self.trainable_params = list(self.model.parameters()) + [self.log_std]
        self.log_std_val = np.float64(self.log_std.data.numpy().ravel())
        self.eps = 0.0

    def get_param_values(self):
        return np.concatenate([p.contiguous().view(-1).data.numpy() for p in self.trainable_params]).copy()

    def set_param_values(self, new_params):
        i = 0
        for p in self.trainable_params:
            n = p.data.numel()
            p.data = torch.from_numpy(new_params[i:i + n].reshape(p.data.shape)).float()
            i += n
        self.log_std_val = np.float64(self.log_std.data.numpy().ravel())


def test_sample_points_takes_mjrl_policy(setup):
    """batch_reinforce.py:88-90 passes its mjrl MLP straight to sample_points: the drop-in wraps
    it once (DevicePolicy.from_mjrl) and reproduces the DevicePolicy run bit for bit; after
    set_param_values (the NPG step, npg_cg.py:186) the next call re-syncs and matches a fresh
    DevicePolicy of the new parameters bit for bit."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    table = reset_table(256, S, 1)
    env = amx.BatchedSimEnv(ens, table, lanes=128, horizon=20, record_means=True)
    mj = _MjrlMLP(pw, log_std)
    for rng in ("reference", "device"):
        # rng='device' draws Philox noise at the engine's running step counter, so its two runs
        # start from two fresh envs (same counter); 'reference' is exact-seeded per trajectory
        env_a = env if rng == "reference" else amx.BatchedSimEnv(ens, table, lanes=128, horizon=20, record_means=True)
        env_b = env if rng == "reference" else amx.BatchedSimEnv(ens, table, lanes=128, horizon=20, record_means=True)
        a = amx.sample_points(env_a, pol, num_to_collect=200, base_seed=9, num_workers=2, rng=rng)
        b = amx.sample_points(env_b, mj, num_to_collect=200, base_seed=9, num_workers=2, rng=rng)
        assert len(a) == len(b)
        for pa, pb in zip(a, b):
            for k in ("observations", "next_observations", "actions"):
                np.testing.assert_array_equal(pa[k], pb[k])
    dp = mj.__dict__["_amx_device_policy"][1]
    new = mj.get_param_values() * 1.01
    mj.set_param_values(new)
    b = amx.sample_points(env, mj, num_to_collect=200, base_seed=9, num_workers=2)
    assert mj.__dict__["_amx_device_policy"][1] is dp  # re-synced in place, not rebuilt
    layers = [(l.weight.data, l.bias.data) for l in mj.model.fc_layers]
    fresh = amx.DevicePolicy(ens.ctx, layers, mj.log_std.data)
    a = amx.sample_points(env, fresh, num_to_collect=200, base_seed=9, num_workers=2)
    assert len(a) == len(b)
    for pa, pb in zip(a, b):
        np.testing.assert_array_equal(pa["actions"], pb["actions"])
        np.testing.assert_array_equal(pa["agent_infos"]["log_std"], pb["agent_infos"]["log_std"])
    with pytest.raises(ValueError):
        amx.sample_points(env, pol, num_to_collect=10, base_seed=2 ** 32, num_workers=2)  # worker 1: seeds >= 2**32


@pytest.mark.parametrize("update", ["optim", "data_add"])
def test_sample_points_sees_in_place_mjrl_updates(setup, update):
    """An in-place update of the mjrl policy's parameters (a torch optimizer step on
    trainable_params, as behavior_cloning.py:125-132, or `p.data.add_`) keeps every tensor's
    storage; the next sample_points must still sample with the new weights: bit-identical to a
    fresh DevicePolicy of them."""
    amx, ens, ens_w, norms, pw, log_std, pol = setup
    from amp_extensions_amd.synthetic import reset_table
    env = amx.BatchedSimEnv(ens, reset_table(256, S, 1), lanes=128, horizon=20, record_means=True)
    mj = _MjrlMLP(pw, log_std)
    amx.sample_points(env, mj, num_to_collect=100, base_seed=3, num_workers=2)
    ptrs = [p.data_ptr() for p in mj.trainable_params]
    if update == "optim":
        opt = torch.optim.SGD(mj.trainable_params, lr=0.05)
        opt.zero_grad()
        loss = sum((p * p).sum() for p in mj.trainable_params)
        loss.backward()
        opt.step()
    else:
        with torch.no_grad():
            for p in mj.trainable_params:
                p.data.add_(0.01)
    assert [p.data_ptr() for p in mj.trainable_params] == ptrs  # storage kept: in place
    b = amx.sample_points(env, mj, num_to_collect=200, base_seed=9, num_workers=2)
    # the mean from the updated model, the noise from log_std_val as mjrl's get_action (its
    # float64 copy is refreshed by set_param_values only, gaussian_mlp.py:53, 91, 102)
    layers = [(l.weight.data, l.bias.data) for l in mj.model.fc_layers]
    fresh = amx.DevicePolicy(ens.ctx, layers, torch.from_numpy(mj.log_std_val))
    a = amx.sample_points(env, fresh, num_to_collect=200, base_seed=9, num_workers=2)
    assert len(a) == len(b)
    for pa, pb in zip(a, b):
        np.testing.assert_array_equal(pa["actions"], pb["actions"])
        np.testing.assert_array_equal(pa["agent_infos"]["log_std"], pb["agent_infos"]["log_std"])
