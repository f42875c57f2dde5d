"""GPU parity of the returns / MLP-baseline / GAE kernels (amx_value_features, amx_value_head,
amx_gae, amx_adv_whiten) against the reference's outputs (G9, mjrl process_samples /
MLPBaseline / process_paths run through the reference code) and the CPU oracle.

Tolerances: features are fp64 math rounded to f32 -> bit-exact; baseline values are an f32
MLP on MFMA vs torch-CPU (different summation order) -> rel 2e-5; returns are independent
of the baseline -> bit-exact; advantages are bit-exact given the device baseline values and
within 1e-5 abs of the reference's (the baseline difference propagates linearly); whitening
uses a different (fixed) reduction order than numpy's pairwise sum -> rel 1e-12.
"""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
S, A = 226, 28


def g9_paths(g):
    lens, term = g["lengths"], g["terminated"]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    return [dict(observations=g["observations"][o:o + l].copy(), rewards=g["rewards"][o:o + l].copy(),
                 terminated=bool(t)) for o, l, t in zip(offs, lens, term)]


@pytest.fixture(scope="module")
def setup():
    import amp_extensions_amd as amx
    ctx = amx.AmxContext(S, A, n_models=4, hidden=64, n_hidden=4, feat_dim=128, device=DEV)
    return amx, ctx


@pytest.mark.parametrize("mode,lam", [("gae", 0.97), ("std", None), ("gae_lambda_out_of_range", 1.5)])
def test_process_samples_vs_reference(golden, setup, mode, lam):
    amx, ctx = setup
    g = golden("g9_gae.npz")
    gamma = float(g["gamma"])
    layers = R.init_mlp_baseline(S, (128, 128), seed=int(g["baseline_seed"]))
    bl = amx.DeviceMLPBaseline(ctx, layers)
    paths = g9_paths(g)
    ret, adv, v = amx.process_samples(paths, bl, gamma, lam)
    torch.cuda.synchronize()
    ref_mode = "gae" if mode == "gae" else "std"  # lambda > 1 selects the standard mode
    # features (fp64 -> f32) bit-exact vs the reference's _features
    n = int(g["lengths"].sum())
    ws = bl.workspace(n)[:n].cpu().numpy()
    np.testing.assert_array_equal(ws[:, :8], g["features_head"])
    np.testing.assert_array_equal(ws[:, S:S + 4], g["features_time"])
    assert not ws[:, S + 4:bl.kf].any()
    vd = np.concatenate([p["baseline"] for p in paths])
    assert vd.dtype == np.float32
    np.testing.assert_allclose(vd, g[f"baseline_{ref_mode}"], rtol=2e-5, atol=1e-6)
    # returns do not depend on the baseline: bit-exact vs the reference
    np.testing.assert_array_equal(np.concatenate([p["returns"] for p in paths]), g[f"returns_{ref_mode}"])
    # advantages: bit-exact vs the oracle fed the device baseline values, close to the reference
    opaths = g9_paths(g)
    offs = np.concatenate([[0], np.cumsum(g["lengths"])])
    by_id = {id(p): vd[offs[i]:offs[i + 1]] for i, p in enumerate(opaths)}
    R.compute_returns(opaths, gamma)
    R.compute_advantages(opaths, lambda p: by_id[id(p)], gamma, lam)
    adv_d = np.concatenate([p["advantages"] for p in paths])
    np.testing.assert_array_equal(adv_d, np.concatenate([p["advantages"] for p in opaths]))
    np.testing.assert_allclose(adv_d, g[f"adv_{ref_mode}"], rtol=0, atol=1e-5)


def test_whitening_vs_reference(golden, setup):
    amx, ctx = setup
    from amp_extensions_amd.gae import whiten_grid
    g = golden("g9_gae.npz")
    adv_ref = torch.from_numpy(g["adv_gae"]).to(DEV)
    n = adv_ref.numel()
    out, stats = whiten_grid(ctx, n, 1, adv_ref.clone(), 1, eps=1e-6, out=torch.empty_like(adv_ref))
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), g["adv_whitened"], rtol=1e-12, atol=1e-13)
    st = stats.cpu().numpy()
    np.testing.assert_allclose(st, [g["adv_gae"].mean(), g["adv_gae"].std()], rtol=1e-13)
    # ragged grid view of the same rows (one lane per path): same values up to the order
    # of the (fixed, but grid-dependent) reduction
    lens = torch.from_numpy(g["lengths"].astype(np.int32)).to(DEV)
    base = torch.from_numpy(np.concatenate([[0], np.cumsum(g["lengths"])[:-1]]).astype(np.int64)).to(DEV)
    out2, _ = whiten_grid(ctx, int(g["lengths"].max()), len(g["lengths"]), adv_ref.clone(), 1, eps=1e-6,
                          out=torch.empty_like(adv_ref), lengths=lens, base=base)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out2.cpu().numpy(), out.cpu().numpy(), rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("B,K,horizon", [(1024, 6, 4), (8192, 5, 3)])
def test_engine_advantages_vs_oracle(setup, B, K, horizon):
    """Lane-buffer layout: trajectories end at done flags, cross rollout boundaries (slot 0
    continues a trajectory: t0 > 0) and are cut at the end of the buffer (bootstrapped)."""
    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    from amp_extensions_amd.ensemble import init_ensemble_weights
    from amp_extensions_amd.policy import init_mlp_policy_params
    S2, A2 = 197, 36
    s, a, s2 = syn.offline(2048, S2, A2, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ctx2 = amx.AmxContext(S2, A2, 4, 128, 2, 128, device=DEV)
    ens = amx.DeviceEnsemble(ctx2, init_ensemble_weights(S2, A2, [128] * 2, 4, 100), norms)
    pw, ls = init_mlp_policy_params(S2, A2)
    pol = amx.DevicePolicy(ctx2, pw, ls, seed=5)
    eng = amx.RolloutEngine(ens, syn.reset_table(4096, S2, 1), lanes=B, term=amx.TerminationConfig(horizon=horizon),
                            policy=pol, seed=3, max_steps=K)
    eng.reset_all()
    eng.rollout(K)
    eng.rollout(K)  # second rollout: lanes start mid-trajectory
    eng.rewards.normal_(std=0.3)
    layers = R.init_mlp_baseline(S2, (128, 64), seed=7)  # 64 wide: exercises the zero padding
    bl = amx.DeviceMLPBaseline(ctx2, layers)
    out = eng.advantages(bl, gamma=0.995, gae_lambda=0.97, whiten=True)
    torch.cuda.synchronize()
    obs = eng.obs[:K].cpu().numpy()
    done = eng.done.cpu().numpy()
    rew = eng.rewards[:, :B].cpu().numpy()
    steps0 = eng.steps0.cpu().numpy()
    assert steps0.max() > 0 and done.sum() > 0
    v = out["values"].cpu().numpy()
    ret, adv = out["returns"].cpu().numpy(), out["advantages"].cpu().numpy()
    paths, rows = R.lanes_to_paths(done, rew, obs, steps0)
    sel = range(0, len(paths), max(1, len(paths) // 600))  # bounded CPU work
    sub = [paths[i] for i in sel]
    feat = R.mlp_baseline_features(sub)
    v_cpu = R.mlp_baseline_predict(layers, feat)
    vd = np.concatenate([v[rows[i][0], rows[i][1]] for i in sel])
    np.testing.assert_allclose(vd, v_cpu, rtol=2e-5, atol=1e-6)
    for i in sel:
        ts, b = rows[i]
        paths[i]["baseline_d"] = v[ts, b]
    R.compute_returns(sub, 0.995)
    R.compute_advantages(sub, lambda p: p["baseline_d"], 0.995, 0.97)
    for j, i in enumerate(sel):
        ts, b = rows[i]
        np.testing.assert_array_equal(ret[ts, b], sub[j]["returns"])
        np.testing.assert_array_equal(adv[ts, b], sub[j]["advantages"])
    aw = out["advantages_whitened"].cpu().numpy()
    exp = (adv - adv.mean()) / (adv.std() + 1e-6)
    np.testing.assert_allclose(aw, exp, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("n", [1, 4095, 4097, 40960, 5_000_003])
def test_whitening_sizes(setup, n):
    """amx_adv_whiten over the chip (per-block count / sum / M2 combined in block order): sizes
    around its 4096-element chunk and past AMX_WHITEN_MAXB x 4096 elements (the chunk grows), in
    place (out aliases adv), against numpy's mean / population std at 1e-12; deterministic."""
    amx, ctx = setup
    from amp_extensions_amd.gae import whiten_grid
    x = np.random.RandomState(n % 1000).randn(n) * 3.0 + 0.7
    d = torch.from_numpy(x).to(DEV)
    out, stats = whiten_grid(ctx, n, 1, d.clone(), 1, eps=1e-6)  # in place
    out2, _ = whiten_grid(ctx, n, 1, d.clone(), 1, eps=1e-6, out=torch.empty_like(d))
    torch.cuda.synchronize()
    ref = (x - x.mean()) / (x.std() + 1e-6)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(stats.cpu().numpy(), [x.mean(), x.std()], rtol=1e-12, atol=1e-14)
    assert torch.equal(out, out2)
