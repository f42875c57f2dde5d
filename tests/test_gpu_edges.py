"""GPU edge cases and full-size properties of the hot path.

Full size (8192 lanes, the bench shape) cannot be replayed through the per-lane Python
oracle in seconds, so it is checked through size-independent properties: the fp64 state
update is exactly s + Δ_k of the recorded member deltas, termination equals the oracle's
fall check on the recorded states (bit-exact), the RFF column partials equal the fp64 sum of
the recorded φ rows, and the rewards obey the algebra of get_bonus_costs.  Small cases cover
ragged lane counts, a single lane, horizon 1 (every lane resets every step), a 2-member
ensemble, hidden widths that are not multiples of 128, non-finite states, and the C ABI's
argument checks.
"""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def offline(n, seed, S, A):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def build(S, A, hidden, M=4, seed=100):
    import amp_extensions_amd as amx
    s, a, s2 = offline(2048, 0, S, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens_w = R.init_ensemble_weights(S, A, hidden, M, seed)
    ctx = amx.AmxContext(S, A, n_models=M, hidden=hidden[0], n_hidden=len(hidden), feat_dim=512, device=DEV)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms)
    ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    return amx, ctx, ens, ens_w, norms


@pytest.mark.parametrize("S,A", [(197, 36), (226, 28)])
def test_full_size_properties(S, A):
    amx, ctx, ens, ens_w, norms = build(S, A, [512] * 4)
    from amp_extensions_amd import synthetic as syn
    from amp_extensions_amd.policy import init_mlp_policy_params
    cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(4096, S, 3)), feature_dim=512, bw_samples=20000,
                             lambda_b=0.0025, seed=100, ctx=ctx)
    pw, ls = init_mlp_policy_params(S, A)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=3)
    table = syn.reset_table(4096, S, 1)
    table[::5, 2] = -0.9  # root sphere on the ground in every 5th reset pose: exercises resets
    B, K = 8192, 2
    eng = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=cost, seed=11, max_steps=K)
    eng.reset_all()
    mk_before = []
    for t in range(K):
        mk_before.append(eng.model_idx.clone())
        eng.step()
        if t == K - 1:
            preds = ens.workspace(B)["preds"][:, :B].clone()
    eng.relabel()
    torch.cuda.synchronize()
    obs, nxt = eng.obs[:K].cpu().numpy(), eng.next_obs.cpu().numpy()
    done = eng.done.cpu().numpy()
    # (1) fp64 state update of the last step is exactly s + (double)Δ_k
    k = mk_before[-1].cpu().numpy()
    p = preds.cpu().numpy()
    np.testing.assert_array_equal(nxt[K - 1], obs[K - 1] + p[k, np.arange(B)].astype(np.float64))
    # (2) termination bit-exact vs the oracle's fall check on the recorded next states
    env = R.SimEnvRef([None], None)
    for t in range(K):
        for b in range(0, B, 7):
            env.ob = nxt[t, b].copy()
            assert bool(done[t, b]) == env.check_collision(), (t, b)
    assert done.sum() > 0
    # (3) carried / reset lane states for the next step
    rows = eng.reset_rows.cpu().numpy()
    for b in range(0, B, 97):
        exp = table[rows[0, b]] if done[0, b] else nxt[0, b]
        np.testing.assert_array_equal(obs[1, b], exp)
    # (4) fp64 feature sums == sum of the recorded phi rows (valid lanes only)
    phi = eng.phi[:K, :B].double().sum(dim=(0, 1)).cpu().numpy()
    tot = eng.phi_sum.cpu().numpy()
    np.testing.assert_allclose(tot, phi, rtol=1e-10, atol=1e-10)
    # (5) reward algebra: reward = -((1-l) clamp(phi.w) - l * min(d/thr, 1) * c_min)
    w = cost.w.cpu().numpy().astype(np.float64)
    v = np.clip(eng.phi[:K, :B].cpu().numpy().astype(np.float64) @ w, -1, 0)
    dh = np.minimum(eng.disc[:K, :B].cpu().numpy() / np.float32(ens.threshold), 1.0)
    ref = -((1 - 0.0025) * v + 0.0025 * dh)
    np.testing.assert_allclose(eng.rewards[:K, :B].cpu().numpy(), ref, rtol=1e-4, atol=1e-6)
    # (6) disagreement of the last step from the recorded member deltas (fp64 reference)
    pp = p.astype(np.float64)
    dref = np.max([np.linalg.norm(pp[i] - pp[j], axis=1) for i in range(4) for j in range(i + 1, 4)], axis=0)
    np.testing.assert_allclose(eng.disc[K - 1, :B].cpu().numpy(), dref, rtol=1e-5)


@pytest.mark.parametrize("B", [1, 129])
def test_ragged_lane_counts_and_horizon_one(B):
    amx, ctx, ens, ens_w, norms = build(226, 28, [64] * 4)
    table, _, _ = offline(32, 1, 226, 28)
    eng = amx.RolloutEngine(ens, table, lanes=B, term=amx.TerminationConfig(horizon=1), seed=2, max_steps=4)
    eng.reset_all()
    rs = np.random.RandomState(0)
    for t in range(4):
        eng.step(actions=torch.from_numpy(rs.randn(B, 28)).to(DEV))
    torch.cuda.synchronize()
    # horizon 1: every lane is done every step and resets into the next ensemble member
    assert eng.done.cpu().numpy().all()
    np.testing.assert_array_equal(eng.reset_count.cpu().numpy(), np.full(B, 5))
    np.testing.assert_array_equal(eng.model_idx.cpu().numpy(), np.full(B, 5 % 4))
    rows = eng.reset_rows.cpu().numpy()
    for t in range(4):
        np.testing.assert_array_equal(rows[t], R.reset_rows(2, np.arange(B), np.full(B, t + 2), 32))
        np.testing.assert_array_equal(eng.obs[t + 1].cpu().numpy(), table[rows[t]])


def test_two_member_ensemble_and_odd_hidden_width():
    """M = 2 (generic disagreement path) with hidden width 100 (zero-padded to 128)."""
    amx, ctx, ens, ens_w, norms = build(226, 28, [100] * 3, M=2)
    rs = np.random.RandomState(4)
    B = 200
    s = torch.from_numpy(rs.randn(B, 226) * 0.5).float()
    a = torch.from_numpy(rs.randn(B, 28)).float()
    preds = ens.forward_preds(s.to(DEV), a.to(DEV), B)[:, :B].cpu().numpy()
    ref = R.ensemble_preds(ens_w, norms, s, a).numpy()
    assert np.abs(preds - ref).max() <= 2e-5 * max(1, np.abs(ref).max())
    d = ens.get_action_discrepancy(s, a).cpu().numpy()
    np.testing.assert_allclose(d, R.compute_discrepancy(ens_w, norms, s, a).numpy(), rtol=1e-4, atol=1e-7)


def test_nonfinite_state_flagged_not_terminated():
    amx, ctx, ens, ens_w, norms = build(226, 28, [64] * 4)
    table, _, _ = offline(16, 1, 226, 28)
    table[:, 150] = np.nan  # a velocity entry: no fall body reads it
    for b in R.FALL_BODIES:
        table[:, 9 * b + 2] = 1.0
    eng = amx.RolloutEngine(ens, table, lanes=8, seed=1, max_steps=1)
    eng.reset_all()
    eng.step(actions=torch.zeros(8, 28, dtype=torch.float64, device=DEV))
    torch.cuda.synchronize()
    assert eng.nonfinite[0].cpu().numpy().all()
    assert not eng.done[0].cpu().numpy().any()  # the reference has no NaN guard (sim_env.py:164-173)


def test_abi_rejects_bad_arguments():
    amx, ctx, ens, ens_w, norms = build(226, 28, [64] * 4)
    from amp_extensions_amd import _native as N
    lib, s = ctx.lib, ctx.stream
    buf = torch.zeros(4, 128, ctx.ldk + 4, dtype=torch.float32, device=DEV)
    W = ens.W[0]
    # rows not a multiple of 128
    rc = lib.amx_gemm_bias_act(ctx.h, 4, 100, 128, ctx.k0_pad, buf.data_ptr(), ctx.ldk, 0, W.data_ptr(),
                               ctx.k0_pad, 0, ens.b[0].data_ptr(), 0, buf.data_ptr(), ctx.ldk, 0, 0, 1, s)
    assert rc == -1 and b"multiple of 128" in lib.amx_last_error()
    # misaligned operand
    rc = lib.amx_gemm_bias_act(ctx.h, 1, 128, 128, ctx.k0_pad, buf.data_ptr() + 4, ctx.ldk, 0, W.data_ptr(),
                               ctx.k0_pad, 0, ens.b[0].data_ptr(), 0, buf.data_ptr(), ctx.ldk, 0, 0, 1, s)
    assert rc == -1 and b"aligned" in lib.amx_last_error()
    # output slice past the row
    rc = lib.amx_gemm_bias_act(ctx.h, 1, 128, 128, ctx.k0_pad, buf.data_ptr(), ctx.ldk, 0, W.data_ptr(),
                               ctx.k0_pad, 0, ens.b[0].data_ptr(), 0, buf.data_ptr(), ctx.ldk, 0, ctx.ldk - 64, 1, s)
    assert rc == -1
    # amx_step before any termination config, then with aliasing state buffers
    ob = torch.zeros(1, 226, dtype=torch.float64, device=DEV)
    i32 = torch.zeros(1, dtype=torch.int32, device=DEV)
    u8 = torch.zeros(1, dtype=torch.uint8, device=DEV)
    rc = lib.amx_step(ctx.h, buf.data_ptr(), 226, 0, i32.data_ptr(), ob.data_ptr(), buf.data_ptr(), i32.data_ptr(),
                      u8.data_ptr(), None, None, 0, None, 1, s)
    assert rc == -1 and b"termination" in lib.amx_last_error()
    ctx.set_termination(amx.TerminationConfig())
    i32 = torch.zeros(1, dtype=torch.int32, device=DEV)
    u8 = torch.zeros(1, dtype=torch.uint8, device=DEV)
    rc = lib.amx_step(ctx.h, buf.data_ptr(), 226, 0, i32.data_ptr(), ob.data_ptr(), ob.data_ptr(), i32.data_ptr(),
                      u8.data_ptr(), None, None, 0, None, 1, s)
    assert rc == -1 and b"alias" in lib.amx_last_error()
    with pytest.raises(ValueError):
        ens.forward_preds(torch.zeros(4, 227, dtype=torch.float64, device=DEV),
                          torch.zeros(4, 28, dtype=torch.float64, device=DEV))


def test_gail_rollout_rewards_match_oracle():
    amx, ctx, ens, ens_w, norms = build(226, 28, [64] * 4)
    es, _, es2 = offline(512, 3, 226, 28)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], 1)
    gc = amx.GAILCost(expert, hidden_dims=(1024, 512), lambda_b=0.0025, seed=100, ctx=ctx)
    wts = R.init_disc_weights(452, (1024, 512), 1, 100)
    table, _, _ = offline(64, 1, 226, 28)
    B, K = 200, 3
    eng = amx.RolloutEngine(ens, table, lanes=B, cost=gc, seed=4, max_steps=K)
    eng.reset_all()
    rs = np.random.RandomState(1)
    acts = rs.randn(K, B, 28)
    for t in range(K):
        eng.step(actions=torch.from_numpy(acts[t]).to(DEV))
    eng.relabel()
    torch.cuda.synchronize()
    obs = eng.obs[:K].cpu().numpy().reshape(-1, 226)
    nxt = eng.next_obs.cpu().numpy().reshape(-1, 226)
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    cost, _ = R.gail_bonus_costs(wts, torch.from_numpy(obs).float(), torch.from_numpy(acts.reshape(-1, 28)).float(),
                                 torch.from_numpy(nxt).float(), disc_fn, 0.0025)
    ref = -cost.numpy()[:, 0]
    got = eng.rewards[:K, :B].cpu().numpy().reshape(-1)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


@pytest.mark.parametrize("S,A,hidden", [(197, 36, [512] * 4), (100, 20, [256] * 3), (300, 40, [128] * 2)])
def test_bf16x6_ensemble_matches_oracle_and_f32(S, A, hidden):
    """The bf16x6 GEMM path (3-limb split, 6 bf16 MFMA products) across output-tile shapes:
    S=197 -> the 128x224 output tile, S=100 -> 128, S=300 -> 384 (three 128 tiles).  Same
    tolerance as the f32 path (2e-5 of max(1, |ref|)), and within 1e-6 of the f32 path."""
    import amp_extensions_amd as amx
    s, a, s2 = offline(2048, 0, S, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens_w = R.init_ensemble_weights(S, A, hidden, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=hidden[0], n_hidden=len(hidden), feat_dim=512, device=DEV)
    e6 = amx.DeviceEnsemble(ctx, ens_w, norms, gemm="bf16x6")
    e32 = amx.DeviceEnsemble(ctx, ens_w, norms, gemm="f32")
    B = 640
    ob = torch.from_numpy(s[:B]).to(DEV)
    ac = torch.from_numpy(a[:B]).to(DEV)
    p6 = e6.forward_preds(ob, ac, B)[:, :B].cpu().numpy().astype(np.float64)
    p32 = e32.forward_preds(ob, ac, B)[:, :B].cpu().numpy().astype(np.float64)
    ref = R.ensemble_preds(ens_w, norms, torch.from_numpy(s[:B]).float(), torch.from_numpy(a[:B]).float()).numpy()
    scale = max(1.0, np.abs(ref).max())
    assert np.abs(p6 - ref).max() / scale <= 2e-5
    assert np.abs(p32 - ref).max() / scale <= 2e-5
    assert np.abs(p6 - p32).max() / scale <= 1e-6


def test_bf16x6_split_is_exact_and_abi_checks():
    """amx_split_bf16x3: limb0 + limb1 + limb2 == the fp32 weight exactly (normal numbers),
    in the K-tiled [row][K/16][3][16] image; bad shapes are rejected."""
    import amp_extensions_amd as amx
    from amp_extensions_amd import _native as N
    ctx = amx.AmxContext(226, 28, n_models=4, hidden=128, n_hidden=2, device=DEV)
    rs = np.random.RandomState(5)
    W = (rs.randn(2, 128, 64) * np.exp(rs.uniform(-20, 20, (2, 128, 64)))).astype(np.float32)
    Wd = torch.from_numpy(W).to(DEV)
    W3 = torch.empty(2, 128, 3 * 64, dtype=torch.int16, device=DEV)
    N.check(ctx.lib.amx_split_bf16x3(ctx.h, 2, 128, 64, Wd.data_ptr(), 64, 128 * 64, W3.data_ptr(), 128 * 192,
                                     ctx.stream))
    torch.cuda.synchronize()
    bits = W3.cpu().numpy().astype(np.uint16).reshape(2, 128, 4, 3, 16).astype(np.uint32) << 16
    limbs = bits.view(np.float32).astype(np.float64)          # [g][r][kt][limb][16]
    total = limbs.sum(axis=3).reshape(2, 128, 64)
    np.testing.assert_array_equal(total, W.astype(np.float64))
    assert (np.abs(limbs[..., 1, :]) <= np.abs(limbs[..., 0, :]) * 2.0 ** -8).all()
    lib, s = ctx.lib, ctx.stream
    buf = torch.zeros(1, 128, 64, dtype=torch.float32, device=DEV)
    rc = lib.amx_split_bf16x3(ctx.h, 1, 128, 40, Wd.data_ptr(), 64, 0, W3.data_ptr(), 128 * 192, s)
    assert rc == -1 and b"multiple of 16" in lib.amx_last_error()
    rc = lib.amx_gemm_bias_act_x6(ctx.h, 1, 100, 128, 64, buf.data_ptr(), 64, 0, W3.data_ptr(), 128 * 192,
                                  buf.data_ptr(), 0, buf.data_ptr(), 128, 0, 0, 1, s)
    assert rc == -1 and b"multiple of 128" in lib.amx_last_error()
